"""Host batches in k pieces (k = 0: as ENET_RC_HOST_SPLIT says) (rc_host.c run_host_split, ENET_RC_HOST_SPLIT=k):
the PCIe-inclusive round trip of bench.py's pcie leg for each k, interleaved
in one process, best of R per k.  usage: python tools/split_ab.py [ks] [rounds] [workload]"""
import os
import sys
import time
import ctypes as C

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from enet_amd import RangeCoder, get_lib  # noqa: E402
import bench  # noqa: E402

ks = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "1,2,3,4").split(",")]
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
wl = sys.argv[3] if len(sys.argv) > 3 else "c2"
pinned = os.environ.get("SPLIT_AB_PINNED") == "1"
lib = get_lib()
coders = {}
env_k = os.environ.get("ENET_RC_HOST_SPLIT")
for k in ks:
    if k:                           # (0: the environment's setting)
        os.environ["ENET_RC_HOST_SPLIT"] = str(k)
    coders[k] = RangeCoder()
if env_k is None:
    os.environ.pop("ENET_RC_HOST_SPLIT", None)
else:
    os.environ["ENET_RC_HOST_SPLIT"] = env_k
d, o, l = bench.make_batch(wl, 1048576 if wl == "c4" else 65536, 1200, 0)
n = len(l)
cap = (2 * l.astype(np.int64) + 64).astype(np.uint32)
coff = np.zeros(n, np.uint64)
coff[1:] = np.cumsum(cap[:-1], dtype=np.uint64)
lcap = l.astype(np.uint32)
p = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
alloc = (lambda k: torch.zeros(k, dtype=torch.uint8).pin_memory().numpy()) if pinned else \
    (lambda k: np.zeros(k, np.uint8))
src = alloc(d.size)
src[:] = d
cout = alloc(int(coff[-1] + cap[-1]))
clen = np.zeros(n, np.uint32)
dout = alloc(d.size)
dlen = np.zeros(n, np.uint32)
nb = float(l.sum(dtype=np.uint64))
best = {k: [1e9, 1e9] for k in ks}
times = {k: [] for k in ks}
for r in range(rounds):
    for k in ks:
        c = coders[k]
        dout[:] = 0
        t0 = time.perf_counter()
        rc = lib.enet_rc_compress_batch_host(c.ctx, p(src), p(o), p(lcap), n, p(cout), p(coff), p(cap), p(clen))
        t1 = time.perf_counter()
        rc |= lib.enet_rc_decompress_batch_host(c.ctx, p(cout), p(coff), p(clen), n, p(dout), p(o), p(lcap), p(dlen))
        t2 = time.perf_counter()
        ok = rc == 0 and np.array_equal(dout, src) and np.array_equal(dlen, lcap)
        times[k].append((t1 - t0, t2 - t1))
        best[k][0] = min(best[k][0], t1 - t0)
        best[k][1] = min(best[k][1], t2 - t1)
        print(f"r{r} k={k} split={lib.enet_rc_last_split(c.ctx)} compress {1e3 * (t1 - t0):.3f} ms "
              f"decompress {1e3 * (t2 - t1):.3f} ms ok={ok}", flush=True)
        assert ok
for k in ks:
    tc = sorted(t[0] for t in times[k][1:])
    td = sorted(t[1] for t in times[k][1:])
    if tc:
        print(f"k={k} median after the first: compress {1e3 * tc[len(tc) // 2]:.3f} ms decompress "
              f"{1e3 * td[len(td) // 2]:.3f} ms", flush=True)
    bc, bd = best[k]
    print(f"k={k} {wl} round trip {nb / (bc + bd) / 2**30:.3f} GiB/s compress {nb / bc / 2**30:.2f} "
          f"decompress {nb / bd / 2**30:.2f} ({1e3 * bc:.3f} + {1e3 * bd:.3f} ms)", flush=True)
