import os, sys, time, ctypes as C
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
os.environ["ENET_RC_HOST_PROFILE"] = "1"
import numpy as np, torch
from enet_amd import RangeCoder, synth, get_lib
lib = get_lib(); rc = RangeCoder()
d, o, l = synth.random_batch(65536, 1200)
n = len(l); cap = (2 * l.astype(np.int64) + 64).astype(np.uint32)
coff = np.zeros(n, np.uint64); coff[1:] = np.cumsum(cap[:-1], dtype=np.uint64)
cout = np.zeros(int(coff[-1] + cap[-1]), np.uint8); clen = np.zeros(n, np.uint32)
dout = np.zeros_like(d); dlen = np.zeros(n, np.uint32); lcap = l.astype(np.uint32)
p = lambda a: a.ctypes.data_as(C.c_void_p)
for _ in range(3):
    t0 = time.perf_counter()
    lib.enet_rc_compress_batch_host(rc.ctx, p(d), p(o), p(lcap), n, p(cout), p(coff), p(cap), p(clen))
    t1 = time.perf_counter()
    lib.enet_rc_decompress_batch_host(rc.ctx, p(cout), p(coff), p(clen), n, p(dout), p(o), p(lcap), p(dlen))
    t2 = time.perf_counter()
    print(f"compress {1e3*(t1-t0):.2f} ms decompress {1e3*(t2-t1):.2f} ms ok={np.array_equal(dout,d)}", flush=True)
