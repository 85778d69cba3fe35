"""Host-batch stress (diagnostic, GPU box): the host-memory entry points
(enet_rc_decompress_batch_host, enet_rc_compress_batch_host) called back to
back on a few precomputed batches, each call into freshly allocated caller
buffers (as an application's would be), every result checked against the
oracle's.  Stops at the first failed call or wrong result and prints it.
usage: python tools/hoststress.py SECONDS [OUT.json]
(ENET_RC_DEBUG=1 adds the failing call site in rc_host.c to stderr;
ENET_RC_NO_HOST_PIN=1 runs the same calls with caller memory never
page-locked -- the A/B this tool exists for, DESIGN.md §2a.
HOSTSTRESS_MMAP=1: each call's output buffer is a fresh anonymous mapping
the process has never touched, as a large new allocation from the C library
often is.)"""
import mmap
import ctypes as C
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from enet_amd import RangeCoder, synth  # noqa: E402
from oracle.pyoracle import compress_batch, fnv_digest  # noqa: E402

limit = float(sys.argv[1])
out_path = sys.argv[2] if len(sys.argv) > 2 else None
P = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
torch.cuda.init()
rc = RangeCoder()
batches = []
for seed, n, game in ((11, 34257, 0), (12, 52000, 0), (13, 23000, 0), (14, 40000, 1)):
    d, o, l = synth.gamestate_batch(n, 1200, seed=seed) if game else synth.mixed_batch(n, lo=1, hi=1400, seed=seed)
    want, wo, wcap, wl = compress_batch(d, o, l, "port")
    # the compressed side in gapped slots (2 len + 64 + 5 apart, as tools/soak.py)
    co = np.zeros(n, np.uint64)
    co[1:] = np.cumsum(2 * l[:-1].astype(np.uint64) + 64 + 5)
    cb0 = np.zeros(int(co[-1]) + int(2 * l[-1]) + 128, np.uint8)
    for t in range(n):
        cb0[int(co[t]): int(co[t]) + int(wl[t])] = want[int(wo[t]): int(wo[t]) + int(wl[t])]
    batches.append((d, o.astype(np.uint64), l.astype(np.uint32), want, wo, wl.astype(np.uint32), co, cb0,
                    f"seed {seed} n {n} game {game}"))
print(f"{len(batches)} batches ready", flush=True)
stats = {"calls": 0, "packets": 0, "seconds": 0.0, "error": None}
t0 = time.time()
last = t0
k = 0
while time.time() - t0 < limit:
    d, o, l, want, wo, wl, co, cb0, name = batches[k % len(batches)]
    k += 1
    n = len(l)
    # decompress from gapped host slots (a fresh copy of the oracle's streams in them)
    # into a fresh back-to-back buffer
    cb = cb0.copy()
    if os.environ.get("HOSTSTRESS_MMAP") == "1":
        mo = mmap.mmap(-1, d.size + 64)
        hout = np.frombuffer(mo, dtype=np.uint8)
    else:
        hout = np.zeros(d.size + 64, np.uint8)
    hl = np.zeros(n, np.uint32)
    r = rc.lib.enet_rc_decompress_batch_host(rc.ctx, P(cb), P(co), P(wl), n, P(hout), P(o), P(l), P(hl))
    stats["calls"] += 1
    if r != 0 or not (np.array_equal(hl, l) and np.array_equal(hout[: d.size], d)):
        stats["error"] = {"call": "decompress", "rc": int(r), "batch": name, "at_call": stats["calls"],
                          "paths": int(rc.lib.enet_rc_last_host_paths(rc.ctx)),
                          "split": int(rc.lib.enet_rc_last_split(rc.ctx))}
        break
    # compress into fresh gapped host slots
    if os.environ.get("HOSTSTRESS_MMAP") == "1":
        mc = mmap.mmap(-1, int(co[-1]) + int(2 * l[-1]) + 128)
        hcb = np.frombuffer(mc, dtype=np.uint8)
    else:
        hcb = np.zeros(int(co[-1]) + int(2 * l[-1]) + 128, np.uint8)
    hcl = np.zeros(n, np.uint32)
    hcap = (2 * l + 64).astype(np.uint32)
    r = rc.lib.enet_rc_compress_batch_host(rc.ctx, P(d), P(o), P(l), n, P(hcb), P(co), P(hcap), P(hcl))
    stats["calls"] += 1
    if r != 0 or not (np.array_equal(hcl, wl) and fnv_digest(hcb, co, hcl) == fnv_digest(want, wo, wl)):
        stats["error"] = {"call": "compress", "rc": int(r), "batch": name, "at_call": stats["calls"],
                          "paths": int(rc.lib.enet_rc_last_host_paths(rc.ctx)),
                          "split": int(rc.lib.enet_rc_last_split(rc.ctx))}
        break
    stats["packets"] += 2 * n
    if time.time() - last > 30:
        last = time.time()
        print(f"t {last - t0:.0f}s calls {stats['calls']}", flush=True)
stats["seconds"] = round(time.time() - t0, 1)
print(json.dumps(stats), flush=True)
if out_path:
    json.dump(stats, open(out_path, "w"), indent=1)
if stats["error"]:
    sys.exit(3)
rc.close()
