"""Round trips of a stream of C2 batches: sequential (compress, then
decompress, one stream -- bench.py's step) against pipelined (batch k + 1's
compress on a second context and stream while batch k decompresses; two
compressed buffers).  Prints ms per round trip for both and checks every
output.  usage: python tools/overlap.py [steps] [kind] [mode]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from enet_amd import RangeCoder  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
kind = sys.argv[2] if len(sys.argv) > 2 else "c2"
dev = torch.device("cuda", 0)
d, o, l = bench.make_batch(kind, 65536, 1200, 0)
n = len(l)
max_len = int(l.max())
din = torch.from_numpy(d).to(dev)
doff = torch.from_numpy(o.astype(np.int64)).to(dev)
dlen = torch.from_numpy(l.astype(np.int32)).to(dev)
cap = (2 * dlen.to(torch.int64) + 64).to(torch.int32)
coff = torch.zeros(n, dtype=torch.int64, device=dev)
coff[1:] = torch.cumsum(cap[:-1].to(torch.int64), 0)
tot = int(coff[-1] + cap[-1])
cout = [torch.empty(tot, dtype=torch.uint8, device=dev) for _ in range(2)]
clen = [torch.zeros(n, dtype=torch.int32, device=dev) for _ in range(2)]
dout = torch.empty_like(din)
dl = torch.zeros(n, dtype=torch.int32, device=dev)
enc, dec = RangeCoder(), RangeCoder()
se, sd = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
enc.compress_batch(din, doff, dlen, cout[0], coff, cap, clen[0], max_len=max_len, stream=se)
torch.cuda.synchronize()
dml = int(clen[0].max().item())
GIB = 1 << 30
in_bytes = int(l.sum(dtype=np.uint64))


def check():
    torch.cuda.synchronize()
    ok = bool(torch.equal(dl, dlen)) and bool(torch.equal(dout, din))
    dl.zero_()
    dout.zero_()
    return ok


def sequential(k):
    for i in range(k):
        enc.compress_batch(din, doff, dlen, cout[0], coff, cap, clen[0], max_len=max_len, stream=se)
        dec.decompress_batch(cout[0], coff, clen[0], dout, doff, dlen, dl, max_len=dml, stream=se)


def pipelined(k):
    # compress k on se into buffer k % 2; decompress k on sd after it; compress
    # k + 2 reuses the buffer after decompress k
    ce = [torch.cuda.Event() for _ in range(k)]
    de = [torch.cuda.Event() for _ in range(k)]
    for i in range(k):
        if i >= 2:
            se.wait_event(de[i - 2])
        enc.compress_batch(din, doff, dlen, cout[i % 2], coff, cap, clen[i % 2], max_len=max_len, stream=se)
        ce[i].record(se)
        sd.wait_event(ce[i])
        dec.decompress_batch(cout[i % 2], coff, clen[i % 2], dout, doff, dlen, dl, max_len=dml, stream=sd)
        de[i].record(sd)


def timed(fn):
    fn(3)
    ok = check()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn(steps)
    torch.cuda.synchronize()
    t = (time.perf_counter() - t0) / steps
    ok = check() and ok
    return t, ok


modes = (("sequential", sequential), ("pipelined", pipelined))
if os.environ.get("OV_PROBE"):
    # which second stream lands on another hardware queue
    pool = [torch.cuda.Stream(dev) for _ in range(6)] + [torch.cuda.Stream(dev, priority=-1)]
    for j, s2 in enumerate(pool):
        sd = s2
        t, ok = timed(pipelined)
        print(f"probe {j} {t * 1e3:7.3f} ms ok={ok}", flush=True)
if len(sys.argv) > 3:
    modes = [m for m in modes if m[0] == sys.argv[3]]
for rep in range(3 if len(sys.argv) <= 3 else 1):
    for name, fn in modes:
        t, ok = timed(fn)
        print(f"{name:10s} {t * 1e3:7.3f} ms/round trip  {in_bytes / t / GIB:6.2f} GiB/s  ok={ok}", flush=True)
