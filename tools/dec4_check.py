"""Diagnostic: how many packets the bucket-history decoder leaves to the lane
kernels, per workload, and the decode time (device-resident)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from enet_amd import RangeCoder, synth  # noqa: E402


def run(kind, n=65536, size=1200):
    d, o, l = {"c2": synth.random_batch, "c3": synth.gamestate_batch}[kind](n, size)
    dev = torch.device("cuda", 0)
    din = torch.from_numpy(d).to(dev)
    doff = torch.from_numpy(o.astype(np.int64)).to(dev)
    dlen = torch.from_numpy(l.astype(np.int32)).to(dev)
    cap = (2 * dlen.to(torch.int64) + 64).to(torch.int32)
    coff = torch.zeros(n, dtype=torch.int64, device=dev)
    coff[1:] = torch.cumsum(cap[:-1].to(torch.int64), 0)
    cout = torch.empty(int(coff[-1] + cap[-1]), dtype=torch.uint8, device=dev)
    clen = torch.zeros(n, dtype=torch.int32, device=dev)
    dout = torch.empty_like(din)
    dl = torch.zeros(n, dtype=torch.int32, device=dev)
    rc = RangeCoder()
    st = torch.cuda.current_stream(dev)
    rc.compress_batch(din, doff, dlen, cout, coff, cap, clen, max_len=size, stream=st)
    torch.cuda.synchronize()
    left_c = rc.last_lane_count()
    mx = int(clen.max().item())
    for _ in range(2):
        rc.decompress_batch(cout, coff, clen, dout, doff, dlen, dl, max_len=mx, stream=st)
    torch.cuda.synchronize()
    t = time.perf_counter()
    rc.decompress_batch(cout, coff, clen, dout, doff, dlen, dl, max_len=mx, stream=st)
    torch.cuda.synchronize()
    t = time.perf_counter() - t
    ok = bool(torch.equal(dl, dlen)) and bool(torch.equal(dout, din))
    print(f"{kind} dec4={os.environ.get('ENET_RC_DEC4', '1')} compress left {left_c}, decompress left "
          f"{rc.last_lane_count()} exact {rc.last_exact_count()}  decode {t * 1e3:.2f} ms ok={ok}", flush=True)
    rc.close()


if __name__ == "__main__":
    for k in sys.argv[1:] or ["c2", "c3"]:
        run(k)
