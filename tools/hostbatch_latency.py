"""Host-pointer batch latency (enet_rc_{compress,decompress}_batch_host) for
small batches, wave kernel vs lane kernel (ENET_RC_SMALL_BATCH=0 forces the
lanes; the variable is read at context creation).  Decompress batches pass
max(out_cap) to the wave decoder, which sizes its LDS arena by it, so up to
~1280 packets of 1200 B fit on the chip at one wavefront per packet.
usage: python tools/hostbatch_latency.py [reps]   (GPU box)
"""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from enet_amd import RangeCoder, synth  # noqa: E402


def run(n, kind, small, reps):
    if small is None:
        os.environ.pop("ENET_RC_SMALL_BATCH", None)
    else:
        os.environ["ENET_RC_SMALL_BATCH"] = str(small)
    d, o, l = (synth.random_batch if kind == "random" else synth.gamestate_batch)(n, 1200)
    ln = l.astype(np.uint32)
    o = o.astype(np.uint64)
    cap = (2 * ln.astype(np.int64) + 64).astype(np.uint32)
    coff = np.zeros(n, np.uint64)
    coff[1:] = np.cumsum(cap[:-1].astype(np.uint64))
    cout = np.zeros(int(coff[-1] + cap[-1]) + 16, np.uint8)
    clen = np.zeros(n, np.uint32)
    dout = np.zeros(d.size + 16, np.uint8)
    dlen = np.zeros(n, np.uint32)
    p = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
    with RangeCoder() as rc:
        lib = rc.lib
        tc, td = [], []
        for _ in range(reps + 2):
            t0 = time.perf_counter()
            assert lib.enet_rc_compress_batch_host(rc.ctx, p(d), p(o), p(ln), n, p(cout), p(coff), p(cap), p(clen)) == 0
            t1 = time.perf_counter()
            assert lib.enet_rc_decompress_batch_host(rc.ctx, p(cout), p(coff), p(clen), n, p(dout), p(o), p(ln),
                                                     p(dlen)) == 0
            t2 = time.perf_counter()
            tc.append(t1 - t0)
            td.append(t2 - t1)
        assert np.array_equal(dlen, ln) and np.array_equal(dout[: d.size], d)
    return round(float(np.median(tc[2:])) * 1e3, 3), round(float(np.median(td[2:])) * 1e3, 3)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    rows = []
    for kind in ("random", "gamestate"):
        for n in (256, 512, 768, 1024, 1280):
            wc, wd = run(n, kind, None, reps)
            lc, ld = run(n, kind, 0, reps)
            rows.append({"kind": kind, "packets": n, "bytes": 1200,
                         "auto_compress_ms": wc, "auto_decompress_ms": wd,
                         "lanes_compress_ms": lc, "lanes_decompress_ms": ld})
            print(json.dumps(rows[-1]), flush=True)


if __name__ == "__main__":
    main()
