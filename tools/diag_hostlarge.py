"""Diagnostic: the host-pointer large-batch round trip (test_host_pointer_batches_large)
repeated per kernel configuration; prints which packets decode wrongly and how."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from enet_amd import RangeCoder, synth  # noqa: E402
from oracle.pyoracle import compress_batch as ocompress  # noqa: E402

VARS = {"lane3": {}, "enc2-slow": {"ENET_RC_ENC2_SLOW": "1"}, "nodec": {"ENET_RC_DEC": "0"}}
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
d, o, l = synth.mixed_batch(30000)
n = len(l)
ln = l.astype(np.uint32)
cap = (2 * ln.astype(np.int64) + 64).astype(np.uint32)
coff = np.zeros(n, np.uint64)
coff[1:] = np.cumsum(cap[:-1].astype(np.uint64) + 3)
want, wo, wcap, wl = ocompress(d, o, l, "port")
p = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
for name, env in VARS.items():
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    rc = RangeCoder()
    for k, v in old.items():
        if v is None:
            os.environ.pop(k, None)
    lib = rc.lib
    for r in range(reps):
        cout = np.zeros(int(coff[-1] + cap[-1]) + 16, np.uint8)
        clen = np.zeros(n, np.uint32)
        assert lib.enet_rc_compress_batch_host(rc.ctx, p(d), p(o), p(ln), n, p(cout), p(coff), p(cap), p(clen)) == 0
        cbad = int((clen != wl).sum())
        dout = np.zeros(int(o[-1]) + int(l[-1]) + 16, np.uint8)
        dlen = np.zeros(n, np.uint32)
        assert lib.enet_rc_decompress_batch_host(rc.ctx, p(cout), p(coff), p(clen), n, p(dout), p(o), p(ln),
                                                 p(dlen)) == 0
        lanes = rc.last_lane_count()
        bad = np.nonzero(dlen != ln)[0]
        cont = [i for i in range(n) if dlen[i] == ln[i] and
                not np.array_equal(dout[int(o[i]): int(o[i]) + int(ln[i])], d[int(o[i]): int(o[i]) + int(ln[i])])]
        print(f"{name} rep {r}: compress mismatches {cbad}, decoder hand-off {lanes}, wrong lengths {len(bad)}, "
              f"wrong bytes {len(cont)}", flush=True)
        for i in list(bad[:8]) + cont[:8]:
            i = int(i)
            got = dout[int(o[i]): int(o[i]) + int(ln[i])]
            ref = d[int(o[i]): int(o[i]) + int(ln[i])]
            first = int(np.argmax(got != ref)) if not np.array_equal(got, ref) else -1
            print(f"   pkt {i}: len {ln[i]} got {dlen[i]} clen {clen[i]} first diff at {first} "
                  f"(slot {i % 65536}, lane {i % 64}, wave {(i // 64) % 4})", flush=True)
    rc.close()
