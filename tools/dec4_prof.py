#!/usr/bin/env python3
"""Per-phase cycle breakdown of the bucket-history decoder (diagnostic build).

    make -C enet_amd/csrc prof4 && python tools/dec4_prof.py [c2|c3] [packets]

Loads enet_amd/lib/libenet_rc_amd_prof4.so (rc_dec4.hip compiled with
-DRC_PROFILE: s_memtime stamps between the phases of a step, summed per
wave; DEC4_PROF_LIB=libenet_rc_amd_drain4.so also waits for all memory at
the top of each step, charged to DRAIN) and prints shader cycles per
wave-step.  A stamp waits for outstanding LDS ops, so LDS latency is charged
to the phase that issued the op; global-memory waits land where the data is
first used (the record: "top").
"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["ENET_RC_LIB"] = os.path.join(ROOT, "enet_amd", "lib",
                                         os.environ.get("DEC4_PROF_LIB", "libenet_rc_amd_prof4.so"))

import torch  # noqa: E402

from enet_amd import RangeCoder, compress_batch, decompress_batch, get_lib, synth  # noqa: E402

NAMES = ["top (record wait, output store)", "groups", "sub-context decode", "root decode",
         "load issue, rank, flags", "insert + record store", "output + input", "", "", "DRAIN (outstanding memory)"]


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "c2"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
    d, o, l = synth.random_batch(n, 1200) if wl == "c2" else synth.gamestate_batch(n, 1200)
    lib = get_lib()
    lib.rc_lane_prof_read.restype = C.c_int
    lib.rc_lane_prof_read.argtypes = [C.c_void_p, C.c_int]
    buf = np.zeros(64, np.uint64)
    din = torch.from_numpy(d).cuda()
    doff = torch.from_numpy(o.astype(np.int64)).cuda()
    dlen = torch.from_numpy(l.astype(np.int32)).cuda()
    with RangeCoder() as rc:
        out, oo, cap, ol = compress_batch(rc, din, doff, dlen, max_len=1200)
        mx = int(ol.max().item())
        back, bo, bl = decompress_batch(rc, out, oo, ol, dlen.clone(), max_len=mx)
        torch.cuda.synchronize()
        lib.rc_lane_prof_read(buf.ctypes.data, 1)
        back, bo, bl = decompress_batch(rc, out, oo, ol, dlen.clone(), max_len=mx)
        torch.cuda.synchronize()
        lib.rc_lane_prof_read(buf.ctypes.data, 1)
        ok = bool(torch.equal(bl, dlen)) and bool(torch.equal(back, din))
    steps = (n // 64) * 1200
    res = {nm: round(float(buf[16 + k]) / steps, 1) for k, nm in enumerate(NAMES) if nm}
    res["TOTAL"] = round(sum(float(buf[16 + k]) for k in range(12)) / steps, 1)
    print(json.dumps({"decompress_cycles_per_wave_step": res, "roundtrip_ok": ok, "workload": wl}, indent=1))


if __name__ == "__main__":
    main()
