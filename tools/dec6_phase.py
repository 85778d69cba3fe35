#!/usr/bin/env python3
"""Per-phase cycle breakdown of the record-light decoder (diagnostic build:
tools/dec6_variants.sh prof6 "-DRC_PROFILE"), C2 or C3:

    python tools/dec6_phase.py [c2|c3] [packets]

Shader cycles per wave, summed over the phases of rc_dec6.hip, divided by
the wave's packet-steps (1200 per packet); rare iterations and the lanes
they served are counts, not cycles."""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["ENET_RC_LIB"] = os.path.join(ROOT, "enet_amd", "lib", os.environ.get("DEC6_PROF_LIB", "libenet_rc_amd_prof6.so"))

import torch  # noqa: E402

from enet_amd import RangeCoder, compress_batch, decompress_batch, get_lib, synth  # noqa: E402

NAMES = {0: "common steps", 5: "common: input advance (src_adv)", 1: "rare: drain + record loads",
         2: "rare: decode", 3: "rare: update, output", 4: "wave bail check"}


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
        decompress_batch(rc, out, oo, ol, dlen.clone(), max_len=mx)
        torch.cuda.synchronize()
        lib.rc_lane_prof_read(buf.ctypes.data, 1)
        back, bo, bl = decompress_batch(rc, out, oo, ol, dlen.clone(), max_len=mx)
        torch.cuda.synchronize()
        lib.rc_lane_prof_read(buf.ctypes.data, 1)
        ok = bool(torch.equal(bl, dlen)) and bool(torch.equal(back, din))
    waves = n // 64
    steps = waves * 1200
    res = {nm: round(float(buf[16 + k]) / steps, 1) for k, nm in NAMES.items()}
    res["TOTAL cycles per packet-step"] = round(sum(float(buf[16 + k]) for k in NAMES) / steps, 1)
    res["rare iterations per wave"] = round(float(buf[16 + 8]) / waves, 1)
    res["stalled lanes per rare iteration"] = round(float(buf[16 + 9]) / max(float(buf[16 + 8]), 1), 2)
    print(json.dumps({"dec6_cycles": res, "roundtrip_ok": ok, "workload": wl}, indent=1))


if __name__ == "__main__":
    main()
