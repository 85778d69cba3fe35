#!/usr/bin/env python3
"""Per-phase cycles of rc_dec7.hip (diagnostic build: tools/dec7_variants.sh
prof7 "-DRC_PROFILE"), C2 or C3:

    DEC7_PROF_LIB=libenet_rc_amd_prof7.so python tools/dec7_phase.py [c2|c3] [packets]

Main wavefronts: shader cycles per packet-step by phase; stalled / stepping
lanes per step; idle steps.  Helper wavefronts: passes, idle passes, lanes
served, cycles serving, ring passes."""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["ENET_RC_LIB"] = os.path.join(ROOT, "enet_amd", "lib", os.environ.get("DEC7_PROF_LIB", "libenet_rc_amd_prof7.so"))
os.environ.setdefault("ENET_RC_DEC", "7")

import torch  # noqa: E402

from enet_amd import RangeCoder, compress_batch, decompress_batch, get_lib, synth  # noqa: E402

NAMES = {0: "main: common step", 1: "main: answers applied", 2: "main: input + publish", 3: "main: bail check + idle"}


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
        handed = rc.last_lane_count()
    waves = n // 64
    steps = waves * 1200
    b = [float(x) for x in buf]
    res = {nm: round(b[16 + k] / steps, 1) for k, nm in NAMES.items()}
    res["TOTAL main cycles per packet-step"] = round(sum(b[16 + k] for k in NAMES) / steps, 1)
    res["loop steps per packet-step"] = round(b[16 + 8] / steps, 3)
    res["stalled lanes per loop step"] = round(b[16 + 9] / max(b[16 + 8], 1), 2)
    res["stepping lanes per loop step"] = round(b[16 + 10] / max(b[16 + 8], 1), 2)
    res["idle loop steps per wave"] = round(b[16 + 11] / max(waves, 1), 1)
    res["done lanes per loop step"] = round(b[16 + 7] / max(b[16 + 8], 1), 2)
    res["lanes with c used up per loop step"] = round(b[16 + 5] / max(b[16 + 8], 1), 2)
    hw = waves   # one helper wavefront per main wavefront
    res["helper passes per wave"] = round(b[32] / hw, 1)
    res["helper idle passes per wave"] = round(b[33] / hw, 1)
    res["helper cycles per wave"] = round(b[34] / hw, 1)
    res["helper requests served per wave"] = round(b[35] / hw, 1)
    res["helper serve cycles per wave"] = round(b[36] / hw, 1)
    res["helper ring passes per wave"] = round(b[37] / hw, 1)
    res["helper cycles to the loads' arrival per wave"] = round(b[38] / hw, 1)
    res["helper compaction cycles per wave"] = round(b[39] / hw, 1)
    res["helper decode cycles per wave"] = round(b[40] / hw, 1)
    res["helper chain iterations per wave"] = round(b[41] / hw, 1)
    res["ring-full lanes per loop step"] = None
    print(json.dumps({"dec7": res, "roundtrip_ok": ok, "lanes_handed_on": handed, "workload": wl}, indent=1))


if __name__ == "__main__":
    main()
