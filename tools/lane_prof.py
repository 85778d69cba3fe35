#!/usr/bin/env python3
"""Per-phase cycle breakdown of the lane kernels (diagnostic build).

    make -C enet_amd/csrc prof3 && python tools/lane_prof.py [c2|c3] [packets]

Loads enet_amd/lib/libenet_rc_amd_prof3.so (rc_lane3.hip compiled with
-DRC_PROFILE: s_memtime stamps between the phases of a step, summed per wave)
and prints, per phase, shader cycles per wave-step (one byte of each of the
wave's 64 packets).  A stamp waits for outstanding LDS ops, so LDS latency is
charged to the phase that issued the op; global-memory waits land where the
data is first used.
"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["ENET_RC_LIB"] = os.path.join(ROOT, "enet_amd", "lib",
                                         os.environ.get("LANE_PROF_LIB", "libenet_rc_amd_prof3.so"))

import torch  # noqa: E402

from enet_amd import RangeCoder, compress_batch, decompress_batch, get_lib, synth  # noqa: E402

V3 = "3" in os.environ.get("LANE_PROF_LIB", "libenet_rc_amd_prof3.so")
COMP3 = ["top (record decode)", "o2 lookup", "o2 encode", "o1 lookup", "o1 encode", "root", "advance (updates, stores)",
         "input refill", "", "DRAIN (outstanding memory)"]
DEC3 = ["top (record decode)", "o2 decode", "o1 decode", "root decode", "lookups", "advance (updates, stores)",
        "output + refill", "", "", "DRAIN (outstanding memory)", "", ""]
COMP = ["take+o1 prefetch", "o2 update", "o2 encode", "o1 update+link", "o1 encode", "o2 load+stores",
        "root lookup/add", "root encode+rescale", "advance/reset", "DRAIN (outstanding memory)"]
DEC = ["o2 decode", "o1 decode", "root decode", "o1 prefetch", "o2 patch", "o1 patch+link",
       "o2 load+stores", "output", "DRAIN (outstanding memory)", "", "", "loop top/advance"]


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
    res = {}
    with RangeCoder() as rc:
        out, oo, cap, ol = compress_batch(rc, din, doff, dlen, max_len=1200)
        torch.cuda.synchronize()
        lib.rc_lane_prof_read(buf.ctypes.data, 1)
        out, oo, cap, ol = compress_batch(rc, din, doff, dlen, max_len=1200)
        torch.cuda.synchronize()
        lib.rc_lane_prof_read(buf.ctypes.data, 1)
        steps = (n // 64) * 1200
        names = COMP3 if V3 else COMP
        comp = {names[k]: round(float(buf[k]) / steps, 1) for k in range(10) if names[k]}
        comp["TOTAL"] = round(float(buf[:12].sum()) / steps, 1)
        res["compress_cycles_per_wave_step"] = comp
        back, bo, bl = decompress_batch(rc, out, oo, ol, dlen.clone(), max_len=int(ol.max().item()))
        torch.cuda.synchronize()
        lib.rc_lane_prof_read(buf.ctypes.data, 1)
        back, bo, bl = decompress_batch(rc, out, oo, ol, dlen.clone(), max_len=int(ol.max().item()))
        torch.cuda.synchronize()
        lib.rc_lane_prof_read(buf.ctypes.data, 1)
        names = DEC3 if V3 else DEC
        dec = {names[k]: round(float(buf[16 + k]) / steps, 1) for k in range(12) if names[k]}
        dec["TOTAL"] = round(float(buf[16:28].sum() - (buf[23] + buf[24] + buf[26] + buf[27] if V3 else 0)) / steps, 1)
        if V3:      # event counts (rc_lane3.hip), per lane-step
            ls = steps * 64.0
            for k in (7, 8, 10, 11):
                dec.pop(names[k], None)
            res["decompress_events_per_lane_step"] = {
                "in a dense order-1 context": round(float(buf[23]) / ls, 4),
                "dense order-1 lookups (order 1 or root steps)": round(float(buf[24]) / ls, 4),
                "order-2 hits whose link misses the LDS cache": round(float(buf[26]) / ls, 4),
                "root steps": round(float(buf[27]) / ls, 4)}
        res["decompress_cycles_per_wave_step"] = dec
        res["roundtrip_ok"] = bool(torch.equal(back, din))
    res["workload"] = wl
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
