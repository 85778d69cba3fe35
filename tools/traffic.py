#!/usr/bin/env python3
"""HBM traffic per launch of each rc_* kernel from rocprofv3 PMC passes.

usage: tools/traffic.py PROFILE_DIR WORKLOAD PACKETS OUT.json

Reads the per-dispatch counter CSVs written by tools/profile.sh (separate
--pmc passes) and reports, per kernel, mean bytes per launch:
  read  = 32*TCC_EA0_RDREQ_32B + 64*TCC_EA0_RDREQ_64B + 128*TCC_EA0_RDREQ_128B
          (request-size-resolved, so the gfx950 "FETCH_SIZE counts a 128-B
          request as 64 B" under-count of MI355X_MICROARCH.md §HBM does not apply)
  write = 64*TCC_EA0_WRREQ_64B + 32*(TCC_EA0_WRREQ - TCC_EA0_WRREQ_64B)
FETCH_SIZE / WRITE_SIZE (KiB) are reported beside them for reference.
The request sizes are calibrated (tools/mb/calib.hip, tools/calib.sh,
profiles/r6/calib_counters.json); the counters include Infinity-Cache hits.
"""
import collections
import csv
import glob
import json
import os
import sys

d, workload, packets, out = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
per = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{d}/pmc*/run_counter_collection.csv")):
    disp = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        if r["Kernel_Name"].startswith("rc_"):
            disp[(r["Kernel_Name"], r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    for (k, _), cs in disp.items():
        for c, v in cs.items():
            per[k][c].append(v)
kernels = {}
for k, cs in per.items():
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    rd = None
    if all(c in m for c in ("TCC_EA0_RDREQ_32B", "TCC_EA0_RDREQ_64B", "TCC_EA0_RDREQ_128B")):
        rd = 32 * m["TCC_EA0_RDREQ_32B"] + 64 * m["TCC_EA0_RDREQ_64B"] + 128 * m["TCC_EA0_RDREQ_128B"]
    wr = None
    if "TCC_EA0_WRREQ" in m and "TCC_EA0_WRREQ_64B" in m:
        wr = 64 * m["TCC_EA0_WRREQ_64B"] + 32 * (m["TCC_EA0_WRREQ"] - m["TCC_EA0_WRREQ_64B"])
    kernels[k] = {
        "hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr,
        "hbm_bytes_per_launch": (rd + wr) if rd is not None and wr is not None else None,
        "FETCH_SIZE_KiB": m.get("FETCH_SIZE"), "WRITE_SIZE_KiB": m.get("WRITE_SIZE"),
        "counters": m,
    }
json.dump({"workload": workload, "packets": packets, "source": os.path.basename(os.path.normpath(d)),
           "note": "bytes the L2 requests from the fabric (TCC_EA0 request counters, request-size "
                   "resolved), Infinity-Cache hits included: an upper bound of HBM traffic, not HBM "
                   "traffic.  Request sizes calibrated on the decoders' access widths by "
                   "tools/mb/calib.hip (profiles/r6/calib_counters.json): a 2/4/16-B store at a "
                   "random address is one 32-B WRREQ, a 16/64-B random load one 128-B RDREQ, 48-B "
                   "1.25; coalesced 16-B-per-lane streams exact.",
           "kernels": kernels}, open(out, "w"), indent=1)
print(json.dumps({k: {kk: vv for kk, vv in v.items() if kk != "counters"} for k, v in kernels.items()}, indent=1))
