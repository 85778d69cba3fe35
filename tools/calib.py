"""Summary of tools/calib.sh: per calibration kernel (tools/mb/calib.hip, in
launch order), memory-side requests per access by size class, and the bytes
traffic.py's formula assigns against the bytes the kernel moves."""
import collections
import csv
import glob
import json
import sys

d = sys.argv[1]
log = [l.split() for l in open(f"{d}/calib.log") if l.strip()]
# name table MB accesses width bytes
runs = [(l[0], int(l[2]), int(l[5]), int(l[7].rstrip("B")) if l[7].rstrip("B").isdigit() else int(l[7]), int(l[-1]))
        for l in log]
per = collections.defaultdict(dict)          # dispatch index -> counters
for f in sorted(glob.glob(f"{d}/pmc*/run_counter_collection.csv")):
    disp = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        if "calib" in r["Kernel_Name"]:
            disp[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, (did, cs) in enumerate(sorted(disp.items())):
        per[k].update(cs)
out = []
for k, (name, mb, acc, width, nbytes) in enumerate(runs):
    m = per.get(k, {})
    wr, wr64 = m.get("TCC_EA0_WRREQ", 0.0), m.get("TCC_EA0_WRREQ_64B", 0.0)
    rd = m.get("TCC_EA0_RDREQ", 0.0)
    r32, r64, r128 = m.get("TCC_EA0_RDREQ_32B", 0.0), m.get("TCC_EA0_RDREQ_64B", 0.0), m.get("TCC_EA0_RDREQ_128B", 0.0)
    row = {"kernel": name, "table_MB": mb, "accesses": acc, "width_B": width, "bytes": nbytes,
           "wrreq_per_access": round(wr / acc, 3), "wrreq64_per_access": round(wr64 / acc, 3),
           "rdreq_per_access": round(rd / acc, 3), "rd32_per_access": round(r32 / acc, 3),
           "rd64_per_access": round(r64 / acc, 3), "rd128_per_access": round(r128 / acc, 3),
           "formula_bytes_per_access": round((64 * wr64 + 32 * (wr - wr64) + 32 * r32 + 64 * r64 + 128 * r128) / acc, 1),
           "FETCH_SIZE_B_per_access": round(m.get("FETCH_SIZE", 0.0) * 1024 / acc, 1),
           "WRITE_SIZE_B_per_access": round(m.get("WRITE_SIZE", 0.0) * 1024 / acc, 1),
           "l2_hit": round(m.get("TCC_HIT_sum", 0.0) / max(m.get("TCC_HIT_sum", 0.0) + m.get("TCC_MISS_sum", 0.0), 1), 3)}
    out.append(row)
    print(json.dumps(row))
json.dump(out, open(f"{d}/calib.json", "w"), indent=1)
