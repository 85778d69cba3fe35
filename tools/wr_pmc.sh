#!/bin/bash
# HBM write requests of one kernel (one PMC pass: TCC_EA0_WRREQ, _64B) on a
# bench workload.  usage: PMC_TAG=x PMC_KERNEL=regex PMC_WL=c3 tools/wr_pmc.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
D=$R/gpurun_out/${PMC_TAG:-wrpmc}
mkdir -p $D
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --kernel-include-regex "${PMC_KERNEL}" \
  --output-format csv -d $D/pmc -o run -- python3 $R/bench.py --workload ${PMC_WL:-c3} --no-cpu --no-pcie --no-crc \
  --no-dgram --no-rccl --no-configs --no-multi --steps 1 --warmup 0 > $D/p.log 2>&1 || exit 1
python3 - "$D" <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for f in glob.glob(sys.argv[1] + "/pmc/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        n[(k, r["Counter_Name"])] += 1
for k, c in acc.items():
    calls = max(v for (kk, _), v in n.items() if kk == k)
    w, w64 = c.get("TCC_EA0_WRREQ_sum", 0) / calls, c.get("TCC_EA0_WRREQ_64B_sum", 0) / calls
    print(f"{k}: {calls} calls, write requests {w/1e6:.1f} M ({w64/1e6:.1f} M of 64 B): {(w64 * 64 + (w - w64) * 32) / 1e9:.3f} GB per launch")
PY
