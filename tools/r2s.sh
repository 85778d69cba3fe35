set -o pipefail
R=$(pwd)
mkdir -p gpurun_out/r2s
cd /tmp && export TMPDIR=/tmp
ENET_RC_DEC4=1 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r2s/kt -o run -- python3 $R/bench.py --no-cpu --no-pcie --no-crc --no-dgram --no-rccl --steps 4 --warmup 1 > $R/gpurun_out/r2s/bench.log 2>&1; echo "rc=$?"
f=$(find $R/gpurun_out/r2s/kt -name "*kernel_trace.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
ks = [(int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name'][:22]) for r in rows]
ks.sort()
t0 = ks[0][0]
for s, e, n in ks[-40:]:
    if (e - s) > 50000:
        print(f"{(s-t0)/1e6:9.3f} {(e-t0)/1e6:9.3f} {(e-s)/1e6:7.3f} {n}")
PY
