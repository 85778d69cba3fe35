set -o pipefail
R=$(pwd)
mkdir -p gpurun_out/r2t
for D in 0 1; do
ENET_RC_DEC4=$D timeout -k 10 300 python3 bench.py --no-cpu --no-pcie --no-crc --no-dgram --no-rccl --steps 10 > gpurun_out/r2t/bench_c2_d$D.log 2>&1; echo "bench dec4=$D rc=$?"
python3 -c "import json; d=json.loads(open('gpurun_out/r2t/bench_c2_d$D.log').read().strip().splitlines()[-1]); print({k: d.get(k) for k in ('value','pipelined_GiBps','sequential_GiBps','compress_GiBps','decompress_GiBps','bit_exact_roundtrip')})"
done
cd /tmp && export TMPDIR=/tmp
ENET_RC_DEC4=1 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r2t/kt -o run -- python3 $R/bench.py --no-cpu --no-pcie --no-crc --no-dgram --no-rccl --steps 4 --warmup 1 > $R/gpurun_out/r2t/bench.log 2>&1; echo "rc=$?"
f=$(find $R/gpurun_out/r2t/kt -name "*kernel_trace.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
ks = sorted(rows, key=lambda r: int(r['Start_Timestamp']))
t0 = int(ks[0]['Start_Timestamp'])
for r in ks[-30:]:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    if e - s > 50000: print(f"{(s-t0)/1e6:9.3f} {(e-t0)/1e6:9.3f} {(e-s)/1e6:7.3f} q={r.get('Queue_Id')} st={r.get('Stream_Id')} {r['Kernel_Name'][:26]}")
PY
