#!/bin/bash
# Round evidence on one GPU box: benches (C2 full line incl. cpu_baseline and
# PCIe-inclusive rate, C3, C4), rocprofv3 kernel trace + PMC passes of the C2
# bench (tools/profile.sh) and the HBM traffic summary (tools/traffic.py).
# usage: tools/evidence.sh TAG   -> gpurun_out/ev_TAG/...
set -e
cd "$(dirname "$0")/.."
T=${1:-r1}
O=gpurun_out/ev_$T
mkdir -p $O
timeout -k 10 400 python bench.py > $O/bench_c2.log 2>&1
timeout -k 10 300 python bench.py --no-cpu --no-pcie --no-crc --workload c3 > $O/bench_c3.log 2>&1
timeout -k 10 300 python bench.py --no-cpu --no-pcie --no-crc --workload c4 --packets 1048576 --steps 2 > $O/bench_c4.log 2>&1
bash tools/profile.sh ev_$T
python3 tools/traffic.py gpurun_out/prof_ev_$T c2 65536 $O/traffic_c2.json
python3 tools/pmc_summary.py gpurun_out/prof_ev_$T > $O/pmc_c2.json
cp gpurun_out/prof_ev_$T/kt/*kernel_stats.csv $O/kernel_stats.csv
echo evidence-done
