#!/bin/bash
# Round evidence on one GPU box: the default bench line (C2 headline with
# C3/C4 configs, cpu_baseline, PCIe-inclusive rate, CRC-32, datagram path,
# multi-GPU C-ABI leg), the host-path phase profile, rocprofv3 kernel trace +
# PMC passes of the C2 bench (tools/profile.sh) and the HBM traffic summary
# (tools/traffic.py).
# usage: tools/evidence.sh TAG   -> gpurun_out/ev_TAG/...
set -e
cd "$(dirname "$0")/.."
T=${1:-r3}
O=gpurun_out/ev_$T
mkdir -p $O
timeout -k 10 500 python bench.py > $O/bench.log 2>&1
timeout -k 10 120 python tools/pcie_prof.py > $O/pcie_phases.log 2>&1
bash tools/profile.sh ev_$T
python3 tools/traffic.py gpurun_out/prof_ev_$T c2 65536 $O/traffic_c2.json
python3 tools/pmc_summary.py gpurun_out/prof_ev_$T > $O/pmc_c2.json
cp gpurun_out/prof_ev_$T/kt/*kernel_stats.csv $O/kernel_stats.csv
echo evidence-done
