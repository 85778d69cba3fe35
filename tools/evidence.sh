#!/bin/bash
# Round evidence on one GPU box.  usage: tools/evidence.sh TAG [bench] [c2] [c3] [c4]
#   bench: the default bench line (C2 headline with the C3/C4 configs,
#          cpu_baseline, PCIe-inclusive rate, CRC-32, datagram path, multi-GPU
#          C-ABI leg) and the host-path phase profile;
#   c2|c3|c4: rocprofv3 kernel trace + PMC passes of that workload's bench
#          (tools/profile.sh), its HBM traffic summary (tools/traffic.py) and
#          PMC summary.
# -> gpurun_out/ev_TAG/{bench.log, pcie_phases.log, <wl>_kernel_stats.csv,
#    traffic_<wl>.json, pmc_<wl>.json}
set -e
cd "$(dirname "$0")/.."
T=${1:-r4}; shift
O=gpurun_out/ev_$T
mkdir -p $O
WHAT="$*"; [ -z "$WHAT" ] && WHAT="bench c2 c3 c4"
for what in $WHAT; do
  case $what in
    bench)
      timeout -k 10 500 python bench.py > $O/bench.log 2>&1
      timeout -k 10 120 python tools/pcie_prof.py > $O/pcie_phases.log 2>&1 ;;
    c2|c3|c4)
      P=65536; [ $what = c4 ] && P=1048576
      bash tools/profile.sh ev_${T}_$what --workload $what --packets $P
      python3 tools/traffic.py gpurun_out/prof_ev_${T}_$what $what $P $O/traffic_$what.json > /dev/null
      python3 tools/pmc_summary.py gpurun_out/prof_ev_${T}_$what > $O/pmc_$what.json
      cp gpurun_out/prof_ev_${T}_$what/kt/*kernel_stats.csv $O/${what}_kernel_stats.csv ;;
  esac
  echo "evidence $what done"
done
