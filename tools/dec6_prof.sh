#!/bin/bash
# Kernel times of the C2 decompress with the fast decoders (diagnostic):
# tools/dec6_prof.sh TAG  -> gpurun_out/TAG/{dec6,dec4,dec6nr}_kernel_stats.csv
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --no-cpu --no-pcie --no-crc --no-dgram --no-configs --no-multi --steps 3"
for v in "dec6 6 0" "dec4 4 0" "dec6nr 6 2"; do
  set -- $v
  ENET_RC_DEC=$2 ENET_RC_DEC6_DEBUG=$3 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$1 -o run -- $B > $O/bench_$1.log 2>&1 || exit 1
  cp $(find $O/kt_$1 -name "*kernel_stats.csv" | head -1) $O/$1_kernel_stats.csv
  echo "$1: $(grep '^{' $O/bench_$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["decompress_GiBps"], d["lane_handoff"])')"
  grep -E "dec6|dec4|lane3" $O/$1_kernel_stats.csv | cut -d, -f1-5
done
