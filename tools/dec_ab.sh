#!/bin/bash
# A/B of decoder configurations on one box: C2 bench line + rocprof kernel stats each.
# usage: tools/dec_ab.sh TAG "name ENV=V ENV=V" ["name ENV=V"]...   (workload: WL=c2|c3|c4)
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$1; shift
O=$R/gpurun_out/$T; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
WL=${WL:-c2}
P=65536; [ "$WL" = c4 ] && P=1048576
for spec in "$@"; do
  set -- $spec; n=$1; shift
  env "$@" timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$n -o run -- python3 $R/bench.py --workload $WL --packets $P --no-cpu --no-pcie --no-crc --no-dgram --no-configs --no-multi --steps 5 > $O/bench_$n.log 2>&1 || { echo "$n failed"; tail -5 $O/bench_$n.log; exit 1; }
  cp $(find $O/kt_$n -name "*kernel_stats.csv" | head -1) $O/${n}_kernel_stats.csv
  echo "$n: $(grep '^{' $O/bench_$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], "c", d["compress_GiBps"], "d", d["decompress_GiBps"], d["bit_exact_roundtrip"], d["lane_handoff"])')"
  grep -E "dec6|dec7|dec4|lane3|enc2" $O/${n}_kernel_stats.csv | cut -d, -f1-5
done
