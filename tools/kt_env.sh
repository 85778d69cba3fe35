#!/bin/bash
# rocprof kernel times under environment settings (one process each) on one
# workload: the bench line and the kernels matching a pattern per setting.
# usage: tools/kt_env.sh TAG WORKLOAD 'kernel-regex' "VAR=x [VAR2=y]" ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$1; W=$2; K=$3; shift 3
O=$R/gpurun_out/$T; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for e in "$@"; do
  i=$((i + 1))
  for kv in $e; do export "$kv"; done
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_${i}_$W -o run -- python3 $R/bench.py --no-cpu --no-pcie --no-crc --no-dgram --no-configs --no-multi --steps ${KT_STEPS:-5} --workload $W ${KT_ARGS} > $O/bench_${i}_$W.log 2>&1 || exit 1
  for kv in $e; do unset "${kv%%=*}"; done
  echo "[$e] $W: $(grep '^{' $O/bench_${i}_$W.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["compress_GiBps"], d["decompress_GiBps"], d["bit_exact_roundtrip"], d["lane_handoff"])') $(grep -E "$K" $(find $O/kt_${i}_$W -name '*kernel_stats.csv' | head -1) | cut -d, -f1,4 | tr '\n' ' ')"
done
