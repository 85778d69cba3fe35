#!/bin/bash
# rocprof kernel trace of bench.py (C2) under environment settings, alternating;
# prints the round-trip period per setting (tools/step_period.py).
# usage: tools/env_kt.sh TAG ROUNDS "ENV=.." "ENV=.." ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$1; N=$2; shift 2
O=$R/gpurun_out/$T; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for r in $(seq 1 $N); do
  i=0
  for e in "$@"; do
    i=$((i+1))
    env $e timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/kt_${i}_$r -o run -- python3 $R/bench.py --no-cpu --no-pcie --no-crc --no-dgram --no-configs --no-multi --steps 10 > $O/bench_${i}_$r.log 2>&1 || exit 1
    echo "$e round $r: $(grep '^{' $O/bench_${i}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["bit_exact_roundtrip"])') $(python3 $R/tools/step_period.py $(find $O/kt_${i}_$r -name '*kernel_trace.csv' | head -1))"
  done
done
