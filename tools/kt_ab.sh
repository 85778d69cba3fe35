#!/bin/bash
# rocprof kernel times of library variants (libenet_rc_amd_<name>.so) on one
# workload: the bench line and the kernels matching a pattern, per variant.
# usage: tools/kt_ab.sh TAG WORKLOAD 'kernel-regex' name...
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$1; W=$2; K=$3; shift 3
O=$R/gpurun_out/$T; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for n in "$@"; do
  ENET_RC_LIB=$R/enet_amd/lib/libenet_rc_amd_$n.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_${n}_$W -o run -- python3 $R/bench.py --no-cpu --no-pcie --no-crc --no-dgram --no-configs --no-multi --steps 5 --workload $W > $O/bench_${n}_$W.log 2>&1 || exit 1
  echo "$n $W: $(grep '^{' $O/bench_${n}_$W.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["compress_GiBps"], d["decompress_GiBps"], d["bit_exact_roundtrip"], d["lane_handoff"])') $(grep -E "$K" $(find $O/kt_${n}_$W -name '*kernel_stats.csv' | head -1) | cut -d, -f1,4 | tr '\n' ' ')"
done
