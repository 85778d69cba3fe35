#!/bin/bash
# rocprof kernel times of rc_decompress_dec6 for library variants (tools/dec6_variants.sh), C2.
# usage: tools/dec6_ab.sh TAG name...
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$1; shift
O=$R/gpurun_out/$T; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for n in "$@"; do
  ENET_RC_LIB=$R/enet_amd/lib/libenet_rc_amd_$n.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$n -o run -- python3 $R/bench.py --no-cpu --no-pcie --no-crc --no-dgram --no-configs --no-multi --steps 3 > $O/bench_$n.log 2>&1 || exit 1
  echo "$n: $(grep '^{' $O/bench_$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["decompress_GiBps"], d["bit_exact_roundtrip"], d["lane_handoff"])') $(grep -E 'dec6' $(find $O/kt_$n -name '*kernel_stats.csv' | head -1) | cut -d, -f1,4 | tr '\n' ' ')"
done
