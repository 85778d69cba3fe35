#!/bin/bash
# rocprof kernel averages of library builds on one workload: tools/ab_kt.sh TAG WORKLOAD "KERNEL_REGEX" name...
# (names: enet_amd/lib/libenet_rc_amd_<name>.so; "cur" = libenet_rc_amd.so)
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$1; W=$2; K=$3; shift 3
O=$R/gpurun_out/$T; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for n in "$@" "$@"; do
  L=$R/enet_amd/lib/libenet_rc_amd_$n.so; [ $n = cur ] && L=$R/enet_amd/lib/libenet_rc_amd.so
  rm -rf $O/kt_$n
  ENET_RC_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$n -o run -- python3 $R/bench.py --workload $W --no-cpu --no-pcie --no-crc --no-dgram --no-configs --no-multi --steps 4 > $O/bench_$n.log 2>&1 || exit 1
  echo "$n: $(grep '^{' $O/bench_$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["compress_GiBps"], d["decompress_GiBps"], d["bit_exact_roundtrip"])') $(grep -E "$K" $(find $O/kt_$n -name '*kernel_stats.csv' | head -1) | cut -d, -f1,4 | tr '\n' ' ')"
done
