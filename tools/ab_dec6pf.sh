#!/bin/bash
# rocprof decoder kernel time of the prefetch variants on C2 (round 5):
# cur (kPfW=1), w2, w3 builds, and cur with the prefetch off (ENET_RC_DEC6_DEBUG=4); twice each, interleaved.
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$1; O=$R/gpurun_out/$T; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for rep in 1 2; do
for n in cur w2 w3 off; do
  L=$R/enet_amd/lib/libenet_rc_amd_$n.so; [ $n = cur ] || [ $n = off ] && L=$R/enet_amd/lib/libenet_rc_amd.so
  D=0; [ $n = off ] && D=4
  rm -rf $O/kt_$n
  ENET_RC_DEC6_DEBUG=$D ENET_RC_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$n -o run -- python3 $R/bench.py --workload c2 --no-cpu --no-pcie --no-crc --no-dgram --no-configs --no-multi --steps 6 > $O/bench_$n.log 2>&1 || exit 1
  echo "$n: $(grep '^{' $O/bench_$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["decompress_GiBps"], d["bit_exact_roundtrip"], d["lane_handoff"])') $(grep -E 'rc_decompress_dec6s' $(find $O/kt_$n -name '*kernel_stats.csv' | head -1) | cut -d, -f1,4 | tr '\n' ' ')"
done
done
