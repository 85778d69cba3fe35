#!/bin/bash
# Interleaved A/B of environment settings on one GPU box, one process per run.
# usage: tools/abenv.sh TAG "ENET_RC_DEC=4" "ENET_RC_DEC=5" [workloads] [rounds] [packets]
#   -> gpurun_out/<TAG>/ab_<i>_<w>_<r>.log + summary lines
cd "$(dirname "$0")/.."
T=$1; A=$2; B=$3; W=${4:-c2}; R=${5:-2}
mkdir -p gpurun_out/$T
for r in $(seq 1 $R); do
  for w in $W; do
    i=0
    for e in "$A" "$B"; do
      i=$((i + 1))
      pk=65536; st=10
      if [ "$w" = c4 ]; then pk=1048576; st=3; fi
      env $e timeout -k 10 200 python bench.py --no-cpu --no-pcie --no-crc --no-dgram --no-configs \
        --steps $st --workload $w --packets $pk > gpurun_out/$T/ab_${i}_${w}_$r.log 2>&1 || exit 1
    done
  done
done
for f in gpurun_out/$T/ab_*.log; do echo "$f $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["compress_GiBps"], d["decompress_GiBps"], d["bit_exact_roundtrip"], d["lane_handoff"])')"; done
