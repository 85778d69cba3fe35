#!/bin/bash
# Interleaved A/B of the fast decoders on one GPU box (ENET_RC_DEC=6 / 4):
# usage: tools/ab_dec.sh TAG [workloads] [rounds]  -> gpurun_out/TAG/abd_<dec>_<w>_<r>.log + summary
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-abd}; mkdir -p $O
for r in $(seq 1 ${3:-2}); do
  for w in ${2:-c2}; do
    for x in 6 4; do
      ENET_RC_DEC=$x timeout -k 10 200 python bench.py --no-cpu --no-pcie --no-crc --no-dgram --no-configs --no-multi --steps 8 --workload $w > $O/abd_${x}_${w}_$r.log 2>&1 || exit 1
    done
  done
done
for f in $O/abd_*.log; do echo "$f $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["compress_GiBps"], d["decompress_GiBps"], d["bit_exact_roundtrip"], d.get("lane_handoff"))')"; done
