#!/bin/bash
# A/B of the lane kernel versions on one GPU box (ENET_RC_KERNEL=lane2 vs the default v3)
cd "$(dirname "$0")/.."
for w in ${1:-c2 c3}; do
  for k in lane3 lane2; do
    ENET_RC_KERNEL=$k timeout -k 10 200 python bench.py --no-cpu --no-pcie --no-crc --workload $w > gpurun_out/abk_${k}_$w.log 2>&1 || exit 1
  done
done
for f in gpurun_out/abk_*.log; do echo "$f $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["compress_GiBps"], d["decompress_GiBps"], d["bit_exact_roundtrip"])')"; done
