#!/bin/bash
# Interleaved A/B/... timing on one GPU box: ENET_RC_LIB=enet_amd/lib/libenet_rc_amd_<X>.so
# usage: tools/abn.sh "A B" [workloads] [rounds]   -> gpurun_out/abn_<X>_<w>_<r>.log + summary
cd "$(dirname "$0")/.."
for r in $(seq 1 ${3:-2}); do
  for w in ${2:-c2 c3}; do
    for x in $1; do
      ENET_RC_LIB=$PWD/enet_amd/lib/libenet_rc_amd_$x.so timeout -k 10 200 python bench.py --no-cpu --no-pcie --no-crc --steps 8 --workload $w > gpurun_out/abn_${x}_${w}_$r.log 2>&1 || exit 1
    done
  done
done
for f in gpurun_out/abn_*.log; do echo "$f $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["compress_GiBps"], d["decompress_GiBps"], d["bit_exact_roundtrip"])')"; done
