#!/bin/bash
# A/B/... timing on one GPU box: ENET_RC_LIB=enet_amd/lib/libenet_rc_amd_<X>.so for each X given.
# usage: tools/abn.sh "A B C" [workloads]   -> gpurun_out/abn_<X>_<w>.log
cd "$(dirname "$0")/.."
for w in ${2:-c2 c3}; do
  for x in $1; do
    ENET_RC_LIB=$PWD/enet_amd/lib/libenet_rc_amd_$x.so timeout -k 10 200 python bench.py --no-cpu --no-pcie --no-crc --workload $w > gpurun_out/abn_${x}_$w.log 2>&1 || exit 1
  done
done
for f in gpurun_out/abn_*.log; do echo "$f $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["compress_GiBps"], d["decompress_GiBps"], d["bit_exact_roundtrip"])')"; done
