#!/bin/bash
# occupancy experiment: lib X with ENET_RC_LANES=L (packets per wavefront)
cd "$(dirname "$0")/.."
B="python bench.py --no-cpu --no-pcie --no-crc --steps 5"
for cfg in $1; do IFS=: read x l <<< "$cfg"
  ENET_RC_LIB=$PWD/enet_amd/lib/libenet_rc_amd_$x.so ENET_RC_LANES=$l timeout -k 10 200 $B ${2:-} > gpurun_out/occ_${x}_$l.log 2>&1 || exit 1
done
for f in gpurun_out/occ_*.log; do echo "$f $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["compress_GiBps"], d["decompress_GiBps"], d["bit_exact_roundtrip"])')"; done
