#!/bin/bash
# A/B timing on one GPU box: enet_amd/lib/libenet_rc_amd_A.so (baseline) vs the
# current libenet_rc_amd.so, interleaved, C2 and C3.  Output: gpurun_out/ab_*.log
cd "$(dirname "$0")/.."
A=$PWD/enet_amd/lib/libenet_rc_amd_A.so
for i in 1 2; do
  for w in c2 c3; do
    ENET_RC_LIB=$A timeout -k 10 200 python bench.py --no-cpu --no-pcie --no-crc --workload $w > gpurun_out/ab_A_${w}_$i.log 2>&1 || exit 1
    timeout -k 10 200 python bench.py --no-cpu --no-pcie --no-crc --workload $w > gpurun_out/ab_B_${w}_$i.log 2>&1 || exit 1
  done
done
