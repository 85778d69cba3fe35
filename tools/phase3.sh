#!/bin/bash
# phase-cycle stamps of the v3 lane kernels (diagnostic builds) -> gpurun_out/phase3_*.json
set -e
cd "$(dirname "$0")/.."
for w in ${1:-c2 c3}; do
  LANE_PROF_LIB=libenet_rc_amd_prof3.so timeout -k 10 120 python tools/lane_prof.py $w > gpurun_out/phase3_$w.json
  LANE_PROF_LIB=libenet_rc_amd_drain3.so timeout -k 10 120 python tools/lane_prof.py $w > gpurun_out/phase3_drain_$w.json
done
