#!/bin/bash
# phase-cycle stamps (diagnostic builds) for C2 and C3 -> gpurun_out/phase_*.json
set -e
cd "$(dirname "$0")/.."
for w in c2 c3; do
  timeout -k 10 120 python tools/lane_prof.py $w > gpurun_out/phase_$w.json
  LANE_PROF_LIB=libenet_rc_amd_drain3.so timeout -k 10 120 python tools/lane_prof.py $w > gpurun_out/phase_drain_$w.json
done
