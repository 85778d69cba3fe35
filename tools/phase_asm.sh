#!/bin/bash
# Static look at the v3 lane kernels per profiling phase: compiles rc_lane3.hip
# with -DRC_PROFILE and prints, for the kernel $1 (compress|decompress), the
# instruction count between consecutive s_memtime stamps (rare paths included).
cd "$(dirname "$0")/../enet_amd/csrc"
K=${1:-compress}
EXTRA=${2:-}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../include -I. -DRC_PROFILE $EXTRA --cuda-device-only -S rc_lane3.hip -o /tmp/l3p.s 2>/dev/null
awk "/^rc_${K}_lane3:/,/s_endpgm/" /tmp/l3p.s > /tmp/kp.s
grep -n "s_memtime" /tmp/kp.s | cut -d: -f1 > /tmp/marks
prev=""
while read m; do
  if [ -n "$prev" ]; then
    n=$(sed -n "${prev},${m}p" /tmp/kp.s | grep -c "^\s*[sv]_\|^\s*ds_\|^\s*global_\|^\s*buffer_")
    sp=$(sed -n "${prev},${m}p" /tmp/kp.s | grep -c "v_writelane\|v_readlane\|accvgpr")
    echo "lines $prev-$m: $n instructions ($sp spill moves)"
  fi
  prev=$m
done < /tmp/marks
