#!/bin/bash
# Builds libenet_rc_amd_<name>.so variants of the lane kernels (rc_lane3.hip) with -D flags (diagnostic).
# usage: tools/lane3_variants.sh name "-DFLAG=.. ..." [name "flags"]...
set -e
cd "$(dirname "$0")/../enet_amd/csrc"
make ARCH=gfx950 > /dev/null
B=build; O=../lib
OBJS="$B/rc_kernels.o $B/rc_route.o $B/rc_enc2.o $B/rc_enc2_wide.o $B/rc_dec6.o $B/rc_crc32.o $B/rc_dgram.o $B/rc_pack.o $B/rc_multi_plan.o $B/rc_io.o $B/rc_multi.o $B/rc_host.o"
while [ $# -gt 1 ]; do
  n=$1; f=$2; shift 2
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I../../include -I. -Wall -Wno-unused-function ${LV_SCHED--mllvm -amdgpu-sched-strategy=iterative-ilp} $f -c rc_lane3.hip -o $B/rc_lane3_$n.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $O/libenet_rc_amd_$n.so $OBJS $B/rc_lane3_$n.o -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,/opt/rocm/lib
  echo built $n
done
