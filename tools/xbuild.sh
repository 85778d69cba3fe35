#!/bin/bash
# Experiment build (diagnostic): libenet_rc_amd_<NAME>.so with rc_enc2.hip and
# rc_dec4.hip compiled with extra flags.  usage: tools/xbuild.sh NAME "-DFOO -DBAR"
set -e
cd "$(dirname "$0")/../enet_amd/csrc"
make ARCH=gfx950 >/dev/null
F="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -I../../include -I. -Wall -Wno-unused-function $2"
/opt/rocm/bin/hipcc $F -c rc_enc2.hip -o build/rc_enc2_$1.o
/opt/rocm/bin/hipcc $F -c rc_dec4.hip -o build/rc_dec4_$1.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../lib/libenet_rc_amd_$1.so build/rc_kernels.o build/rc_lane.o \
  build/rc_lane3.o build/rc_enc2_$1.o build/rc_dec4_$1.o build/rc_crc32.o build/rc_dgram.o build/rc_pack.o build/rc_io.o \
  build/rc_host.o -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,/opt/rocm/lib
