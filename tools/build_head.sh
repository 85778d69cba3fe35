#!/bin/bash
# Builds the library of a git revision (default HEAD) as enet_amd/lib/libenet_rc_amd_<name>.so,
# for A/B runs against the working tree (diagnostic).  usage: tools/build_head.sh [name] [rev]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
N=${1:-head}; REV=${2:-HEAD}
T=/tmp/rc_build_$N
rm -rf $T && mkdir -p $T
git -C $R archive $REV enet_amd/csrc include | tar -x -C $T
make -C $T/enet_amd/csrc -j8 > /dev/null
cp $T/enet_amd/lib/libenet_rc_amd.so $R/enet_amd/lib/libenet_rc_amd_$N.so
echo built $N from $REV
