#!/bin/bash
# Kernel-trace + PMC profile of bench.py on the GPU box (run under gpurun).
# usage: tools/profile.sh TAG [bench args...]
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- \
    python3 $R/bench.py --no-cpu --no-pcie "$@" > $OUT/bench_kt.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    --output-format csv -d $OUT/pmc1 -o run -- python3 $R/bench.py --no-cpu --no-pcie --steps 1 --warmup 0 "$@" > $OUT/bench_pmc1.log 2>&1
echo done
