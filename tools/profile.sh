#!/bin/bash
# Kernel-trace + PMC profile of bench.py on the GPU box (run under gpurun).
# usage: tools/profile.sh TAG [bench args...]
# Separate passes per counter group (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --no-cpu --no-pcie --no-dgram --no-configs --no-multi"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- $B "$@" > $OUT/bench_kt.log 2>&1
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVE_CYCLES" \
           "SQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" \
           "GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INST_CYCLES_SALU SQ_INST_CYCLES_VMEM_RD" \
           "TCC_EA0_RDREQ TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B" \
           "TCC_EA0_WRREQ TCC_EA0_WRREQ_64B" \
           "SQ_WAVES SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_IFETCH"; do
  i=$((i+1))
  echo "pmc pass $((i)) $grp"
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc$i -o run -- $B --steps 1 --warmup 0 "$@" > $OUT/bench_pmc$i.log 2>&1 || echo "pmc group $i failed: $grp" >> $OUT/errors.txt
done
echo done
