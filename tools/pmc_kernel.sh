#!/bin/bash
# PMC passes for one kernel of the C2 bench (diagnostic): instruction mix, wait split,
# LDS, instruction cache.  usage: PMC_TAG=x PMC_KERNEL=regex [ENV=..] tools/pmc_kernel.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
D=$R/gpurun_out/${PMC_TAG:-pmc}
mkdir -p $D
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --workload ${PMC_WL:-c2} --no-cpu --no-pcie --no-crc --no-dgram --no-rccl --no-configs --no-multi --steps 1 --warmup 0"
K=${PMC_KERNEL:-rc_decompress_dec7}
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVE_CYCLES" \
           "SQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS" \
           "SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_IFETCH SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_SENDMSG" \
           "SQC_ICACHE_HITS SQC_ICACHE_MISSES" ; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $set --kernel-include-regex "$K" --output-format csv -d $D/pmc$i -o run -- $B > $D/p$i.log 2>&1; echo "pass $i rc=$?"
done
python3 $R/tools/pmc_summary.py $D > $D/summary.json
cat $D/summary.json
