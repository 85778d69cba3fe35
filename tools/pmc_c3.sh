#!/bin/bash
# PMC passes over the C3 bench (rc_decompress_lane3 and the wide encoder) -> gpurun_out/pmc_c3/p*
cd "$(dirname "$0")/.." && export TMPDIR=/tmp
O=gpurun_out/pmc_c3; mkdir -p $O
B="python bench.py --workload c3 --no-cpu --no-pcie --no-crc --no-dgram --no-configs --no-multi --steps 2 --warmup 1"
timeout -k 10 180 rocprofv3 --kernel-include-regex "rc_" --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_INST_ANY -d $O/p1 -o p1 --output-format csv -- $B > $O/p1.log 2>&1 &&
timeout -k 10 180 rocprofv3 --kernel-include-regex "rc_" --pmc SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_WAIT_ANY SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d $O/p2 -o p2 --output-format csv -- $B > $O/p2.log 2>&1
