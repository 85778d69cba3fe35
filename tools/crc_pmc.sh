#!/bin/bash
# PMC passes over tools/crc_time.py (rc_crc32_batch on C2 and C4) -> gpurun_out/crc_pmc/p*
cd "$(dirname "$0")/.." && export TMPDIR=/tmp
O=gpurun_out/crc_pmc; mkdir -p $O
timeout -k 10 120 rocprofv3 --kernel-include-regex rc_crc32 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD -d $O/p1 -o p1 --output-format csv -- python tools/crc_time.py > $O/p1.log 2>&1 &&
timeout -k 10 120 rocprofv3 --kernel-include-regex rc_crc32 --pmc SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum -d $O/p2 -o p2 --output-format csv -- python tools/crc_time.py > $O/p2.log 2>&1 &&
timeout -k 10 120 rocprofv3 --kernel-include-regex rc_crc32 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python tools/crc_time.py > $O/kt.log 2>&1
