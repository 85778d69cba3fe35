#!/bin/bash
# UTCL1 (TLB) counters for the lane kernels: two builds loaded in one process (tools/abx.py)
cd "$(dirname "$0")/.."
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_STALL_INFLIGHT_MAX_sum -d $R/gpurun_out/tlb1 -o p -- python3 $R/tools/abx.py A B --rounds 3 > $R/gpurun_out/tlb1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_UTCL1_THRASHING_STALL_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum -d $R/gpurun_out/tlb2 -o p -- python3 $R/tools/abx.py A B --rounds 3 > $R/gpurun_out/tlb2.log 2>&1 || exit 1
