# PMC instruction mix and wait split of the bucket-history decoder (C2)
set -o pipefail
R=$(pwd)
D=gpurun_out/${PMC_TAG:-pmc_dec4}
mkdir -p $D
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --no-cpu --no-pcie --no-crc --no-dgram --no-rccl --no-configs --no-multi --steps 1 --warmup 0"
K=${PMC_KERNEL:-rc_decompress_dec4}
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVE_CYCLES --kernel-include-regex "$K" --output-format csv -d $R/$D/p1 -o run -- $B > $R/$D/p1.log 2>&1; echo "p1 rc=$?"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS --kernel-include-regex "$K" --output-format csv -d $R/$D/p2 -o run -- $B > $R/$D/p2.log 2>&1; echo "p2 rc=$?"
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --kernel-include-regex "$K" --output-format csv -d $R/$D/p3 -o run -- $B > $R/$D/p3.log 2>&1; echo "p3 rc=$?"
for d in p1 p2 p3; do f=$(find $R/$D/$d -name "*counter_collection.csv" | head -1); echo "== $d"; python3 -c "
import csv,sys,collections
rows=list(csv.DictReader(open('$f')))
agg=collections.defaultdict(float)
for r in rows: agg[(r['Kernel_Name'],r['Counter_Name'])]+=float(r['Counter_Value'])
for k,v in sorted(agg.items()): print(k[0][:24],k[1],v)
"; done
