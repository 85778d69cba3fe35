# PMC instruction mix of the two-pass encoder kernels (bench C2, one compress pass)
set -o pipefail
R=$(pwd)
T=${1:-x}
mkdir -p gpurun_out/pmc_$T
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --no-cpu --no-pcie --no-crc --no-dgram --no-rccl --no-configs --no-multi --steps 1 --warmup 0"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVE_CYCLES --kernel-include-regex "rc_enc2" --output-format csv -d $R/gpurun_out/pmc_$T/p1 -o run -- $B > $R/gpurun_out/pmc_$T/p1.log 2>&1; echo "p1 rc=$?"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS --kernel-include-regex "rc_enc2" --output-format csv -d $R/gpurun_out/pmc_$T/p2 -o run -- $B > $R/gpurun_out/pmc_$T/p2.log 2>&1; echo "p2 rc=$?"
for d in p1 p2; do f=$(find $R/gpurun_out/pmc_$T/$d -name "*counter_collection.csv" | head -1); echo "== $d"; python3 -c "
import csv,collections
rows=list(csv.DictReader(open('$f')))
agg=collections.defaultdict(float); disp=collections.defaultdict(set)
for r in rows:
    agg[(r['Kernel_Name'],r['Counter_Name'])]+=float(r['Counter_Value']); disp[r['Kernel_Name']].add(r['Dispatch_Id'])
for k,v in sorted(agg.items()): print(k[0][:16],k[1],v/len(disp[k[0]]))
"; done
