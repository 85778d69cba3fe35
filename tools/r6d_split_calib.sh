set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r6d
bash $R/tools/calib.sh r6d/calib > $R/gpurun_out/r6d/calib_run.log 2>&1
ENET_RC_LIB=$R/enet_amd/lib/libenet_rc_amd_hcount.so timeout -k 10 120 python3 $R/tools/dec6_split.py > $R/gpurun_out/r6d/split.json 2>$R/gpurun_out/r6d/split.err
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES --output-format csv -d $R/gpurun_out/r6d/pmc_sq -o run -- python3 $R/bench.py --no-cpu --no-pcie --no-dgram --no-configs --no-multi --no-crc --steps 1 --warmup 0 > $R/gpurun_out/r6d/pmc_sq.log 2>&1
echo ok
