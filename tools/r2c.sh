set -o pipefail
R=$(pwd)
mkdir -p gpurun_out/r2c
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r2c/kt -o run -- python3 $R/bench.py --no-cpu --no-pcie --no-crc --no-dgram --no-rccl --steps 3 --warmup 1 > $R/gpurun_out/r2c/bench.log 2>&1; echo "rc=$?"
find $R/gpurun_out/r2c/kt -name "*kernel_stats.csv" | head -1 | xargs cat | cut -d, -f1-8
