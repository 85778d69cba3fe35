set -o pipefail
R=$(pwd)
mkdir -p gpurun_out/r2m
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r2m/tests.log 2>&1; echo "tests rc=$?"
tail -3 gpurun_out/r2m/tests.log
timeout -k 10 300 python3 bench.py > gpurun_out/r2m/bench_full.log 2>&1; echo "bench rc=$?"
tail -c 3000 gpurun_out/r2m/bench_full.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r2m/kt -o run -- python3 $R/bench.py --no-cpu --no-pcie --no-crc --no-dgram --no-rccl --steps 3 --warmup 1 > $R/gpurun_out/r2m/bench_prof.log 2>&1; echo "prof rc=$?"
find $R/gpurun_out/r2m/kt -name "*kernel_stats.csv" | head -1 | xargs cat | cut -d, -f1-4 | head -12
