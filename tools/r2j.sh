set -o pipefail
R=$(pwd)
mkdir -p gpurun_out/r2j
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 240 --timeout-method thread -k "lane3" > gpurun_out/r2j/tests.log 2>&1; echo "tests rc=$?"
tail -3 gpurun_out/r2j/tests.log
timeout -k 10 200 python3 tools/enc2_prof.py > gpurun_out/r2j/prof.log 2>&1; echo "prof rc=$?"; cat gpurun_out/r2j/prof.log | grep -v amdgpu.ids
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r2j/kt -o run -- python3 $R/bench.py --no-cpu --no-pcie --no-crc --no-dgram --no-rccl --steps 3 --warmup 1 > $R/gpurun_out/r2j/bench.log 2>&1; echo "rc=$?"
find $R/gpurun_out/r2j/kt -name "*kernel_stats.csv" | head -1 | xargs cat | cut -d, -f1-4 | head -4
grep -o '"bit_exact_roundtrip": [a-z]*' $R/gpurun_out/r2j/bench.log
