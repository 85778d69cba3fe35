set -o pipefail
R=$(pwd)
mkdir -p gpurun_out/r2p
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r2p/tests.log 2>&1; echo "tests rc=$?"
tail -2 gpurun_out/r2p/tests.log
cd /tmp && export TMPDIR=/tmp
for L in 64 32; do
ENET_RC_ENC2_LANES=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r2p/kt$L -o run -- python3 $R/bench.py --no-cpu --no-pcie --no-crc --no-dgram --no-rccl --steps 3 --warmup 1 > $R/gpurun_out/r2p/bench$L.log 2>&1; echo "rc=$? L=$L"
find $R/gpurun_out/r2p/kt$L -name "*kernel_stats.csv" | head -1 | xargs cat | cut -d, -f1-4 | grep enc2
grep -o '"bit_exact_roundtrip": [a-z]*' $R/gpurun_out/r2p/bench$L.log
done
