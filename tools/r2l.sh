set -o pipefail
R=$(pwd)
mkdir -p gpurun_out/r2l
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_dgram.py tests/test_integration.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r2l/tests.log 2>&1; echo "tests rc=$?"
tail -3 gpurun_out/r2l/tests.log
for W in c2 c3 c4; do
P=""; [ $W = c4 ] && P="--packets 1048576 --steps 2"
timeout -k 10 300 python3 bench.py --no-cpu --no-pcie --no-crc --no-dgram --no-rccl --workload $W $P > gpurun_out/r2l/bench_$W.log 2>&1; echo "bench $W rc=$?"
python3 -c "import json; d=json.loads(open('gpurun_out/r2l/bench_$W.log').read().strip().splitlines()[-1]); print({k: d.get(k) for k in ('value','compress_GiBps','decompress_GiBps','bit_exact_roundtrip')})"
done
