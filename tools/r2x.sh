set -o pipefail
R=$(pwd)
mkdir -p gpurun_out/r2x
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r2x/tests.log 2>&1; echo "tests rc=$?"
tail -2 gpurun_out/r2x/tests.log
for W in c2 c3; do
timeout -k 10 300 python3 bench.py --no-cpu --no-pcie --no-crc --no-dgram --no-rccl --workload $W --steps 10 > gpurun_out/r2x/bench_$W.log 2>&1; echo "bench $W rc=$?"
python3 -c "import json; d=json.loads(open('gpurun_out/r2x/bench_$W.log').read().strip().splitlines()[-1]); print({k: d.get(k) for k in ('value','compress_GiBps','decompress_GiBps','bit_exact_roundtrip')})"
done
ENET_RC_DEC4=0 timeout -k 10 300 python3 bench.py --no-cpu --no-pcie --no-crc --no-dgram --no-rccl --steps 10 > gpurun_out/r2x/bench_c2_lane3.log 2>&1; echo "bench lane3 rc=$?"
python3 -c "import json; d=json.loads(open('gpurun_out/r2x/bench_c2_lane3.log').read().strip().splitlines()[-1]); print({k: d.get(k) for k in ('value','compress_GiBps','decompress_GiBps','bit_exact_roundtrip')})"
