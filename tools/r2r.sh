set -o pipefail
R=$(pwd)
mkdir -p gpurun_out/r2r
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r2r/tests.log 2>&1; echo "tests rc=$?"
tail -2 gpurun_out/r2r/tests.log
for D in 0 1; do
for W in c2 c3; do
ENET_RC_DEC4=$D timeout -k 10 300 python3 bench.py --no-cpu --no-pcie --no-crc --no-dgram --no-rccl --workload $W --steps 10 > gpurun_out/r2r/bench_${W}_d$D.log 2>&1; echo "bench $W dec4=$D rc=$?"
python3 -c "import json; d=json.loads(open('gpurun_out/r2r/bench_${W}_d$D.log').read().strip().splitlines()[-1]); print({k: d.get(k) for k in ('value','pipelined_GiBps','sequential_GiBps','compress_GiBps','decompress_GiBps','bit_exact_roundtrip')})"
done
done
