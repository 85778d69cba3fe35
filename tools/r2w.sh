set -o pipefail
R=$(pwd)
mkdir -p gpurun_out/r2w
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r2w/tests.log 2>&1; echo "tests rc=$?"
tail -2 gpurun_out/r2w/tests.log
timeout -k 10 300 python3 bench.py --no-cpu --no-pcie --no-crc --no-dgram --no-rccl > gpurun_out/r2w/bench_c2.log 2>&1; echo "bench rc=$?"
python3 -c "import json; d=json.loads(open('gpurun_out/r2w/bench_c2.log').read().strip().splitlines()[-1]); print({k: d.get(k) for k in ('value','compress_GiBps','decompress_GiBps','bit_exact_roundtrip')})"
PMC_TAG=r2w/pmc PMC_KERNEL=rc_enc2 bash tools/pmc_dec4.sh 2>&1 | grep -E "WAVE_CYCLES|RDREQ_sum|WRREQ"
