set -o pipefail
R=$(pwd)
mkdir -p gpurun_out/r2v
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r2v/tests.log 2>&1; echo "tests rc=$?"
tail -2 gpurun_out/r2v/tests.log
for W in c2 c3; do
timeout -k 10 300 python3 bench.py --no-cpu --no-pcie --no-crc --no-dgram --no-rccl --workload $W > gpurun_out/r2v/bench_$W.log 2>&1; echo "bench $W rc=$?"
python3 -c "import json; d=json.loads(open('gpurun_out/r2v/bench_$W.log').read().strip().splitlines()[-1]); print({k: d.get(k) for k in ('value','compress_GiBps','decompress_GiBps','bit_exact_roundtrip')})"
done
timeout -k 10 200 python3 tools/dec4_check.py c2
PMC_TAG=r2v/pmc bash tools/pmc_dec4.sh 2>&1 | grep -E "VALU|SALU|WAVE_CYCLES|WAIT_ANY|ACTIVE_INST_ANY|RDREQ|WRREQ"
