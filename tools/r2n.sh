set -o pipefail
R=$(pwd)
mkdir -p gpurun_out/r2n
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r2n/tests.log 2>&1; echo "tests rc=$?"
tail -3 gpurun_out/r2n/tests.log
for W in c2 c3 c4; do
P=""; [ $W = c4 ] && P="--packets 1048576 --steps 2"
timeout -k 10 300 python3 bench.py --no-cpu --no-pcie --no-crc --no-dgram --no-rccl --workload $W $P > gpurun_out/r2n/bench_$W.log 2>&1; echo "bench $W rc=$?"
python3 -c "import json; d=json.loads(open('gpurun_out/r2n/bench_$W.log').read().strip().splitlines()[-1]); print({k: d.get(k) for k in ('value','compress_GiBps','decompress_GiBps','bit_exact_roundtrip')})"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r2n/kt -o run -- python3 $R/bench.py --no-cpu --no-pcie --no-crc --no-dgram --no-rccl --steps 3 --warmup 1 > $R/gpurun_out/r2n/bench_prof.log 2>&1; echo "prof rc=$?"
find $R/gpurun_out/r2n/kt -name "*kernel_stats.csv" | head -1 | xargs cat | cut -d, -f1-4 | head -8
