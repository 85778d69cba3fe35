set -o pipefail
R=$(pwd)
mkdir -p gpurun_out/r2q
export ENET_RC_DEC4=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r2q/tests.log 2>&1; echo "tests rc=$?"
tail -2 gpurun_out/r2q/tests.log
timeout -k 10 200 python3 tools/dec4_check.py c2 c3
PMC_TAG=r2q/pmc bash tools/pmc_dec4.sh 2>&1 | grep -E "VALU|SALU|WAVE_CYCLES|WAIT_ANY|ACTIVE_INST_ANY|RDREQ_sum|WRREQ_sum"
