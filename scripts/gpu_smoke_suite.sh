set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; tail -2 gpurun_out/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/ > gpurun_out/gpu_suite.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_suite.log; [ $rc -ne 0 ] && exit $rc
bash scripts/gpu_sweep_wave_mlp.sh
