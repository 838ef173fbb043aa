set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/gpu_suite.log 2>&1
rc=$?; tail -5 gpurun_out/gpu_suite.log; exit $rc
