set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_fullsize.py -k "wave" > gpurun_out/wave_tests.log 2>&1
rc=$?; tail -30 gpurun_out/wave_tests.log; [ $rc -ne 0 ] && exit $rc
bash scripts/ab_arms.sh w64 "--workload humanoid_ca --steps 30" -,MPPI_FC_WAVE=0 -,MPPI_FC_WAVE=2 -,MPPI_FC_WAVE=1 -,MPPI_FC_WAVE=0 -,MPPI_FC_WAVE=2
