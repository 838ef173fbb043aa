set -o pipefail
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_fullsize.py -k "wave_kernel" > gpurun_out/wave32_tests.log 2>&1
rc=$?; tail -4 gpurun_out/wave32_tests.log; [ $rc -ne 0 ] && exit $rc
bash scripts/ab_arms.sh w32 "--workload humanoid_ca --steps 30" -,MPPI_FC_WAVE=2 -,MPPI_FC_WAVE=3 -,MPPI_FC_WAVE=2 -,MPPI_FC_WAVE=3
