set -o pipefail
L=humanoid_mppi-rl_amd/lib
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fullsize.py -k "wave or config4" > gpurun_out/wave_tests5.log 2>&1
rc=$?; tail -3 gpurun_out/wave_tests5.log; [ $rc -ne 0 ] && exit $rc
bash scripts/ab_arms.sh w64e "--workload humanoid_ca --steps 30" - $L/libmppi_hip_prev.so - $L/libmppi_hip_prev.so
