set -o pipefail
L=humanoid_mppi-rl_amd/lib
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fullsize.py -k "wave" > gpurun_out/wave_tests4.log 2>&1
rc=$?; tail -3 gpurun_out/wave_tests4.log; [ $rc -ne 0 ] && exit $rc
bash scripts/ab_arms.sh w64d "--workload humanoid_ca --steps 30" - $L/libmppi_hip_r8m2.so $L/libmppi_hip_pk.so $L/libmppi_hip_r0.so $L/libmppi_hip_gram1.so - $L/libmppi_hip_r8m2.so $L/libmppi_hip_pk.so $L/libmppi_hip_r0.so $L/libmppi_hip_gram1.so
