set -o pipefail
L=humanoid_mppi-rl_amd/lib
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fullsize.py -k "wave" > gpurun_out/wave_tests2.log 2>&1
rc=$?; tail -3 gpurun_out/wave_tests2.log; [ $rc -ne 0 ] && exit $rc
bash scripts/ab_arms.sh w64c "--workload humanoid_ca --steps 30" - $L/libmppi_hip_ring4.so $L/libmppi_hip_ring8.so $L/libmppi_hip_prio.so $L/libmppi_hip_stag1.so $L/libmppi_hip_gram1.so - $L/libmppi_hip_ring4.so $L/libmppi_hip_ring8.so $L/libmppi_hip_prio.so $L/libmppi_hip_stag1.so $L/libmppi_hip_gram1.so
