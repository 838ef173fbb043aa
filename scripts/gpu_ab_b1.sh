set -o pipefail
L=humanoid_mppi-rl_amd/lib
MPPI_HIP_LIB=$L/libmppi_hip_b1l4.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fullsize.py -m gpu -k "wave_kernel_agrees or humanoid_v1" > gpurun_out/ab_b1_tests.log 2>&1 && tail -2 gpurun_out/ab_b1_tests.log &&
bash scripts/ab_arms.sh b1 "--workload humanoid_ca --steps 30" - $L/libmppi_hip_b1l4.so $L/libmppi_hip_b1l2.so - $L/libmppi_hip_b1l4.so $L/libmppi_hip_b1l2.so
