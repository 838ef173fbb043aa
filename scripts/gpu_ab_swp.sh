set -o pipefail
L=humanoid_mppi-rl_amd/lib
mkdir -p gpurun_out
timeout -k 10 120 ./tools/issue_probe > gpurun_out/issue_probe.txt 2>&1 && cat gpurun_out/issue_probe.txt &&
for v in swp swp2; do MPPI_HIP_LIB=$L/libmppi_hip_$v.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fullsize.py -m gpu -k "wave_kernel_agrees or humanoid_v1 or config4_64" > gpurun_out/ab_${v}_tests.log 2>&1 && tail -1 gpurun_out/ab_${v}_tests.log || exit 1; done &&
bash scripts/ab_arms.sh swp "--workload humanoid_ca --steps 30" - $L/libmppi_hip_swp.so $L/libmppi_hip_swp2.so - $L/libmppi_hip_swp.so $L/libmppi_hip_swp2.so
