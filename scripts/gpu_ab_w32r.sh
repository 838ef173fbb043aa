set -o pipefail
L=humanoid_mppi-rl_amd/lib
bash scripts/ab_arms.sh w32r "--workload humanoid_ca --steps 30" - $L/libmppi_hip_r8.so $L/libmppi_hip_late.so - $L/libmppi_hip_r8.so $L/libmppi_hip_late.so
