set -o pipefail
L=humanoid_mppi-rl_amd/lib
bash scripts/ab_arms.sh rnt "--workload humanoid_ca --steps 30" - $L/libmppi_hip_nt.so - $L/libmppi_hip_nt.so &&
bash scripts/ab_arms.sh rnt8 "--workload humanoid_ca --solves 8 --steps 40" - $L/libmppi_hip_nt.so - $L/libmppi_hip_nt.so
