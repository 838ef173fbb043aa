set -o pipefail
L=humanoid_mppi-rl_amd/lib
bash scripts/ab_arms.sh rd64 "--workload humanoid_ca --steps 30" - $L/libmppi_hip_ru8.so $L/libmppi_hip_ru2.so $L/libmppi_hip_blk512.so $L/libmppi_hip_blk1024.so $L/libmppi_hip_t512.so - $L/libmppi_hip_ru8.so $L/libmppi_hip_ru2.so $L/libmppi_hip_blk512.so $L/libmppi_hip_blk1024.so $L/libmppi_hip_t512.so
