set -o pipefail
L=humanoid_mppi-rl_amd/lib
bash scripts/ab_arms.sh td64 "--workload humanoid_ca --steps 30" - $L/libmppi_hip_tasc.so - $L/libmppi_hip_tasc.so &&
bash scripts/ab_arms.sh tdm64 "--workload humanoid_mlp --steps 30" - $L/libmppi_hip_tasc.so - $L/libmppi_hip_tasc.so &&
bash scripts/ab_arms.sh td8 "--workload humanoid_ca --solves 8 --steps 50" - $L/libmppi_hip_tasc.so &&
bash scripts/ab_arms.sh td5 "--workload humanoid_ca_stream --steps 3" - $L/libmppi_hip_tasc.so &&
bash scripts/gpu_suite.sh
