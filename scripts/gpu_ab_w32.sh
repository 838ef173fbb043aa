set -o pipefail
bash scripts/ab_arms.sh w32b "--workload humanoid_ca --steps 30" -,MPPI_FC_WAVE=2 -,MPPI_FC_WAVE=3 -,MPPI_FC_WAVE=2 -,MPPI_FC_WAVE=3 -,MPPI_FC_WAVE=2 -,MPPI_FC_WAVE=3
