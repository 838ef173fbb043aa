set -o pipefail
bash scripts/ab_arms.sh s8 "--workload humanoid_ca --solves 8 --steps 40" -,MPPI_FC_WAVE=0 -,MPPI_FC_WAVE=1 -,MPPI_FC_WAVE=2 || exit 1
bash scripts/ab_arms.sh c5 "--workload humanoid_ca_stream --steps 3" -,MPPI_FC_WAVE=0 -,MPPI_FC_WAVE=1 || exit 1
bash scripts/ab_arms.sh s48 "--workload humanoid_ca --solves 48 --steps 30" -,MPPI_FC_WAVE=0 -,MPPI_FC_WAVE=2 -,MPPI_FC_WAVE=1 || exit 1
bash scripts/pmc_mfma.sh wave_ca64_ring4 --workload humanoid_ca
