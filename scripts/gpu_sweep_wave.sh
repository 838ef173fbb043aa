# Which CA rollout kernel is fastest at which batch size (config #4 shape): M-split, layer-pipelined, per-wave NS=1/2
set -o pipefail
for s in 16 24 32 48 96 128; do
  bash scripts/ab_arms.sh sw$s "--workload humanoid_ca --solves $s --steps 20" -,MPPI_FC_WAVE=0,MPPI_FC_PIPE=0 -,MPPI_FC_WAVE=0,MPPI_FC_PIPE=1 -,MPPI_FC_WAVE=1 -,MPPI_FC_WAVE=2 || exit 1
done
