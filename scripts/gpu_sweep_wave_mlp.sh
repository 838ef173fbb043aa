# Which MLP rollout kernel is fastest at which batch size (humanoid MLP, config #4 shape): M-split vs per-wave NS=1/2
set -o pipefail
for s in 16 24 32 48; do
  bash scripts/ab_arms.sh mw$s "--workload humanoid_mlp --solves $s --steps 20" -,MPPI_FC_WAVE=0 -,MPPI_FC_WAVE=1 -,MPPI_FC_WAVE=2 || exit 1
done
