#!/bin/bash
# Round-4 GPU session 2: where the few-tiles-per-CU M-split rollout's time goes, measured with timing-only diagnostic
# builds (results wrong, timing representative): each drops one barrier, the cost-ring flush or the control loads.
set -u
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
g=scripts/gpu_check.sh
L=humanoid_mppi-rl_amd/lib
arms="- $L/libmppi_hip_d_nolnbar.so $L/libmppi_hip_d_nobar2.so $L/libmppi_hip_d_nobar3.so $L/libmppi_hip_d_nobar4.so $L/libmppi_hip_d_nocost.so $L/libmppi_hip_d_noctrl.so -"
mkdir -p gpurun_out/s2
bash $g s2/diag8 900 bash scripts/ab_arms.sh d8 "--workload humanoid_ca --global-solves 8 --steps 50" $arms &&
bash $g s2/diag5 900 bash scripts/ab_arms.sh d5 "--workload humanoid_ca_stream --steps 4 --warmup 1" $arms &&
bash $g s2/diag3 900 bash scripts/ab_arms.sh d3 "--workload quad_mlp --steps 50" $arms
