#!/bin/bash
# Round-4 GPU session 11: fc_wave32_kernel with the block-diagonal layer 0 (w32_bd, default) -- the GPU suite, then
# the headline A/B against the dense form (MPPI_W32_BD=0 at load)
set -u
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
g=scripts/gpu_check.sh
mkdir -p gpurun_out/s11
bash $g s11/tests 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread &&
bash $g s11/ab_bd 900 bash scripts/ab_arms.sh bdx "--workload humanoid_ca --steps 30" -,MPPI_W32_BD=0 - -,MPPI_W32_BD=0 -
