#!/bin/bash
# Round-4 GPU session 12: block-diagonal layer 0 form 2 (108 MFMAs per wave-step; default) in fc_wave32_kernel and in
# the 16x16 fc_wave_kernel -- the GPU suite, then A/B against form 1 (112) and the dense layer 0 (124): headline 64
# solves (wave32) and 32 solves (the N = 2 strong shard: fc_wave_kernel NS = 1)
set -u
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
g=scripts/gpu_check.sh
mkdir -p gpurun_out/s12
bash $g s12/tests 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread &&
bash $g s12/ab_bd2 900 bash scripts/ab_arms.sh bd2 "--workload humanoid_ca --steps 30" -,MPPI_W32_BD=0 -,MPPI_W32_BD=1 - -,MPPI_W32_BD=0 -,MPPI_W32_BD=1 - &&
bash $g s12/ab_bd16 900 bash scripts/ab_arms.sh bd16 "--workload humanoid_ca --global-solves 32 --steps 40" -,MPPI_W32_BD=0 - -,MPPI_W32_BD=0 -
