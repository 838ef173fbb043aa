#!/bin/bash
# split-bf16 per-wave kernel: its test and the x3 parity tests, then the 64-solve x3 bench A/B
set -u
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
g=scripts/gpu_check.sh
mkdir -p gpurun_out/s16
bash $g s16/tests 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_subsets.py tests/test_gpu_parity.py -m gpu -q -x -k "split_bf16 or x3 or 2]" --timeout 300 --timeout-method thread &&
bash $g s16/ab_x3 600 bash scripts/ab_arms.sh x3w "--workload humanoid_ca --precision bf16x3 --steps 20" -,MPPI_X3_WAVE=0 - -,MPPI_X3_WAVE=0 -
