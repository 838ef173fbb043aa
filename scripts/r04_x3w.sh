#!/bin/bash
# split-bf16 per-wave kernel with the LDS fragment ring (7 deep; 4 and 14 as variants): tests, A/B
set -u
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
g=scripts/gpu_check.sh
L=humanoid_mppi-rl_amd/lib
mkdir -p gpurun_out/s17
bash $g s17/tests 600 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -q -x -k "split_bf16 or 2]" --timeout 300 --timeout-method thread &&
bash $g s17/ab_ring 600 bash scripts/ab_arms.sh x3r "--workload humanoid_ca --precision bf16x3 --steps 20" - $L/libmppi_hip_xr4.so $L/libmppi_hip_xr14.so -,MPPI_X3_WAVE=0 - $L/libmppi_hip_xr4.so $L/libmppi_hip_xr14.so
