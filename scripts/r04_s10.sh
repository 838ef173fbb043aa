#!/bin/bash
# Round-4 GPU session 10: wave kernel tests after the fragment-sequence refactor; timing-only block-diagonal layer-0
# diagnostics of fc_wave32_kernel (bd1: 112 MFMAs per wave-step, bd2: 108) against the shipped 124, headline 64 solves
set -u
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
g=scripts/gpu_check.sh
L=humanoid_mppi-rl_amd/lib
mkdir -p gpurun_out/s10
bash $g s10/tests 600 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -q -x -k "wave or config4" --timeout 300 --timeout-method thread &&
bash $g s10/ab_bd 900 bash scripts/ab_arms.sh bd "--workload humanoid_ca --steps 30" - $L/libmppi_hip_bd1.so $L/libmppi_hip_bd2.so - $L/libmppi_hip_bd1.so $L/libmppi_hip_bd2.so
