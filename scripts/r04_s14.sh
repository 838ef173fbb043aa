#!/bin/bash
# Round-4 GPU session 14: the M-split CA kernel with the LayerNorm statistic from the Gram factor (variant library
# libmppi_hip_gram.so, -DMPPI_MSPLIT_GRAM=1): parity of the CA tests on it, then A/B against the shipped library
set -u
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
g=scripts/gpu_check.sh
V=humanoid_mppi-rl_amd/lib/libmppi_hip_gram.so
mkdir -p gpurun_out/s14
env MPPI_HIP_LIB=$V bash $g s14/tests 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_subsets.py -m gpu -q -x -k "ca or humanoid or config4 or config5" --timeout 300 --timeout-method thread &&
bash $g s14/ab_8 600 bash scripts/ab_arms.sh g8 "--workload humanoid_ca --global-solves 8 --steps 50" - $V - $V &&
bash $g s14/ab_5 600 bash scripts/ab_arms.sh g5 "--workload humanoid_ca_stream --steps 4 --warmup 1" - $V - $V &&
bash $g s14/ab_16 600 bash scripts/ab_arms.sh g16 "--workload humanoid_ca --global-solves 16 --steps 50" - $V
