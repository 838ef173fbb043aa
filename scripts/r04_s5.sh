#!/bin/bash
# Round-4 GPU session 5: the LDS-DMA control path of the CA M-split kernel (tests, A/B against per-step loads)
set -u
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
g=scripts/gpu_check.sh
mkdir -p gpurun_out/s5
bash $g s5/tests 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_subsets.py -m gpu -q -x --timeout 300 --timeout-method thread &&
bash $g s5/ab_cdma8 600 bash scripts/ab_arms.sh c8 "--workload humanoid_ca --global-solves 8 --steps 50" -,MPPI_FC_CDMA=0 -,MPPI_FC_CDMA=1 -,MPPI_FC_CDMA=0 -,MPPI_FC_CDMA=1 &&
bash $g s5/ab_cdma5 600 bash scripts/ab_arms.sh c5 "--workload humanoid_ca_stream --steps 4 --warmup 1" -,MPPI_FC_CDMA=0 -,MPPI_FC_CDMA=1 -,MPPI_FC_CDMA=0 -,MPPI_FC_CDMA=1 &&
bash $g s5/ab_cdma16 600 bash scripts/ab_arms.sh c16 "--workload humanoid_ca --global-solves 16 --steps 50" -,MPPI_FC_CDMA=0 -,MPPI_FC_CDMA=1 &&
bash $g s5/ab_r8 600 bash scripts/ab_arms.sh r8 "--workload humanoid_ca --steps 30" - humanoid_mppi-rl_amd/lib/libmppi_hip_r8.so - humanoid_mppi-rl_amd/lib/libmppi_hip_r8.so
