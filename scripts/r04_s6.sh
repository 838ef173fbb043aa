#!/bin/bash
# Round-4 GPU session 6: two-step control prefetch in the M-split fc body (tests, A/B against one-step prefetch)
set -u
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
g=scripts/gpu_check.sh
B=humanoid_mppi-rl_amd/lib/libmppi_hip_base.so
mkdir -p gpurun_out/s6
bash $g s6/tests 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_subsets.py -m gpu -q -x --timeout 300 --timeout-method thread &&
bash $g s6/ab_pf8 600 bash scripts/ab_arms.sh p8 "--workload humanoid_ca --global-solves 8 --steps 50" $B - $B - &&
bash $g s6/ab_pf5 600 bash scripts/ab_arms.sh p5 "--workload humanoid_ca_stream --steps 4 --warmup 1" $B - $B - &&
bash $g s6/ab_pf16 600 bash scripts/ab_arms.sh p16 "--workload humanoid_ca --global-solves 16 --steps 50" $B - &&
bash $g s6/ab_pfx3 600 bash scripts/ab_arms.sh px3 "--workload humanoid_ca --precision bf16x3 --steps 20" $B - &&
bash $g s6/ab_pff32 600 bash scripts/ab_arms.sh pf32 "--workload humanoid_ca --precision fp32 --global-solves 8 --steps 30" $B -
