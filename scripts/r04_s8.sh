#!/bin/bash
# Round-4 GPU session 8: U + eps prefetch distance PD in registers (2 shipped; 3 variant) against the one-step
# prefetch base library; tests first
set -u
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
g=scripts/gpu_check.sh
L=humanoid_mppi-rl_amd/lib
B=$L/libmppi_hip_base.so
mkdir -p gpurun_out/s8
bash $g s8/tests 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_subsets.py -m gpu -q -x --timeout 300 --timeout-method thread &&
bash $g s8/ab_8 600 bash scripts/ab_arms.sh r8 "--workload humanoid_ca --global-solves 8 --steps 50" $B - $L/libmppi_hip_pd3.so $B - $L/libmppi_hip_pd3.so &&
bash $g s8/ab_5 600 bash scripts/ab_arms.sh r5 "--workload humanoid_ca_stream --steps 4 --warmup 1" $B - $L/libmppi_hip_pd3.so &&
bash $g s8/ab_16 600 bash scripts/ab_arms.sh r16 "--workload humanoid_ca --global-solves 16 --steps 50" $B - $L/libmppi_hip_pd3.so &&
bash $g s8/ab_x3 600 bash scripts/ab_arms.sh rx3 "--workload humanoid_ca --precision bf16x3 --steps 20" $B - $B - &&
bash $g s8/ab_f32 600 bash scripts/ab_arms.sh rf32 "--workload humanoid_ca --precision fp32 --global-solves 8 --steps 30" $B - &&
bash $g s8/ab_q3 600 bash scripts/ab_arms.sh rq3 "--workload quad_mlp --steps 50" $B -
