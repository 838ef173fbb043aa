#!/bin/bash
# Round-4 GPU session 9: prefetch distance PD (2 shipped; 1, 3 variants; PD 1 carries sums as the base) against the one-step
# prefetch base library; tests first
set -u
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
g=scripts/gpu_check.sh
L=humanoid_mppi-rl_amd/lib
B=$L/libmppi_hip_base.so
mkdir -p gpurun_out/s9
bash $g s9/tests 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_subsets.py -m gpu -q -x --timeout 300 --timeout-method thread &&
bash $g s9/ab_8 600 bash scripts/ab_arms.sh t8 "--workload humanoid_ca --global-solves 8 --steps 50" $B - $L/libmppi_hip_pd3.so $L/libmppi_hip_pd1.so $B - $L/libmppi_hip_pd3.so $L/libmppi_hip_pd1.so &&
bash $g s9/ab_5 600 bash scripts/ab_arms.sh t5 "--workload humanoid_ca_stream --steps 4 --warmup 1" $B - $L/libmppi_hip_pd3.so &&
bash $g s9/ab_16 600 bash scripts/ab_arms.sh t16 "--workload humanoid_ca --global-solves 16 --steps 50" $B - $L/libmppi_hip_pd3.so &&
bash $g s9/ab_x3 600 bash scripts/ab_arms.sh tx3 "--workload humanoid_ca --precision bf16x3 --steps 20" $B - $B - &&
bash $g s9/ab_f32 600 bash scripts/ab_arms.sh tf32 "--workload humanoid_ca --precision fp32 --global-solves 8 --steps 30" $B - &&
bash $g s9/ab_q3 600 bash scripts/ab_arms.sh tq3 "--workload quad_mlp --steps 50" $B -
