#!/bin/bash
# Round-4 GPU session 3: the new parity tests (sample subsets at full size, split bf16, chained solves with the
# overlapped noise generator), the overlap A/B, the split-bf16 config #4 line, then session 2's diagnostic A/B
set -u
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
g=scripts/gpu_check.sh
L=humanoid_mppi-rl_amd/lib
mkdir -p gpurun_out/s3
bash $g s3/tests_new 600 python -u -m pytest tests/test_gpu_subsets.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py -m gpu -v --timeout 300 --timeout-method thread -k "subset or split or config4_full_size or humanoid_v1_cost or chained or graph_stream or bench" &&
bash $g s3/ab_ovl64 600 bash scripts/ab_arms.sh o64 "--workload humanoid_ca --steps 30" -,MPPI_GEN_OVERLAP=0 -,MPPI_GEN_OVERLAP=1 -,MPPI_GEN_OVERLAP=0 -,MPPI_GEN_OVERLAP=1 &&
bash $g s3/ab_ovl8 600 bash scripts/ab_arms.sh o8 "--workload humanoid_ca --global-solves 8 --steps 50" -,MPPI_GEN_OVERLAP=0 -,MPPI_GEN_OVERLAP=1 -,MPPI_GEN_OVERLAP=0 -,MPPI_GEN_OVERLAP=1 &&
bash $g s3/ab_ovl3 600 bash scripts/ab_arms.sh o3 "--workload quad_mlp --steps 50" -,MPPI_GEN_OVERLAP=0 -,MPPI_GEN_OVERLAP=1 &&
bash $g s3/ab_ovl2 600 bash scripts/ab_arms.sh o2 "--workload cartpole --steps 50" -,MPPI_GEN_OVERLAP=0 -,MPPI_GEN_OVERLAP=1 &&
bash $g s3/ab_ovlm 600 bash scripts/ab_arms.sh om "--workload humanoid_mlp --steps 30" -,MPPI_GEN_OVERLAP=0 -,MPPI_GEN_OVERLAP=1 &&
bash $g s3/bench_x3 300 python3 -u bench.py --precision bf16x3 --steps 10 --warmup 2 --no-cpu-baseline --no-traffic --no-kernel-trace &&
bash $g s3/ab_fo8 600 bash scripts/ab_arms.sh fo8 "--workload humanoid_ca --global-solves 8 --steps 50" - $L/libmppi_hip_fo.so - $L/libmppi_hip_fo.so &&
bash $g s3/ab_fo5 600 bash scripts/ab_arms.sh fo5 "--workload humanoid_ca_stream --steps 4 --warmup 1" - $L/libmppi_hip_fo.so &&
bash $g s3/ab_fo3 600 bash scripts/ab_arms.sh fo3 "--workload quad_mlp --steps 50" - $L/libmppi_hip_fo.so
