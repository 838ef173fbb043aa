#!/bin/bash
# Round-4 GPU session 4: split-bf16 with two sample tiles per wave (tests, A/B against one tile), then the few-tiles
# diagnostics (scripts/r04_s2.sh)
set -u
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
g=scripts/gpu_check.sh
mkdir -p gpurun_out/s4
bash $g s4/tests_x3 600 python -u -m pytest tests/test_gpu_subsets.py tests/test_gpu_fullsize.py -m gpu -v --timeout 300 --timeout-method thread -k "subset or split or config4_full_size or humanoid_v1_cost" &&
bash $g s4/ab_x3 600 bash scripts/ab_arms.sh x3 "--workload humanoid_ca --precision bf16x3 --steps 10 --warmup 2" -,MPPI_X3_TILES=1 -,MPPI_X3_TILES=2 -,MPPI_X3_TILES=1 -,MPPI_X3_TILES=2 &&
bash $g s4/ab_x3m 600 bash scripts/ab_arms.sh x3m "--workload humanoid_mlp --precision bf16x3 --steps 10 --warmup 2" -,MPPI_X3_TILES=1 -,MPPI_X3_TILES=2 &&
bash scripts/r04_s2.sh
