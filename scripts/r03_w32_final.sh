#!/bin/bash
# After making fc_wave32_kernel the default for >= 12 tiles per CU: GPU suite, config #4 bench lines, kernel stats, PMC.
set -u
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
g=scripts/gpu_check.sh
bash $g w32f/gpu_tests 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread &&
bash $g w32f/bench_humanoid_ca 400 python3 -u bench.py &&
bash $g w32f/bench_humanoid_ca_global64 400 python3 -u bench.py --global-solves 64 &&
bash $g w32f/bench_humanoid_ca_48solves 400 python3 -u bench.py --solves 48 &&
bash $g w32f/ab 400 bash scripts/ab_arms.sh w32c "--workload humanoid_ca --steps 30" -,MPPI_FC_WAVE=2 - -,MPPI_FC_WAVE=2 - &&
bash $g w32f/prof_humanoid_ca 300 rocprofv3 --kernel-trace --stats -d gpurun_out/w32f/prof_humanoid_ca -o run --output-format csv -- python3 bench.py --steps 10 --warmup 1 --no-cpu-baseline --no-traffic --no-kernel-trace &&
bash $g w32f/pmc 200 bash scripts/pmc_mfma.sh ca_bf16_wave32 --workload humanoid_ca
