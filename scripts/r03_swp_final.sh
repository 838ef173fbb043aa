#!/bin/bash
# Closing evidence after the software-pipelined wave32 conversions became the default (config #4 >= 12 tiles per CU)
set -u
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
g=scripts/gpu_check.sh
L=humanoid_mppi-rl_amd/lib
mkdir -p gpurun_out/last
bash $g last/smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" &&
bash $g last/gpu_tests 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread &&
bash scripts/ab_arms.sh swpf "--workload humanoid_ca --steps 30" - $L/libmppi_hip_swp0.so - $L/libmppi_hip_swp0.so &&
bash $g last/bench_humanoid_ca 400 python3 -u bench.py &&
bash $g last/bench_humanoid_ca_global64 400 python3 -u bench.py --global-solves 64 &&
bash $g last/bench_humanoid_ca_48solves 400 python3 -u bench.py --solves 48 &&
bash $g last/prof_humanoid_ca 300 rocprofv3 --kernel-trace --stats -d gpurun_out/last/prof_humanoid_ca -o run --output-format csv -- \
  python3 bench.py --workload humanoid_ca --steps 10 --warmup 1 --no-cpu-baseline --no-traffic --no-kernel-trace &&
bash $g last/pmc_ca 200 bash scripts/pmc_mfma.sh ca_bf16_wave32 --workload humanoid_ca
