#!/bin/bash
# Round-3 final evidence on the GPU box, part $1:
#   a: the -m gpu suite, full bench lines (CPU baseline, live PMC traffic, kernel trace) for the bf16 workloads
#      (config #4: the default 64 solves per GPU, the same split over the ranks, the 8-solve shard, 32 and 48 solves)
#   b: the remaining bench lines, rocprofv3 kernel stats of every workload, MFMA-utilisation counters
set -u
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
g=scripts/gpu_check.sh
o=gpurun_out/final; mkdir -p $o
if [ "$1" = a ]; then
  bash $g final/gpu_tests 500 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread &&
  bash $g final/bench_humanoid_ca 400 python3 -u bench.py &&
  bash $g final/bench_humanoid_ca_global64 400 python3 -u bench.py --global-solves 64 &&
  bash $g final/bench_humanoid_ca_8perGPU 400 python3 -u bench.py --solves 8 &&
  bash $g final/bench_humanoid_ca_32solves 400 python3 -u bench.py --solves 32 &&
  bash $g final/bench_humanoid_ca_48solves 400 python3 -u bench.py --solves 48 &&
  bash $g final/bench_humanoid_ca_fp32 400 python3 -u bench.py --precision fp32 --steps 20 &&
  bash $g final/bench_humanoid_mlp 400 python3 -u bench.py --workload humanoid_mlp
elif [ "$1" = b ]; then
  bash $g final/bench_humanoid_mlp 400 python3 -u bench.py --workload humanoid_mlp &&
  bash scripts/refresh_profiles.sh bench quad_mlp cartpole cartpole_fa humanoid_ca_stream quad_fa
else
  bash scripts/refresh_profiles.sh prof humanoid_ca humanoid_mlp quad_mlp cartpole cartpole_fa humanoid_ca_stream quad_fa &&
  bash $g final/pmc_ca_bf16 200 bash scripts/pmc_mfma.sh ca_bf16_wave --workload humanoid_ca &&
  bash $g final/pmc_ca_bf16_8 200 bash scripts/pmc_mfma.sh ca_bf16_8 --workload humanoid_ca --solves 8 &&
  bash $g final/pmc_hmlp_bf16 200 bash scripts/pmc_mfma.sh hmlp_bf16_wave --workload humanoid_mlp
fi
