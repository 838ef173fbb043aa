#!/bin/bash
# Round-3 closing evidence from the final code, part $1:
#   a: smoke, the -m gpu suite, config #4 bench lines (default 64/GPU, --global-solves 64, 8, 32, 48 solves, fp32)
#   b: the other workloads' bench lines
#   c: rocprofv3 kernel stats of every workload, MFMA counters of the per-wave kernels
set -u
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
g=scripts/gpu_check.sh
o=gpurun_out/last; mkdir -p $o
if [ "$1" = a ]; then
  bash $g last/smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" &&
  bash $g last/gpu_tests 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread &&
  bash $g last/bench_humanoid_ca 400 python3 -u bench.py &&
  bash $g last/bench_humanoid_ca_global64 400 python3 -u bench.py --global-solves 64 &&
  bash $g last/bench_humanoid_ca_8perGPU 400 python3 -u bench.py --solves 8 &&
  bash $g last/bench_humanoid_ca_32solves 400 python3 -u bench.py --solves 32 &&
  bash $g last/bench_humanoid_ca_48solves 400 python3 -u bench.py --solves 48 &&
  bash $g last/bench_humanoid_ca_fp32 400 python3 -u bench.py --precision fp32 --steps 20
elif [ "$1" = b ]; then
  for w in humanoid_mlp quad_mlp cartpole cartpole_fa humanoid_ca_stream quad_fa; do
    steps=50; case $w in quad_fa) steps=3;; humanoid_ca_stream) steps=20;; cartpole_fa) steps=10;; esac
    bash $g last/bench_$w 420 python3 -u bench.py --workload $w --steps $steps --warmup 2 || exit 1
  done
else
  for w in humanoid_ca humanoid_mlp quad_mlp cartpole cartpole_fa humanoid_ca_stream quad_fa; do
    steps=10; case $w in quad_fa) steps=2;; humanoid_ca_stream) steps=2;; esac
    bash $g last/prof_$w 300 rocprofv3 --kernel-trace --stats -d gpurun_out/last/prof_$w -o run --output-format csv -- \
      python3 bench.py --workload $w --steps $steps --warmup 1 --no-cpu-baseline --no-traffic --no-kernel-trace || exit 1
  done
  bash $g last/pmc_ca 200 bash scripts/pmc_mfma.sh ca_bf16_wave32 --workload humanoid_ca &&
  bash $g last/pmc_mlp 200 bash scripts/pmc_mfma.sh hmlp_bf16_wave --workload humanoid_mlp
fi
