#!/bin/bash
# Round-4 evidence from the current code, part $1 (-> gpurun_out/r4/):
#   a: smoke, the -m gpu suite, config #4 bench lines (default = 64 solves strong on this GPU, the 8-solve shard with
#      and without the world-1 forced gather, fp32, split bf16), config #5
#   b: the other workloads' bench lines
#   c: rocprofv3 kernel stats of every workload, MFMA counters of the per-wave kernels
#   d: horizon probes (after the clock ramp) of the few-tiles regime and config #3
#   e: after the block-diagonal form 2: smoke, the suite, config #4 lines (64 solves; 32 = the N = 2 shard; 16 = N = 4),
#      the kernel stats and MFMA counters of the 64-solve line
#   f: after the split-bf16 per-wave kernel: smoke, the suite, config #4 bf16 and split-bf16 lines, split-bf16 stats
#   g: after its AGPR-form unit: smoke, the suite, the split-bf16 line, its stats and MFMA counters
#   h: closing pass on the final build: smoke, the suite, the default line + kernel stats, the split-bf16 line
#   i: closing pass, the other lines: config #4's N = 2 / 4 / 8 shards, config #5, every other workload
#   j: after the iterative-ILP scheduler for the per-wave units: h, the 32-solve and humanoid MLP lines, MFMA counters
set -u
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
g=scripts/gpu_check.sh
o=gpurun_out/r4; mkdir -p $o
if [ "$1" = a ]; then
  bash $g r4/smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" &&
  bash $g r4/gpu_tests 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread &&
  bash $g r4/bench_humanoid_ca 400 python3 -u bench.py &&
  bash $g r4/bench_humanoid_ca_8solves 400 python3 -u bench.py --global-solves 8 &&
  env MPPI_FORCE_GATHER=1 bash $g r4/bench_humanoid_ca_8solves_gather 400 python3 -u bench.py --global-solves 8 --no-traffic &&
  bash $g r4/bench_humanoid_ca_bf16x3 400 python3 -u bench.py --precision bf16x3 --steps 20 &&
  bash $g r4/bench_humanoid_ca_fp32 400 python3 -u bench.py --precision fp32 --steps 20 &&
  bash $g r4/bench_humanoid_ca_stream 420 python3 -u bench.py --workload humanoid_ca_stream --steps 20 --warmup 2
elif [ "$1" = b ]; then
  for w in humanoid_mlp quad_mlp cartpole cartpole_fa quad_fa; do
    steps=50; case $w in quad_fa) steps=3;; cartpole_fa) steps=10;; esac
    bash $g r4/bench_$w 420 python3 -u bench.py --workload $w --steps $steps --warmup 2 || exit 1
  done
elif [ "$1" = e ]; then
  bash $g r4/smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" &&
  bash $g r4/gpu_tests 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread &&
  bash $g r4/bench_humanoid_ca 400 python3 -u bench.py &&
  bash $g r4/bench_humanoid_ca_32solves 400 python3 -u bench.py --global-solves 32 &&
  bash $g r4/bench_humanoid_ca_16solves 400 python3 -u bench.py --global-solves 16 &&
  bash $g r4/prof_humanoid_ca 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4/prof_humanoid_ca -o run --output-format csv -- \
    python3 bench.py --steps 10 --warmup 1 --no-cpu-baseline --no-traffic --no-kernel-trace &&
  bash $g r4/pmc_ca 200 bash scripts/pmc_mfma.sh ca_bf16_wave32_bd2 --workload humanoid_ca
elif [ "$1" = f ]; then
  # after the split-bf16 per-wave kernel: smoke, the suite, the default and split-bf16 config #4 lines, split-bf16 stats
  bash $g r4/smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" &&
  bash $g r4/gpu_tests 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread &&
  bash $g r4/bench_humanoid_ca 400 python3 -u bench.py &&
  bash $g r4/bench_humanoid_ca_bf16x3 400 python3 -u bench.py --precision bf16x3 --steps 20 &&
  bash $g r4/prof_humanoid_ca_bf16x3 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4/prof_humanoid_ca_bf16x3 -o run --output-format csv -- \
    python3 bench.py --precision bf16x3 --steps 10 --warmup 1 --no-cpu-baseline --no-traffic --no-kernel-trace
elif [ "$1" = g ]; then
  # after the split-bf16 kernel's AGPR-form unit: smoke, the suite, the split-bf16 line, its stats and MFMA counters
  bash $g r4/smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" &&
  bash $g r4/gpu_tests 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread &&
  bash $g r4/bench_humanoid_ca_bf16x3 400 python3 -u bench.py --precision bf16x3 --steps 20 &&
  bash $g r4/prof_humanoid_ca_bf16x3 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4/prof_humanoid_ca_bf16x3 -o run --output-format csv -- \
    python3 bench.py --precision bf16x3 --steps 10 --warmup 1 --no-cpu-baseline --no-traffic --no-kernel-trace &&
  bash $g r4/pmc_x3 200 bash scripts/pmc_mfma.sh ca_bf16x3_wave_agpr --workload humanoid_ca --precision bf16x3
elif [ "$1" = h ]; then
  # closing pass on the final build: smoke, the suite, the default line and its kernel stats, the split-bf16 line
  bash $g r4/smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" &&
  bash $g r4/gpu_tests 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread &&
  bash $g r4/bench_humanoid_ca 400 python3 -u bench.py &&
  bash $g r4/prof_humanoid_ca 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4/prof_humanoid_ca -o run --output-format csv -- \
    python3 bench.py --steps 10 --warmup 1 --no-cpu-baseline --no-traffic --no-kernel-trace &&
  bash $g r4/bench_humanoid_ca_bf16x3 400 python3 -u bench.py --precision bf16x3 --steps 20
elif [ "$1" = i ]; then
  # closing pass, the other lines on the final build: the N = 2 / 4 / 8 shards of config #4, config #5, every other workload
  bash $g r4/bench_humanoid_ca_32solves 400 python3 -u bench.py --global-solves 32 &&
  bash $g r4/bench_humanoid_ca_16solves 400 python3 -u bench.py --global-solves 16 &&
  bash $g r4/bench_humanoid_ca_8solves 400 python3 -u bench.py --global-solves 8 &&
  bash $g r4/bench_humanoid_ca_stream 420 python3 -u bench.py --workload humanoid_ca_stream --steps 20 --warmup 2 &&
  for w in humanoid_mlp quad_mlp cartpole cartpole_fa quad_fa; do
    steps=50; case $w in quad_fa) steps=3;; cartpole_fa) steps=10;; esac
    bash $g r4/bench_$w 420 python3 -u bench.py --workload $w --steps $steps --warmup 2 || exit 1
  done
elif [ "$1" = j ]; then
  # after the iterative-ILP scheduler for the per-wave units: the closing pass h, then the other per-wave lines
  bash "$0" h &&
  bash $g r4/bench_humanoid_ca_32solves 400 python3 -u bench.py --global-solves 32 &&
  bash $g r4/bench_humanoid_mlp 420 python3 -u bench.py --workload humanoid_mlp --steps 50 --warmup 2 &&
  bash $g r4/pmc_x3 200 bash scripts/pmc_mfma.sh ca_bf16x3_wave_iilp --workload humanoid_ca --precision bf16x3 &&
  bash $g r4/pmc_w32 200 bash scripts/pmc_mfma.sh ca_bf16_wave32_iilp --workload humanoid_ca
elif [ "$1" = d ]; then
  bash $g r4/horizon_B8 300 python3 -u tools/horizon_probe.py --B=8 --ramp &&
  bash $g r4/horizon_B2 300 python3 -u tools/horizon_probe.py --B=2 --ramp &&
  bash $g r4/horizon_quad 300 python3 -u tools/horizon_probe.py --B=1 --quad --ramp
else
  for w in humanoid_ca humanoid_mlp quad_mlp cartpole cartpole_fa humanoid_ca_stream quad_fa; do
    steps=10; case $w in quad_fa) steps=2;; humanoid_ca_stream) steps=2;; esac
    bash $g r4/prof_$w 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4/prof_$w -o run --output-format csv -- \
      python3 bench.py --workload $w --steps $steps --warmup 1 --no-cpu-baseline --no-traffic --no-kernel-trace || exit 1
  done
  bash $g r4/pmc_ca 200 bash scripts/pmc_mfma.sh ca_bf16_wave32_bd --workload humanoid_ca &&
  bash $g r4/pmc_ca8 200 bash scripts/pmc_mfma.sh ca_bf16_msplit_8 --workload humanoid_ca --global-solves 8
fi
