#!/bin/bash
# GPU passes of a round (-> gpurun_out/$ROUND/<pass>/, ROUND defaults to "cur"), part $1:
#   base: the default line (config #4, fp32-accurate split mode) and the lines around it on the current build
#   suite: smoke + the -m gpu suite
#   ab <tag> "<bench args>" <arm>...: same-box A/B arms (scripts/ab_arms.sh)
set -u
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
g=scripts/gpu_check.sh
p=${2:-x}
R=${ROUND:-cur}
mkdir -p gpurun_out/$R/$p
case "$1" in
base)
  bash $g $R/$p/bench_humanoid_ca 420 python3 -u bench.py &&
  bash $g $R/$p/bench_humanoid_ca_8solves 300 python3 -u bench.py --global-solves 8 --no-cpu-baseline &&
  bash $g $R/$p/bench_humanoid_ca_bf16 300 python3 -u bench.py --precision bf16 --no-cpu-baseline --no-traffic &&
  bash $g $R/$p/bench_humanoid_mlp 300 python3 -u bench.py --workload humanoid_mlp --no-cpu-baseline --no-traffic --steps 20
  ;;
suite)
  bash $g $R/$p/smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" &&
  bash $g $R/$p/gpu_tests 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread
  ;;
x3)  # the split per-wave kernel: its tests, then same-box A/B against the base library (two pairs)
  bash $g $R/$p/gpu_tests_x3 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -k \
    "split_bf16 or fp32_accurate or config4_full_size_matches_oracle or config5_full_size_subset or humanoid_64_solves" &&
  bash scripts/ab_arms.sh x3 "--workload humanoid_ca" humanoid_mppi-rl_amd/lib/libmppi_hip_base.so - \
    humanoid_mppi-rl_amd/lib/libmppi_hip_base.so - > gpurun_out/$R/$p/ab_x3.log 2>&1; cat gpurun_out/$R/$p/ab_x3.log
  ;;
sweep)  # the split path's routing across shard sizes (the strong-scaling shards: 64 / N solves)
  a="--workload humanoid_ca --global-solves"
  for arms in "8|- -,MPPI_X3_WAVE=2 -,MPPI_X3_TILES=1" "16|- -,MPPI_X3_WAVE=2 -,MPPI_X3_WAVE=2,MPPI_X3_PAIR=1" \
              "32|- -,MPPI_X3_PAIR=1 -,MPPI_X3_WAVE=0" "48|- -,MPPI_X3_PAIR=0" "64|- -,MPPI_X3_PAIR=0"; do
    gs=${arms%%|*}
    bash scripts/ab_arms.sh sweep$gs "$a $gs" ${arms#*|} || exit 1
  done > gpurun_out/$R/$p/sweep.log 2>&1; cat gpurun_out/$R/$p/sweep.log
  ;;
msplit)  # the split M-split kernels (few-tiles shards): their tests, then same-box A/B against the HEAD library
  bash $g $R/$p/gpu_tests_ms 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -k \
    "split_bf16 or fp32_accurate or config5_full_size_subset or x3 or 8_solves or mlp" &&
  for gs in 8 16; do
    bash scripts/ab_arms.sh ms$gs "--workload humanoid_ca --global-solves $gs" humanoid_mppi-rl_amd/lib/libmppi_hip_head.so - \
      humanoid_mppi-rl_amd/lib/libmppi_hip_head.so - || exit 1
  done > gpurun_out/$R/$p/ab_ms.log 2>&1 &&
  bash scripts/ab_arms.sh msmlp "--workload humanoid_mlp --global-solves 8" humanoid_mppi-rl_amd/lib/libmppi_hip_head.so - \
    >> gpurun_out/$R/$p/ab_ms.log 2>&1; cat gpurun_out/$R/$p/ab_ms.log
  ;;
ab)  # bash scripts/gpu_pass.sh ab <pass> <tag> "<bench args>" <arm>...: same-box A/B arms (scripts/ab_arms.sh)
  shift 2; tag=$1; args=$2; shift 2
  bash scripts/ab_arms.sh $tag "$args" "$@" > gpurun_out/$R/$p/ab_$tag.log 2>&1; rc=$?; cat gpurun_out/$R/$p/ab_$tag.log; exit $rc
  ;;
final)  # the closing evidence pass: bench lines (CPU baseline, PMC traffic, kernel trace) + rocprofv3 stats of the default
  bash $g $R/$p/bench_humanoid_ca 420 python3 -u bench.py &&
  bash $g $R/$p/bench_humanoid_ca_bf16 300 python3 -u bench.py --precision bf16 --no-cpu-baseline &&
  bash $g $R/$p/bench_humanoid_ca_8solves 300 python3 -u bench.py --global-solves 8 --no-cpu-baseline &&
  bash $g $R/$p/bench_humanoid_ca_16solves 300 python3 -u bench.py --global-solves 16 --no-cpu-baseline &&
  bash $g $R/$p/bench_humanoid_ca_32solves 300 python3 -u bench.py --global-solves 32 --no-cpu-baseline &&
  MPPI_FORCE_GATHER=1 bash $g $R/$p/bench_humanoid_ca_8solves_gather 300 python3 -u bench.py --global-solves 8 --no-cpu-baseline --no-traffic &&
  bash $g $R/$p/bench_cartpole_fa 300 python3 -u bench.py --workload cartpole_fa --no-cpu-baseline &&
  bash $g $R/$p/bench_humanoid_mlp 300 python3 -u bench.py --workload humanoid_mlp --no-cpu-baseline &&
  bash $g $R/$p/bench_humanoid_ca_stream 420 python3 -u bench.py --workload humanoid_ca_stream --steps 20 --no-cpu-baseline &&
  bash $g $R/$p/bench_quad_mlp 300 python3 -u bench.py --workload quad_mlp --no-cpu-baseline &&
  bash $g $R/$p/bench_cartpole 300 python3 -u bench.py --workload cartpole --no-cpu-baseline &&
  bash $g $R/$p/bench_quad_fa 300 python3 -u bench.py --workload quad_fa --steps 3 --warmup 1 --no-cpu-baseline &&
  bash $g $R/$p/prof_humanoid_ca 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$R/$p/prof_humanoid_ca -o run \
    --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-traffic --no-kernel-trace &&
  bash scripts/pmc_mfma.sh ${R}_${p}_x3p --workload humanoid_ca > /dev/null &&
  bash scripts/pmc_mfma.sh ${R}_${p}_x3h8 --workload humanoid_ca --global-solves 8 > /dev/null
  ;;
tests)  # a subset: bash scripts/gpu_pass.sh tests <pass> "<pytest -k expr>"
  bash $g $R/$p/gpu_tests_k 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -k "$3"
  ;;
esac
