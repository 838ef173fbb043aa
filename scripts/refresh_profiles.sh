#!/bin/bash
# Round profile set (GPU box): full bench lines (CPU baseline + live PMC traffic) and rocprofv3 --kernel-trace --stats
# summaries per workload -> gpurun_out/final/.  usage: bash scripts/refresh_profiles.sh <bench|prof> <workload...>
set -u
mode=$1; shift
out=gpurun_out/final; mkdir -p $out
export TMPDIR=/tmp
for w in "$@"; do
  if [ "$mode" = bench ]; then
    steps=50; case $w in quad_fa) steps=3;; humanoid_ca_stream) steps=20;; cartpole_fa) steps=10;; esac
    timeout -k 10 420 python3 -u bench.py --workload $w --steps $steps --warmup 2 > $out/bench_$w.log 2>&1
  else
    steps=10; case $w in quad_fa) steps=2;; humanoid_ca_stream) steps=2;; esac
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_$w -o run --output-format csv -- \
      python3 bench.py --workload $w --steps $steps --warmup 1 --no-cpu-baseline --no-traffic --no-kernel-trace > $out/prof_$w.log 2>&1
  fi
  rc=$?; echo "== $mode $w rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $out/*_$w.log; exit $rc; fi
done
