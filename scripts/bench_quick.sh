#!/bin/bash
# quick bench lines (no CPU baseline / PMC): bash scripts/bench_quick.sh <tag> <workload...>
set -u
tag=$1; shift
for w in "$@"; do
  timeout -k 10 200 python3 bench.py --workload $w --steps 30 --warmup 5 --no-cpu-baseline --no-traffic \
    > gpurun_out/q_${tag}_${w}.log 2>&1
  rc=$?; echo "== $w rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/q_${tag}_${w}.log; exit $rc; fi
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(f\"value {d['value']:.4g} ms/step {d['ms_per_step']:.4f} kernels {({k: round(v*1e3,1) for k,v in d['kernel_ms'].items()})} frac {d['roofline']['frac']:.4f}\")" gpurun_out/q_${tag}_${w}.log
done
