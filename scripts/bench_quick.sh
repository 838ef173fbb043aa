#!/bin/bash
# quick bench lines (no CPU baseline / PMC / kernel trace): bash scripts/bench_quick.sh <tag> <workload...>
set -u
tag=$1; shift
for w in "$@"; do
  timeout -k 10 200 python3 bench.py --workload $w --steps 30 --warmup 5 --no-cpu-baseline --no-traffic --no-kernel-trace \
    > gpurun_out/q_${tag}_${w}.log 2>&1
  rc=$?; echo "== $w rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/q_${tag}_${w}.log; exit $rc; fi
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(f\"value {d['value']:.4g} ms/step {d['ms_per_step']:.4f} rollout(clock) {r['avg_launch_us']:.1f} us frac {r['frac']:.4f} plain {({k: round(v*1e3,1) for k,v in (d['plain_solve_kernel_ms'] or {}).items()})}\")" gpurun_out/q_${tag}_${w}.log
done
