#!/bin/bash
# A/B a kernel-variant env var on one bench workload: bash scripts/ab_env.sh <VAR> <workload> <value...>
set -u
var=$1; w=$2; shift 2
for v in "$@"; do
  env $var=$v timeout -k 10 200 python3 bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline --no-traffic --no-kernel-trace \
    > gpurun_out/ab_${w}_${var}_$v.log 2>&1
  rc=$?; echo "== $w $var=$v rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/ab_${w}_${var}_$v.log; exit $rc; fi
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2].split('/')[-1] if len(sys.argv) > 2 else '', f\"value {d['value']:.4g} ms/step {d['ms_per_step']:.4f} rollout {r['avg_launch_us']:.1f} us frac {r['frac']:.4f}\")" gpurun_out/ab_${w}_${var}_$v.log
done
