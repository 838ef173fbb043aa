#!/bin/bash
# A/B a kernel-variant env var on one bench workload: bash scripts/ab_env.sh <VAR> <workload> <value...>
set -u
var=$1; w=$2; shift 2
for v in "$@"; do
  env $var=$v timeout -k 10 200 python3 bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline --no-traffic \
    > gpurun_out/ab_${w}_${var}_$v.log 2>&1
  rc=$?; echo "== $w $var=$v rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/ab_${w}_${var}_$v.log; exit $rc; fi
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(f\"value {d['value']:.4g} ms/step {d['ms_per_step']:.4f} kernels {({k: round(v*1e3,1) for k,v in d['kernel_ms'].items()})} frac {d['roofline']['frac']:.4f}\")" gpurun_out/ab_${w}_${var}_$v.log
done
