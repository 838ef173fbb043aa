#!/bin/bash
# Same-box A/B of several builds of libmppi_hip on one workload: bash scripts/ab_libs.sh <workload> <steps> <lib...>
set -u
w=$1; steps=$2; shift 2
for lib in "$@"; do
  MPPI_HIP_LIB=$lib timeout -k 10 300 python3 bench.py --workload $w --steps $steps --warmup 1 --no-cpu-baseline \
    --no-traffic > gpurun_out/ablibs.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/ablibs.log; exit $rc; fi
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2].split('/')[-1] if len(sys.argv) > 2 else '', f\"value {d['value']:.4g} ms/step {d['ms_per_step']:.4f} rollout {r['avg_launch_us']:.1f} us frac {r['frac']:.4f}\")" gpurun_out/ablibs.log $lib
done
