#!/bin/bash
# Same-box A/B of two builds of libmppi_hip: bash scripts/ab_lib.sh <workload> <lib_a.so> <lib_b.so> [reps]
set -u
w=$1; la=$2; lb=$3; reps=${4:-2}
for r in $(seq 1 $reps); do
  for lib in $la $lb; do
    MPPI_HIP_LIB=$lib timeout -k 10 200 python3 bench.py --workload $w --steps 40 --warmup 5 --no-cpu-baseline \
      --no-traffic > gpurun_out/ablib.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then tail -5 gpurun_out/ablib.log; exit $rc; fi
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2].split('/')[-1] if len(sys.argv) > 2 else '', f\"value {d['value']:.4g} ms/step {d['ms_per_step']:.4f} rollout {r['avg_launch_us']:.1f} us frac {r['frac']:.4f}\")" gpurun_out/ablib.log $lib
  done
done
