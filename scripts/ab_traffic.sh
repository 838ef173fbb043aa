#!/bin/bash
# Same-box A/B of builds of libmppi_hip on one workload WITH the live PMC traffic pass (FETCH_SIZE / WRITE_SIZE of the
# dominant kernel): bash scripts/ab_traffic.sh <workload> <steps> <lib...>
set -u
w=$1; steps=$2; shift 2
export TMPDIR=/tmp
for lib in "$@"; do
  MPPI_HIP_LIB=$lib timeout -k 10 600 python3 bench.py --workload $w --steps $steps --warmup 1 --no-cpu-baseline \
    --no-kernel-trace --no-plain-pass > gpurun_out/abtraffic.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/abtraffic.log; exit $rc; fi
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2].split('/')[-1], f\"value {d['value']:.4g} ms/step {d['ms_per_step']:.4f} rollout {r['avg_launch_us']:.1f} us frac {r['frac']:.4f} | {r.get('traffic_note')}\")" gpurun_out/abtraffic.log $lib
done
