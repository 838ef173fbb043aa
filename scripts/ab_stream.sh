#!/bin/bash
# Same-box A/B of libmppi_hip builds on the receding-horizon stream (config #5, 4 steps each; ab_lib.sh runs 40 steps,
# which overflow the kernel clock slots at 256 solves per step).  usage: bash scripts/ab_stream.sh <lib.so...>
for lib in "$@"; do
  MPPI_HIP_LIB=$lib timeout -k 10 200 python3 bench.py --workload humanoid_ca_stream --steps 4 --warmup 1 --no-cpu-baseline --no-traffic --no-kernel-trace > gpurun_out/abs.log 2>&1 || { tail -5 gpurun_out/abs.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/abs.log').read().strip().splitlines()[-1]); print(sys.argv[1].split('/')[-1], d['ms_per_step'], d['roofline']['avg_launch_us'])" $lib
done
