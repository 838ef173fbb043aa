#!/bin/bash
# rocprofv3 kernel-trace --stats summaries of the bench workloads -> gpurun_out/prof_<workload>/ (copy to profiles/)
set -u
for w in "$@"; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$w -o run --output-format csv -- \
    python3 bench.py --workload $w --steps 10 --warmup 2 --no-cpu-baseline --no-traffic --no-kernel-trace > gpurun_out/prof_$w.log 2>&1
  rc=$?; echo "== prof $w rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
