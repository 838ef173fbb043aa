#!/bin/bash
# PMC passes (one counter per run, as MI355X_MICROARCH.md prescribes) for the dominant kernel of each workload
# -> gpurun_out/final/pmc_<workload>_<counter>/.  usage: bash scripts/pmc_round.sh <workload...>
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/final
for w in "$@"; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 200 rocprofv3 --pmc $c -d gpurun_out/final/pmc_${w}_$c -o pmc --output-format csv -- \
      python3 bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-traffic > gpurun_out/final/pmc_${w}_$c.log 2>&1
    rc=$?; echo "== pmc $w $c rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 gpurun_out/final/pmc_${w}_$c.log; exit $rc; fi
  done
done
