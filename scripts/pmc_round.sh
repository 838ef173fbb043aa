#!/bin/bash
# PMC passes (one counter per pass, as MI355X_MICROARCH.md prescribes) for the dominant kernel of each workload
# -> gpurun_out/final/pmc_<workload>/ (pass_1 = FETCH_SIZE, pass_2 = WRITE_SIZE).  One rocprofv3 call with a
# two-pass input file: the launcher then runs the command as a child per pass (no exec into it).
# usage: bash scripts/pmc_round.sh <workload...>
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/final
printf 'pmc: FETCH_SIZE\npmc: WRITE_SIZE\n' > gpurun_out/final/pmc_counters.txt
for w in "$@"; do
  timeout -k 10 300 rocprofv3 -i gpurun_out/final/pmc_counters.txt -d gpurun_out/final/pmc_${w} -o pmc --output-format csv -- \
    python3 bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-traffic --no-kernel-trace > gpurun_out/final/pmc_${w}.log 2>&1
  rc=$?; echo "== pmc $w rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/final/pmc_${w}.log; exit $rc; fi
done
