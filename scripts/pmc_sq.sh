#!/bin/bash
# SQ stall breakdown of the rollout kernel for a bench workload (two rocprofv3 passes of 4 SQ counters from one input
# file: with several passes the profiler launcher runs the command as a child instead of exec-ing into it).
# usage: bash scripts/pmc_sq.sh <name> <bench args...>
set -u
name=$1; shift
out=gpurun_out/pmc_$name
mkdir -p gpurun_out
# PMC_PASSES overrides the passes: ';'-separated, each a space-separated list of counters
passes=${PMC_PASSES:-"SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY;SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL"}
echo "$passes" | tr ';' '\n' | sed 's/^/pmc: /' > "$out.txt"
timeout -k 10 300 rocprofv3 -i "$out.txt" -d "$out" -o pmc --output-format csv -- \
  python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-traffic --no-kernel-trace "$@" > "$out.log" 2>&1
rc=$?
echo "== pmc $name rc=$rc"
python3 - "$out" <<'PY'
import csv, os, sys, collections
d = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for root, _, fs in os.walk(d):
    for f in fs:
        if f.endswith("counter_collection.csv"):
            for r in csv.DictReader(open(os.path.join(root, f))):
                acc[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in acc.items():
    print(k, {n: round(sum(v) / len(v)) for n, v in sorted(c.items())})
PY
exit $rc
