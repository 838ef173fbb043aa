#!/bin/bash
# FETCH_SIZE calibration of the per-wave rollouts' eps pattern (tools/fetch_calib.hip) -> gpurun_out/fetch_calib.txt
set -u
export TMPDIR=/tmp
d=gpurun_out/fetch_calib
rm -rf $d; mkdir -p $d
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d $d -o p --output-format csv -- ./tools/fetch_calib > $d/run.log 2>&1 || exit $?
python3 - $d <<'PY' | tee gpurun_out/fetch_calib.txt
import csv, os, sys, collections
d = sys.argv[1]
known = 64 * 21 * 64 * 1024 * 4
vals = collections.defaultdict(list)
for root, _, fs in os.walk(d):
    for f in fs:
        if f.endswith("counter_collection.csv"):
            for r in csv.DictReader(open(os.path.join(root, f))):
                if r["Counter_Name"] == "FETCH_SIZE":
                    vals[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]))
print(f"known bytes per launch: {known} (config #4 eps, 64 solves x 21 x 64 x 1024 fp32)")
for k, v in vals.items():
    if "eps_rows" in k or "stream16" in k:  # eps_rows: 128-B segments, eps_rows16: 64-B, stream16: 16 B/lane
        kb = sum(v) / len(v)
        print(f"{k}: FETCH_SIZE {kb:.0f} KB per launch ({len(v)} launches) -> factor known / (FETCH_SIZE * 1024) = {known / (kb * 1024):.3f}")
PY
