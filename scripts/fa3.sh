set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/fa3
N=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fa3/prof -o run --output-format csv -- python3 scripts/fa_layered_ab.py > gpurun_out/fa3/prof.log 2>&1
rc=$?
f=$(find gpurun_out/fa3/prof -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/fa3/kernel_stats.csv 2>/dev/null
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/fa3/kernel_stats.csv")))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:12]:
    print(f'{r["Name"][:90]:90s} n={r["Calls"]:>6s} avg={float(r["AverageNs"])/1e3:9.1f}us tot={float(r["TotalDurationNs"])/1e6:9.2f}ms')
PY
exit $rc
