# same-box A/B of layered-FA build variants: bash scripts/fa_ab.sh <tag> <lib>... ('-' = the default library);
# per variant one rocprofv3 kernel trace of scripts/fa_layered_ab.py (3 solves) -> per-kernel average durations
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tag=$1; shift
export MPPI_FA_LAYERED=${MPPI_FA_LAYERED:-1}
out=gpurun_out/fa_ab/$tag; mkdir -p $out
i=0
for lib in "$@"; do
  i=$((i+1))
  if [ "$lib" = "-" ]; then unset MPPI_HIP_LIB; else export MPPI_HIP_LIB=$GRAFT_REPO_ROOT/$lib; fi
  d=$out/v$i
  N=2 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- python3 scripts/fa_layered_ab.py > $d.log 2>&1 || { echo "variant $lib failed"; tail -5 $d.log; exit 1; }
  f=$(find $d -name "*kernel_stats.csv" | head -1)
  python3 - "$f" "$lib" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows if "fal_" in r["Name"] or "fa_rollout" in r["Name"]) / 3 / 1e6
print(f"== {sys.argv[2]}: rollout kernels {tot:.2f} ms/solve")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:7]:
    n = r["Name"].replace("mppi::", "").replace("(mppi::FalGemm)", "")
    print(f'   {n[:60]:60s} n={r["Calls"]:>5s} avg={float(r["AverageNs"])/1e3:8.1f}us')
PY
done
