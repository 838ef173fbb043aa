# PMC counters of the layered FA kernels (scripts/fa_layered_ab.py, 2 solves): MFMA busy, LDS conflicts, waits
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
name=$1
out=gpurun_out/pmc_fa_$name
mkdir -p gpurun_out
cat > "$out.pmc.txt" <<'PM'
pmc: SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT
pmc: SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS
pmc: SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE GRBM_COUNT
PM
N=1 timeout -k 10 300 rocprofv3 -i "$out.pmc.txt" -d "$out" -o pmc --output-format csv -- python3 scripts/fa_layered_ab.py > "$out.log" 2>&1
rc=$?
python3 - "$out" > "$out.txt" <<'PY'
import csv, os, sys, collections
d = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for root, _, fs in os.walk(d):
    for f in fs:
        if f.endswith("counter_collection.csv"):
            for r in csv.DictReader(open(os.path.join(root, f))):
                k = r["Kernel_Name"].split("(")[0].replace("void ", "")
                acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in sorted(acc.items(), key=lambda kv: -sum(kv[1].get("SQ_WAVE_CYCLES", [0]))):
    a = {n: sum(v) / len(v) for n, v in c.items()}
    busy = a.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / max(1024 * a.get("GRBM_GUI_ACTIVE", 1) / 8, 1)
    wc = max(a.get("SQ_WAVE_CYCLES", 1), 1)
    print(f"{k[:80]}  mfma_busy={busy:.3f} wait_any={a.get('SQ_WAIT_ANY',0)/wc:.2f} wait_inst={a.get('SQ_WAIT_INST_ANY',0)/wc:.2f} "
          f"active={a.get('SQ_ACTIVE_INST_ANY',0)/wc:.2f} lds_conf/idx={a.get('SQ_LDS_BANK_CONFLICT',0)/max(a.get('SQ_LDS_IDX_ACTIVE',1),1):.3f} "
          f"waves={a.get('SQ_WAVES',0):.0f} mfma/wave={a.get('SQ_INSTS_MFMA',0)/max(a.get('SQ_WAVES',1),1):.0f} "
          f"valu/wave={a.get('SQ_INSTS_VALU',0)/max(a.get('SQ_WAVES',1),1):.0f} lds/wave={a.get('SQ_INSTS_LDS',0)/max(a.get('SQ_WAVES',1),1):.0f} "
          f"vmem/wave={a.get('SQ_INSTS_VMEM',0)/max(a.get('SQ_WAVES',1),1):.0f}")
PY
cat "$out.txt"
exit $rc
