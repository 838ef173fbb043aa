#!/bin/bash
# MFMA utilisation of a bench workload's kernels from rocprofv3 PMC counters (MI355X_MICROARCH.md "rocprofv3 PMC
# slots", "Per-instruction cycle constants"): two passes of one rocprofv3 call (input file, one "pmc:" line per pass,
# <= 8 SQ + 2 GRBM counters each), the bench run short (--steps 3), profiled arms only compared with profiled arms.
#   mfma_busy   = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)   (GRBM_GUI_ACTIVE sums the 8 XCDs;
#                 SQ_VALU_MFMA_BUSY_CYCLES counts MFMA-pipe cycles summed over SIMDs)
#   mfma_flop   = (SQ_INSTS_VALU_MFMA_MOPS_BF16 + _F16 + _F32) x 512 per dispatch (the gfx94x MfmaFlops formula)
#   wave split  = SQ_ACTIVE_INST_ANY / SQ_WAIT_INST_ANY / SQ_WAIT_ANY over SQ_WAVE_CYCLES (disjoint, quad-cycles)
# usage: bash scripts/pmc_mfma.sh <name> <bench args...>     -> gpurun_out/pmc_mfma_<name>.{txt,log,csv dir}
set -u
name=$1; shift
out=gpurun_out/pmc_mfma_$name
mkdir -p gpurun_out
cat > "$out.pmc.txt" <<'EOF'
pmc: SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT
pmc: SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS
pmc: SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_VALU_MFMA_MOPS_F16 GRBM_GUI_ACTIVE GRBM_COUNT
EOF
timeout -k 10 300 rocprofv3 -i "$out.pmc.txt" -d "$out" -o pmc --output-format csv -- \
  python3 bench.py --steps 3 --warmup 1 --ramp-ms 0 --no-cpu-baseline --no-traffic --no-kernel-trace --no-plain-pass "$@" \
  > "$out.log" 2>&1
rc=$?
echo "== pmc_mfma $name rc=$rc"
python3 - "$out" "$name $*" > "$out.txt" <<'PY'
import csv, os, sys, collections
d, label = sys.argv[1], sys.argv[2]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for root, _, fs in os.walk(d):
    for f in fs:
        if f.endswith("counter_collection.csv"):
            for r in csv.DictReader(open(os.path.join(root, f))):
                k = r["Kernel_Name"].split("(")[0].replace("void ", "")
                acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
print(f"# rocprofv3 PMC, bench.py {label} (3 timed steps + 1 warmup; per-dispatch averages)")
for k, c in sorted(acc.items(), key=lambda kv: -sum(kv[1].get("SQ_WAVE_CYCLES", [0]))):
    a = {n: sum(v) / len(v) for n, v in c.items()}
    n_disp = max(len(v) for v in c.values())
    line = {n: round(v) for n, v in sorted(a.items())}
    print(f"{k[:110]}  dispatches={n_disp}")
    print("   ", line)
    gui = a.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
    if gui > 0 and "SQ_VALU_MFMA_BUSY_CYCLES" in a:
        print(f"    mfma_busy = {a['SQ_VALU_MFMA_BUSY_CYCLES'] / (1024.0 * gui):.3f} of the 1024 SIMDs' cycles "
              f"({gui:.0f} cycles per XCD)")
    if a.get("SQ_INSTS_MFMA"):
        print(f"    busy cycles per MFMA = {a.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / a['SQ_INSTS_MFMA']:.1f} "
              "(16x16x32 bf16: 16 per the guide's cycle table; 16x16x4 f32: 32)")
    flop = 512.0 * (a.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", 0) + a.get("SQ_INSTS_VALU_MFMA_MOPS_F16", 0) +
                    a.get("SQ_INSTS_VALU_MFMA_MOPS_F32", 0))
    if flop:
        print(f"    mfma_flop per dispatch = {flop:.4g}")
    wc = a.get("SQ_WAVE_CYCLES", 0.0)
    if wc:
        parts = {n: a.get(n, 0.0) / wc for n in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY")}
        print("    wave cycles: " + ", ".join(f"{n[3:]} {v:.2f}" for n, v in parts.items()))
    if a.get("SQ_LDS_IDX_ACTIVE"):
        print(f"    LDS: bank-conflict cycles / LDS-array cycles = {a.get('SQ_LDS_BANK_CONFLICT', 0) / a['SQ_LDS_IDX_ACTIVE']:.3f}; "
              f"LDS-array busy = {a['SQ_LDS_IDX_ACTIVE'] / (256.0 * gui) if gui else 0:.3f} of the 256 CUs' cycles "
              "(if SQ_LDS_IDX_ACTIVE counts cycles)")
    if a.get("SQ_WAVES"):
        print(f"    per wave: VALU {a.get('SQ_INSTS_VALU', 0) / a['SQ_WAVES']:.0f}, MFMA {a.get('SQ_INSTS_MFMA', 0) / a['SQ_WAVES']:.0f}, "
              f"LDS {a.get('SQ_INSTS_LDS', 0) / a['SQ_WAVES']:.0f} instructions")
PY
cat "$out.txt"
exit $rc
