#!/bin/bash
# Round-4 late session: the split-bf16 bench line with PMC traffic (bench alias fix), then a same-box A/B of the
# headline fc_wave32_kernel with the block's younger half at s_setprio 1 and/or started ~4-6k cycles late.
set -u
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
g=scripts/gpu_check.sh
L=humanoid_mppi-rl_amd/lib
mkdir -p gpurun_out/r4
bash $g r4/bench_humanoid_ca_bf16x3 400 python3 -u bench.py --precision bf16x3 --steps 20 &&
bash $g s19/ab_prio 900 bash scripts/ab_arms.sh w32p "--workload humanoid_ca" - $L/libmppi_hip_w32p.so $L/libmppi_hip_w32o2.so $L/libmppi_hip_w32o3.so $L/libmppi_hip_w32po3.so - $L/libmppi_hip_w32p.so $L/libmppi_hip_w32o2.so $L/libmppi_hip_w32o3.so $L/libmppi_hip_w32po3.so
