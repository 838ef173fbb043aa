#!/bin/bash
# Round-4 GPU session 1: the suite after the hygiene / boundary changes, smoke, the wave32 spill fix A/B, the
# few-tiles regime's stamps and horizon probe, WRITE_SIZE of the fixed wave32 kernel.
set -u
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
g=scripts/gpu_check.sh
L=humanoid_mppi-rl_amd/lib
mkdir -p gpurun_out/s1
bash $g s1/smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" &&
bash $g s1/gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread &&
bash $g s1/ab_w32 600 bash scripts/ab_arms.sh w32 "--workload humanoid_ca --steps 30" $L/libmppi_hip_head.so - $L/libmppi_hip_head.so - &&
bash $g s1/ab_8 300 bash scripts/ab_arms.sh s8 "--workload humanoid_ca --global-solves 8 --steps 50" - - &&
bash $g s1/stamps_B8 200 python -u tools/stamps.py --B=8 &&
bash $g s1/stamps_B2 200 python -u tools/stamps.py --B=2 &&
bash $g s1/horizon_B8 300 python -u tools/horizon_probe.py --B=8 &&
bash $g s1/horizon_B2 300 python -u tools/horizon_probe.py --B=2 &&
bash $g s1/pmc_w32 200 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/s1/pmc -o pmc --output-format csv -- \
  python3 bench.py --workload humanoid_ca --steps 3 --warmup 1 --no-cpu-baseline --no-traffic --no-kernel-trace --ramp-ms 0
