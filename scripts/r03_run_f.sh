#!/bin/bash
set -u
export TMPDIR=/tmp
g=scripts/gpu_check.sh
L=humanoid_mppi-rl_amd/lib
bash $g r03f/gpu_tests 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread &&
bash $g r03f/ab_fa 900 bash scripts/ab_traffic.sh quad_fa 2 $L/libmppi_hip.so $L/libmppi_hip_fasep.so $L/libmppi_hip_fapfr3.so &&
bash $g r03f/hp8 200 python -u tools/horizon_probe.py --B=8 &&
bash $g r03f/hp2 200 python -u tools/horizon_probe.py --B=2
