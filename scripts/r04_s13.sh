#!/bin/bash
# Round-4 GPU session 13d: 2 lanes (32x32 kernel forced, phase offset) with the reduce grid at 128 / 64 blocks
set -u
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
g=scripts/gpu_check.sh
mkdir -p gpurun_out/s13
env MPPI_FC_WAVE=3 MPPI_REDUCE_BLOCKS=128 bash $g s13/lanes_rb128 400 python3 -u tools/lanes_probe.py 300 --offset --lanes=1 --lanes=2 --lanes=1 --lanes=2 &&
env MPPI_FC_WAVE=3 MPPI_REDUCE_BLOCKS=64 bash $g s13/lanes_rb64 400 python3 -u tools/lanes_probe.py 300 --offset --lanes=2 --lanes=2 &&
env MPPI_FC_WAVE=3 bash $g s13/lanes_rb256 400 python3 -u tools/lanes_probe.py 300 --offset --lanes=1 --lanes=2 --lanes=1 --lanes=2
