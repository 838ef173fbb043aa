#!/bin/bash
# Round-4 late A/B driver for the split-bf16 line: the split-bf16 tests on the default build, then same-box arms
#   bash scripts/r04_abx.sh <tag> <arm>...   (arms as scripts/ab_arms.sh; each list runs twice)
set -u
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
g=scripts/gpu_check.sh
tag=$1; shift
bash $g $tag/tests 600 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -q -x -k "split_bf16" --timeout 300 --timeout-method thread &&
bash $g $tag/ab 900 bash scripts/ab_arms.sh $tag "--workload humanoid_ca --precision bf16x3 --steps 20" "$@" "$@"
