#!/bin/bash
# Round-4 late A/B driver: the wave parity tests on the default build, then same-box arms of the config #4 line
#   bash scripts/r04_ab.sh <tag> <arm>...   (arms as scripts/ab_arms.sh; each list runs twice)
set -u
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
g=scripts/gpu_check.sh
tag=$1; shift
bash $g $tag/tests 600 python -u -m pytest ${TESTFILES:-tests/test_gpu_fullsize.py tests/test_gpu_parity.py} -m gpu -q -x -k "${TESTS:-wave or w32 or config4}" --timeout 300 --timeout-method thread &&
bash $g $tag/ab 900 bash scripts/ab_arms.sh $tag "--workload humanoid_ca" "$@" "$@"
