#!/bin/bash
# Run one GPU test selection against several builds of libmppi_hip, twice each (determinism / regression bisect):
# bash scripts/det_check.sh "<pytest -k expr>" <lib...>
set -u
k=$1; shift
for lib in "$@"; do
  for rep in 1 2; do
    MPPI_HIP_LIB=$PWD/$lib timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "$k" --timeout 120 \
      --timeout-method thread > gpurun_out/det.log 2>&1
    rc=$?
    echo "$(basename $lib) rep $rep rc=$rc $(tail -1 gpurun_out/det.log)"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -20 gpurun_out/det.log; exit $rc; fi
  done
done
