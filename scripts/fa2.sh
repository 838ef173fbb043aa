set -o pipefail
mkdir -p gpurun_out/fa2
timeout -k 10 200 python -u scripts/fa_layered_diag.py > gpurun_out/fa2/diag.log 2>&1 && \
MPPI_FA_LAYERED=0 timeout -k 10 200 python -u scripts/fa_layered_diag.py >> gpurun_out/fa2/diag.log 2>&1
rc=$?; cat gpurun_out/fa2/diag.log; exit $rc
