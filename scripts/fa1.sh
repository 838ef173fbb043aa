set -o pipefail
mkdir -p gpurun_out/fa1
K="fa_d512 or fa_wide_bf16 or fa_quad_full or fa_train_py"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_subsets.py -m gpu -v --timeout 200 --timeout-method thread -k "$K" > gpurun_out/fa1/tests.log 2>&1
rc1=$?
MPPI_FA_LAYERED=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 200 --timeout-method thread -k "fa_d512_layered_env" > gpurun_out/fa1/tests_fused.log 2>&1
grep -E "PASS|FAIL|Max abs|Max rel|passed|failed" gpurun_out/fa1/tests.log gpurun_out/fa1/tests_fused.log | tail -40
[ $rc1 -eq 0 ] || exit 1
timeout -k 10 200 python -u scripts/fa_layered_ab.py > gpurun_out/fa1/ab.log 2>&1 && \
MPPI_FA_LAYERED=0 timeout -k 10 200 python -u scripts/fa_layered_ab.py >> gpurun_out/fa1/ab.log 2>&1
rc=$?; cat gpurun_out/fa1/ab.log; exit $rc
