set -o pipefail
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_fullsize.py -k "wave_mlp" > gpurun_out/wave_mlp_tests.log 2>&1
rc=$?; tail -15 gpurun_out/wave_mlp_tests.log; [ $rc -ne 0 ] && exit $rc
bash scripts/ab_arms.sh m64 "--workload humanoid_mlp --steps 30" -,MPPI_FC_WAVE=0 -,MPPI_FC_WAVE=2 -,MPPI_FC_WAVE=1 -,MPPI_FC_WAVE=0 -,MPPI_FC_WAVE=2
