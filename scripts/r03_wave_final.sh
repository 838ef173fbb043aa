#!/bin/bash
# Round-3 (late) evidence for the per-wave CA rollout: bench tests, full bench lines of config #4 (default: 64 solves
# per GPU, weak; --global-solves 64: strong; the 8-solve N = 8 shard; 48 and 32 solves), rocprofv3 kernel stats of the
# default command, MFMA-utilisation counters of fc_wave_kernel.
set -u
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
g=scripts/gpu_check.sh
bash $g wf/bench_tests 400 python -u -m pytest tests/test_gpu_parity.py -k "bench" -v --timeout 200 --timeout-method thread &&
bash $g wf/bench_humanoid_ca 400 python3 -u bench.py &&
bash $g wf/bench_humanoid_ca_global64 400 python3 -u bench.py --global-solves 64 --no-cpu-baseline &&
bash $g wf/bench_humanoid_ca_8perGPU 400 python3 -u bench.py --solves 8 --no-cpu-baseline &&
bash $g wf/bench_humanoid_ca_48solves 400 python3 -u bench.py --solves 48 --no-cpu-baseline &&
bash $g wf/bench_humanoid_ca_32solves 400 python3 -u bench.py --solves 32 --no-cpu-baseline &&
bash $g wf/prof_humanoid_ca 300 rocprofv3 --kernel-trace --stats -d gpurun_out/wf/prof_humanoid_ca -o run --output-format csv -- python3 bench.py --steps 10 --warmup 1 --no-cpu-baseline --no-traffic --no-kernel-trace &&
bash $g wf/pmc_ca_bf16 200 bash scripts/pmc_mfma.sh ca_bf16_wave --workload humanoid_ca
