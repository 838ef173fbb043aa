#!/bin/bash
# Round-3 evidence pass on the GPU box: MFMA-utilisation counters (scripts/pmc_mfma.sh) of the learned-dynamics
# rollouts, and full bench lines for config #4 at 64 solves and in exact fp32.  Each step under its own timeout.
set -u
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
g=scripts/gpu_check.sh
bash $g r03b/pmc_ca_bf16 200 bash scripts/pmc_mfma.sh ca_bf16 --workload humanoid_ca &&
bash $g r03b/pmc_ca_fp32 200 bash scripts/pmc_mfma.sh ca_fp32 --workload humanoid_ca --precision fp32 &&
bash $g r03b/pmc_hmlp_bf16 200 bash scripts/pmc_mfma.sh hmlp_bf16 --workload humanoid_mlp &&
bash $g r03b/pmc_qmlp_bf16 200 bash scripts/pmc_mfma.sh qmlp_bf16 --workload quad_mlp &&
bash $g r03b/pmc_cpfa_bf16 200 bash scripts/pmc_mfma.sh cpfa_bf16 --workload cartpole_fa &&
bash $g r03b/pmc_qfa_bf16 250 bash scripts/pmc_mfma.sh qfa_bf16 --workload quad_fa &&
bash $g r03b/bench_ca64 400 python3 -u bench.py --solves 64 --steps 30 &&
bash $g r03b/bench_ca_fp32 400 python3 -u bench.py --precision fp32 --steps 20
