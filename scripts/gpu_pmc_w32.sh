set -o pipefail
MPPI_FC_WAVE=2 bash scripts/pmc_mfma.sh w16 --workload humanoid_ca > /dev/null 2>&1 || exit 1
MPPI_FC_WAVE=3 bash scripts/pmc_mfma.sh w32 --workload humanoid_ca > /dev/null 2>&1 || exit 1
grep -A8 "fc_wave" gpurun_out/pmc_mfma_w16.txt | grep -v "{"; grep -A8 "fc_wave" gpurun_out/pmc_mfma_w32.txt | grep -v "{"
