// Learned-dynamics MPPI rollout, bf16 with two 16-sample tiles per wave (fc_rollout_kernel_wide, fc_rollout.h): the
// instantiations for the folded humanoid CA and MLP(128 x 2) nets and their launch.  Own translation unit so it takes
// its own codegen flags (build.py PER_FILE_FLAGS: accumulators in VGPRs, -amdgpu-mfma-vgpr-form).
#include "fc_rollout.h"

namespace mppi {

template <int ARCH, int COST>
static hipError_t launch_wide_t(const SolveArgs& a, FcArgs fa, int img_lds, hipStream_t stream) {
  using L = Lay<ARCH, MPPI_PREC_BF16, COST>;
  const int total_groups = a.B * (a.Kp >> 4);
  if ((a.Kp >> 4) % 2 != 0) return hipErrorInvalidValue;  // both tiles of a block in one solve
  fa.groups_per_block = 1;
  const size_t lds = (size_t)img_lds + 2 * (size_t)L::BYTES;
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  auto kern = fc_rollout_kernel_wide<ARCH, COST>;
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(kern, dim3(total_groups / 2), dim3(64 * kSplit), lds, stream, a, fa);
  return hipGetLastError();
}

template <int ARCH>
static hipError_t launch_wide_cost(int cost, const SolveArgs& a, const FcArgs& fa, int img_lds, hipStream_t s) {
  switch (cost) {
    case MPPI_COST_HUMANOID_V3: return launch_wide_t<ARCH, MPPI_COST_HUMANOID_V3>(a, fa, img_lds, s);
    case MPPI_COST_HUMANOID_V1: return launch_wide_t<ARCH, MPPI_COST_HUMANOID_V1>(a, fa, img_lds, s);
    case MPPI_COST_QUAD_JL: return launch_wide_t<ARCH, MPPI_COST_QUAD_JL>(a, fa, img_lds, s);
    case MPPI_COST_QUAD_EST: return launch_wide_t<ARCH, MPPI_COST_QUAD_EST>(a, fa, img_lds, s);
    case MPPI_COST_CARTPOLE_EST: return launch_wide_t<ARCH, MPPI_COST_CARTPOLE_EST>(a, fa, img_lds, s);
    case MPPI_COST_CARTPOLE: return launch_wide_t<ARCH, MPPI_COST_CARTPOLE>(a, fa, img_lds, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_fc_wide(int arch, int cost, const SolveArgs& a, FcArgs fa, int img_lds, hipStream_t stream) {
  if (arch == kArchCA) {  // the CA kernel is built for the humanoid (qpos 28) with its two costs
    if (cost == MPPI_COST_HUMANOID_V1) return launch_wide_t<kArchCA, MPPI_COST_HUMANOID_V1>(a, fa, img_lds, stream);
    return launch_wide_t<kArchCA, MPPI_COST_HUMANOID_V3>(a, fa, img_lds, stream);
  }
  if (arch == kArchMLP) return launch_wide_cost<kArchMLP>(cost, a, fa, img_lds, stream);
  return hipErrorInvalidValue;
}

}  // namespace mppi
