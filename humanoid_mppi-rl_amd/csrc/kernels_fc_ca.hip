// Learned-dynamics MPPI rollout, CrossAttention net (the humanoid surrogate, BASELINE configs #4 / #5): the CA
// instantiation of fc_rollout_kernel (fc_rollout.h), built with -fno-slp-vectorize (build.py PER_FILE_FLAGS).
#include "fc_rollout.h"

namespace mppi {

hipError_t launch_fc_ca(const SolveArgs& a, const FcArgs& fa, int precision, hipStream_t stream) {
  // bf16: the per-wave kernel for batches with >= 6 tiles per CU (fc_wave_ns), else the M-split kernel below.  The
  // A/B-only library (MPPI_AB_ARMS=1 build.py, csrc/ab/) adds the layer-pipelined kernel when forced (MPPI_FC_PIPE=1).
#ifdef MPPI_AB_ARMS
  if (precision == MPPI_PREC_BF16 && fa.lds_bytes == 0 && fc_pipe_wanted(a)) return launch_fc_pipe(a, fa, stream);
#endif
  // the engine's fp16-form probe (mppi_api.hip x3_probe): fc_wave32_x3p_kernel whatever the batch
  if (precision == MPPI_PREC_BF16X3 && fa.x3_route == 1) {
    if (fa.w32x3_off < 0 || fa.ln_n != 256 || a.Kp < 32 || a.Kp % 32 != 0 || a.nu < 20 || a.nu > 22)
      return hipErrorInvalidValue;
    return launch_fc_wave_x3p(a, fa, stream);
  }
  if (precision == MPPI_PREC_BF16X3 && fa.x3_route == 2) {  // ... and fc_rollout_kernel_x3h, the shards' fp16 form
    if (!fc_x3h_wanted(a, fa)) return hipErrorInvalidValue;
    return launch_fc_x3h(a, fa, stream);
  }
  if (precision == MPPI_PREC_BF16X3 && fc_wave_x3_wanted(a, fa)) return launch_fc_wave_x3(a, fa, stream);
  // split bf16 below that: the M-split kernels -- the fp16 form at one group per block and two blocks per CU
  // (kernels_fc_x3h.hip), the two-product bf16 layer 1 at two groups per block (kernels_fc_x3d.hip)
  if (precision == MPPI_PREC_BF16X3 && fc_x3d_wanted(a, fa))
    return fc_x3h_wanted(a, fa) ? launch_fc_x3h(a, fa, stream) : launch_fc_x3d(a, fa, stream);
  if (precision == MPPI_PREC_BF16 && fa.lds_bytes == 0 && a.nu <= 24) {
    const int ns = fc_wave_ns(a, fa);
    if (ns) return launch_fc_wave(a, fa, ns, stream);
  }
  if (a.cost_kind == MPPI_COST_HUMANOID_V1) return launch_prec<kArchCA, MPPI_COST_HUMANOID_V1>(a, fa, precision, stream);
  return launch_prec<kArchCA, MPPI_COST_HUMANOID_V3>(a, fa, precision, stream);
}

#ifdef MPPI_STAMPS
int fc_ca_stamps(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * kNumStamps) != hipSuccess) return -2;
  if (reset) {
    unsigned long long z[kNumStamps] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), z, sizeof(z)) != hipSuccess) return -2;
  }
  return 0;
}
#endif

}  // namespace mppi
