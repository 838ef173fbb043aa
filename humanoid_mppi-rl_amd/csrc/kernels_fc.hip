// Learned-dynamics MPPI rollout, fc-stack nets: the MLP instantiations of fc_rollout_kernel (fc_rollout.h) and the
// dispatcher (the CA instantiation lives in kernels_fc_ca.hip).
#include "fc_rollout.h"

#include <atomic>
#include <cstdlib>

namespace mppi {

thread_local const char* g_rollout_kernel = "";

int current_device_cus() {
  constexpr int kMaxDev = 64;
  static std::atomic<int> cache[kMaxDev];
  int dev = 0, n = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 256;
  if (dev >= 0 && dev < kMaxDev) {
    const int c = cache[dev].load(std::memory_order_relaxed);
    if (c > 0) return c;
  }
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  if (dev >= 0 && dev < kMaxDev) cache[dev].store(n, std::memory_order_relaxed);
  return n;
}

bool fc_f32_stream() {
  static const bool on = [] {
    const char* e = std::getenv("MPPI_F32_STREAM");
    return e && e[0] == '1';
  }();
  return on;
}

int fc_x3_tiles() {
  const char* e = std::getenv("MPPI_X3_TILES");
  return e ? std::atoi(e) : 2;
}

#ifdef MPPI_AB_ARMS
int fc_wide() {
  static const int on = [] {
    const char* e = std::getenv("MPPI_FC_WIDE");
    return e ? (e[0] == '1' ? 1 : 0) : 0;
  }();
  return on;
}
#endif

hipError_t launch_fc_rollout(const SolveArgs& a, const FcNet& n, hipStream_t stream) {
  if (n.arch == kArchGeneric) return launch_fc_generic(a, n, stream);  // any other fc-stack shape
  FcArgs fa;
  fa.img = reinterpret_cast<const char*>(n.d_img);
  fa.img_bytes = n.img_bytes;
  fa.lds_bytes = n.lds_bytes;
  for (int i = 0; i < 4; ++i) {
    fa.w_off[i] = n.w_off[i];
    fa.b_off[i] = n.b_off[i];
  }
  fa.lnb_off = n.lnb_off;
  fa.ln_n = n.ln_n;
  fa.qp = n.qp;
  fa.qv = n.qv;
  fa.groups_per_block = 1;
  fa.g_off = n.g_off;
  fa.wave = n.wave;
  fa.w32_off = n.w32_off;
  fa.w32_bd = n.w32_bd;
  fa.w0bd_off = n.w0bd_off;
  fa.gbd_off = n.gbd_off;
  fa.w32x3_off = n.w32x3_off;
  fa.w32x3_l1lo_off = n.w32x3_l1lo_off;
  fa.wmx3_off = n.wmx3_off;
  fa.wmx3_lo_off = n.wmx3_lo_off;
  fa.wm32x3_off = n.wm32x3_off;
  fa.wm32x3_lo_off = n.wm32x3_lo_off;
  fa.x3_l1 = n.x3_l1;
  fa.w32f16_off = n.w32f16_off;
  fa.wmf16_off = n.wmf16_off;
  fa.wmf16_x_off = n.wmf16_x_off;
  fa.wmf16_0_off = n.wmf16_0_off;
  fa.wmf16_0b_off = n.wmf16_0b_off;
  fa.x3_f16 = n.x3_f16;
  fa.x3_route = n.x3_route;
  if (n.arch == kArchCA) {
    // the CA kernel is built for the humanoid (qpos 28) with its two costs
    if (a.cost_kind != MPPI_COST_HUMANOID_V3 && a.cost_kind != MPPI_COST_HUMANOID_V1) return hipErrorInvalidValue;
    return launch_fc_ca(a, fa, n.precision, stream);
  }
  if (n.arch == kArchMLP) {
    if (n.precision == MPPI_PREC_BF16 && n.wave && fa.lds_bytes == 0) {  // large batches: the per-wave kernel
      const int ns = fc_wave_mlp_ns(a, fa);
      if (ns) return launch_fc_wave_mlp(a, fa, ns, stream);
    }
    if (n.precision == MPPI_PREC_BF16X3 && fc_wave32_mlp_x3_wanted(a, fa))  // the split per-wave kernels
      return launch_fc_wave32_mlp_x3(a, fa, stream);
    if (n.precision == MPPI_PREC_BF16X3 && fc_wave_mlp_x3_wanted(a, fa))
      return launch_fc_wave_mlp_x3(a, fa, stream);
    return launch_cost<kArchMLP>(a, fa, n.precision, stream);
  }
  return hipErrorInvalidValue;
}


#ifdef MPPI_STAMPS
extern "C" int mppi_debug_stamps(unsigned long long* out, int reset) {  // both fc translation units' sums
  unsigned long long s[kNumStamps];
  if (fc_ca_stamps(s, reset) != 0) return -2;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * kNumStamps) != hipSuccess) return -2;
  for (int i = 0; i < kNumStamps; ++i) out[i] += s[i];
  if (reset) {
    unsigned long long z[kNumStamps] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), z, sizeof(z)) != hipSuccess) return -2;
  }
  return 0;
}
#endif

}  // namespace mppi
