// Shared by the FeatureAttention rollout kernels (kernels_fa.hip: general FA kernels; kernels_fa_small.hip: the
// small-net kernel, compiled separately so it can take its own codegen flags, build.py PER_FILE_FLAGS).
#pragma once
#include <hip/hip_runtime.h>

#include "costs.h"
#include "mppi_internal.h"

namespace mppi {

// Diagnostic build only (-DMPPI_STAMPS): per-phase s_memtime sums of the horizon loop, accumulated over all waves
// into g_fa_stamps (read by mppi_debug_fa_stamps). The shipped kernel contains none of this.
#ifdef MPPI_STAMPS
constexpr int kNumFaStamps = 8;
static __device__ unsigned long long g_fa_stamps[kNumFaStamps];  // one per translation unit (summed on read)
#define FA_STAMP(i)                                                            \
  do {                                                                         \
    __builtin_amdgcn_sched_barrier(0);                                         \
    unsigned long long t_;                                                     \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory"); \
    __builtin_amdgcn_sched_barrier(0);                                         \
    st_[i] += t_ - tprev_;                                                     \
    tprev_ = t_;                                                               \
  } while (0)
#else
#define FA_STAMP(i) \
  do {              \
  } while (0)
#endif

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;

struct FaArgs {
  const char* img;
  int img_bytes;
  int D, L, G, nx, nu, nlayers;
  int we, be, ge, bte, pos, wout;
  int ln1g[kFaMaxLayers], ln1b[kFaMaxLayers], bqkv[kFaMaxLayers], bo[kFaMaxLayers];
  int ln2g[kFaMaxLayers], ln2b[kFaMaxLayers], b1[kFaMaxLayers], b2[kFaMaxLayers];
  int wqkv[kFaMaxLayers], wo[kFaMaxLayers], w1[kFaMaxLayers], w2[kFaMaxLayers];
  float enc_mw, enc_mb, enc_vw, enc_cwb, enc_vb, b_out;
  int vec_lds;  // bytes of the image's fp32-vector prefix staged in LDS (0: read from L2)
  int s_wqkv[kFaMaxLayers], s_w1[kFaMaxLayers], s_w2[kFaMaxLayers];  // fa_small_kernel image
  int s_c1, s_c2;  // fa_small_kernel: centred, gamma-scaled encoding weight / bias vectors
  int s_bqkv[kFaMaxLayers], s_b1[kFaMaxLayers];  // fa_small_kernel: biases of the LayerNorm-folded GEMMs
};

// sum over the 4 lane groups (lanes n, n+16, n+32, n+48), result in every lane
__device__ __forceinline__ float fa_group_sum(float v) {
  auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  const float s = __uint_as_float(p[0]) + __uint_as_float(p[1]);
  auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(s), __float_as_uint(s), false, false);
  return __uint_as_float(q[0]) + __uint_as_float(q[1]);
}
// two group sums in one chain of 3 swaps (rows = 16-lane groups): swap16(a, b), add -> rows hold (a01, b01, a23,
// b23); swap32, add -> (A, B, A, B); swap16 -> A and B in every lane (2 fa_group_sum: 4 swaps, 4 adds)
__device__ __forceinline__ void fa_group_sum2(float& a, float& b) {
  auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b), false, false);
  const float t = __uint_as_float(p[0]) + __uint_as_float(p[1]);
  auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(t), __float_as_uint(t), false, false);
  const float u = __uint_as_float(q[0]) + __uint_as_float(q[1]);
  auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(u), __float_as_uint(u), false, false);
  a = __uint_as_float(r[0]);
  b = __uint_as_float(r[1]);
}

// max over the 4 lane groups (lanes n, n+16, n+32, n+48), result in every lane
__device__ __forceinline__ float fa_group_max(float v) {
  auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  const float s = fmaxf(__uint_as_float(p[0]), __uint_as_float(p[1]));
  auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(s), __float_as_uint(s), false, false);
  return fmaxf(__uint_as_float(q[0]), __uint_as_float(q[1]));
}

// running cost of one sample from its state row (compile-time gather per kind: no scratch)
template <int KIND>
__device__ __forceinline__ float fa_cost_t(const float* x, float u0, float usq, const float* cx, int t1) {
  constexpr CostIdx ci = cost_idx(KIND);
  float v[kCostMaxIdx];
#pragma unroll
  for (int i = 0; i < ci.n; ++i) v[i] = x[ci.idx[i]];
  return cost_eval_t<KIND>(v, u0, usq, cx, t1);
}
// t1: the reference's 1-based rollout step (the terminal term passes H)
__device__ __forceinline__ float fa_cost(int kind, const float* x, float u0, float usq, const float* cx, int t1) {
  switch (kind) {
    case MPPI_COST_CARTPOLE: return fa_cost_t<MPPI_COST_CARTPOLE>(x, u0, usq, cx, t1);
    case MPPI_COST_CARTPOLE_EST: return fa_cost_t<MPPI_COST_CARTPOLE_EST>(x, u0, usq, cx, t1);
    case MPPI_COST_HUMANOID_V3: return fa_cost_t<MPPI_COST_HUMANOID_V3>(x, u0, usq, cx, t1);
    case MPPI_COST_HUMANOID_V1: return fa_cost_t<MPPI_COST_HUMANOID_V1>(x, u0, usq, cx, t1);
    case MPPI_COST_QUAD_JL: return fa_cost_t<MPPI_COST_QUAD_JL>(x, u0, usq, cx, t1);
    default: return fa_cost_t<MPPI_COST_QUAD_EST>(x, u0, usq, cx, t1);
  }
}

// kernels_fa_small.hip
hipError_t launch_fa_small(const SolveArgs& a, const FaArgs& fa, hipStream_t stream);
#ifdef MPPI_STAMPS
int fa_small_stamps(unsigned long long* out, int reset);
#endif

}  // namespace mppi
