// Learned-dynamics MPPI rollout: x_{t+1} = x_t + net([x_t, u_t]) for every (solve, sample), the H loop
// inside the kernel, cost accumulated in registers.  Replaces the per-horizon-step torch launch chain of
// src/cartpole_mppi_estimator.py:84-119 / src/quadruped_mppi_estimator.py:67-78 (net = learning/model.py)
// and the K x H mj_step calls of src/Humanoid_mppi_v3.jl:131-150.
//
// Mapping (DESIGN.md "fc-stack rollout"):
//   * one wave = 16 samples of one solve; lane l: sample n = l & 15, lane group g = l >> 4.
//   * every activation lives in the MFMA C/D layout of v_mfma_f32_16x16x32_bf16: m-tile mt, register r
//     holds feature 16*mt + 4*g + r of sample n.  The next layer consumes it as its B operand with no
//     lane movement: bf16 B k-step ks = D tiles {2ks, 2ks+1}, element j <-> feature 32ks+16(j>>2)+4g+(j&3);
//     the host packs the weight (A operand) fragments in that permuted k order (mppi_nets.cpp).
//   * bf16: the packed weight image (<= 120 KiB) is copied to LDS once per block and read as one
//     ds_read_b128 per lane per MFMA; bias, LayerNorm and the state stay fp32.
//   * fp32 (parity mode): v_mfma_f32_16x16x4_f32, each D register (mt, r) is one 4-deep k-step;
//     the fp32 image (> LDS) is read from L2.
//   * state x (64 slots, fp32) is the last layer's D layout, so x += dx is lane-local.
//   * a sample's features span its 4 lanes {n, n+16, n+32, n+48}: sums over them and moves between
//     them use v_permlane16_swap / v_permlane32_swap (VALU, no LDS round trip).
#include <hip/hip_runtime.h>

#include "costs.h"
#include "mppi_internal.h"

namespace mppi {

// Diagnostic build only (-DMPPI_STAMPS): per-segment s_memtime sums of the horizon loop, accumulated over all
// waves into g_stamps (read by mppi_debug_stamps). The shipped kernel contains none of this.
#ifdef MPPI_STAMPS
constexpr int kNumStamps = 8;
__device__ unsigned long long g_stamps[kNumStamps];
#define STAMP(i)                                                               \
  do {                                                                         \
    __builtin_amdgcn_sched_barrier(0);                                         \
    unsigned long long t_;                                                     \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory"); \
    __builtin_amdgcn_sched_barrier(0);                                         \
    st_[i] += t_ - tprev_;                                                     \
    tprev_ = t_;                                                               \
  } while (0)
#else
#define STAMP(i) \
  do {           \
  } while (0)
#endif

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

// Network shapes in m-tiles of 16 rows. IN_T input tiles = state slots (4) [+ control slots (2)].
// State slot of state index i: i < QP ? i : 32 + (i - QP)  (CA: qpos | qvel halves; MLP: identity).
template <int ARCH>
struct Arch;
template <>
struct Arch<kArchCA> {  // folded CrossAttentionStatePredictor(28, 27, 21, 128), learning/model.py:157-202
  static constexpr int NL = 3, IN_T = 4, MT0 = 16, MT1 = 8, MT2 = 4, MT3 = 4;
  static constexpr bool LN0 = true;
  static constexpr int BLOCKS0 = 2;  // block-diagonal: qpos slots -> rows [0,128), qvel slots -> [128,256)
  static constexpr int QP = 28;
};
template <>
struct Arch<kArchMLP> {  // MLPStatePredictor(nx, nu, 128, hidden_layers=2), learning/model.py:6-46
  static constexpr int NL = 4, IN_T = 6, MT0 = 8, MT1 = 8, MT2 = 8, MT3 = 4;
  static constexpr bool LN0 = false;
  static constexpr int BLOCKS0 = 1;
  static constexpr int QP = 64;
};

struct FcArgs {
  const char* img;  // packed image in global memory
  int img_bytes;
  int w_off[4], b_off[4];
  int lng_off, lnb_off, ln_n;
  int qp, qv;  // state slots: x[0, qp) -> [0, qp); x[qp, qp+qv) -> [32, 32+qv)
};

// ------------------------------------------------------------------------------------------------ lane groups

// sum over the 4 lanes of a sample (lane groups 0..3), result in every lane; order (g0+g1)+(g2+g3).
__device__ __forceinline__ float group_sum(float v) {
  auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  const float s = __uint_as_float(p[0]) + __uint_as_float(p[1]);
  auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(s), __float_as_uint(s), false, false);
  return __uint_as_float(q[0]) + __uint_as_float(q[1]);
}

// value held by lane group GO of this sample, broadcast to all 4 lane groups.
template <int GO>
__device__ __forceinline__ float group_bcast(float v) {
  auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  const unsigned h = p[GO & 1];
  auto q = __builtin_amdgcn_permlane32_swap(h, h, false, false);
  return __uint_as_float(q[GO >> 1]);
}

// ------------------------------------------------------------------------------------------------ layers

// bf16: out = W * in + b ; W fragments in LDS at w (one bf16x8 per lane per (mt, ks)).
// `lane` is made opaque once per horizon step by the caller (asm barrier) so the compiler cannot hoist
// the loop-invariant fragment loads out of the H loop (it would then spill ~400 VGPRs of weights).
template <int MTO, int MTI, int BLOCKS>
__device__ __forceinline__ void layer_bf16(f32x4 (&out)[MTO], const f32x4 (&in)[MTI], const bf16x8* __restrict__ w,
                                           const float* __restrict__ bias, int lane, int g) {
  constexpr int KS = MTI / 2;
  bf16x8 bop[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      bop[ks][j] = (__bf16)in[2 * ks][j];
      bop[ks][4 + j] = (__bf16)in[2 * ks + 1][j];
    }
  }
#pragma unroll
  for (int mt = 0; mt < MTO; ++mt) out[mt] = *reinterpret_cast<const f32x4*>(bias + 16 * mt + 4 * g);
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
    for (int mt = 0; mt < MTO; ++mt) {
      if (BLOCKS == 1 || (mt / (MTO / BLOCKS)) == (ks / (KS / BLOCKS)))
        out[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[(mt * KS + ks) * 64 + lane], bop[ks], out[mt], 0, 0, 0);
    }
  }
}

// fp32: exact-f32 MFMA; W fragments [mt][mi][r][lane] floats in global memory (L2-resident).
template <int MTO, int MTI, int BLOCKS>
__device__ __forceinline__ void layer_f32(f32x4 (&out)[MTO], const f32x4 (&in)[MTI], const float* __restrict__ w,
                                          const float* __restrict__ bias, int lane, int g) {
#pragma unroll
  for (int mt = 0; mt < MTO; ++mt) out[mt] = *reinterpret_cast<const f32x4*>(bias + 16 * mt + 4 * g);
#pragma unroll
  for (int mi = 0; mi < MTI; ++mi) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int mt = 0; mt < MTO; ++mt) {
        if (BLOCKS == 1 || (mt / (MTO / BLOCKS)) == (mi / (MTI / BLOCKS)))
          out[mt] = __builtin_amdgcn_mfma_f32_16x16x4f32(w[((mt * MTI + mi) * 4 + r) * 64 + lane], in[mi][r], out[mt],
                                                         0, 0, 0);
      }
    }
  }
}

template <int MT>
__device__ __forceinline__ void relu(f32x4 (&h)[MT]) {
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r) h[mt][r] = fmaxf(h[mt][r], 0.0f);
}

// LayerNorm over all 16*MT features of each sample (two-pass, like torch), then ReLU.
template <int MT>
__device__ __forceinline__ void layernorm_relu(f32x4 (&h)[MT], const float* __restrict__ gam,
                                               const float* __restrict__ bet, int g) {
  float s = 0.0f;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) s += (h[mt][0] + h[mt][1]) + (h[mt][2] + h[mt][3]);
  constexpr float inv_n = 1.0f / (16.0f * MT);
  const float mean = group_sum(s) * inv_n;
  float v = 0.0f;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float d = h[mt][r] - mean;
      v = fmaf(d, d, v);
    }
  const float rstd = 1.0f / sqrtf(group_sum(v) * inv_n + 1e-5f);
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const f32x4 ga = *reinterpret_cast<const f32x4*>(gam + 16 * mt + 4 * g);
    const f32x4 be = *reinterpret_cast<const f32x4*>(bet + 16 * mt + 4 * g);
#pragma unroll
    for (int r = 0; r < 4; ++r) h[mt][r] = fmaxf(fmaf((h[mt][r] - mean) * rstd, ga[r], be[r]), 0.0f);
  }
}

// Gather the state entries cost COST reads (cost_idx order) into every lane of the sample.
template <int COST, int QP>
__device__ __forceinline__ void gather_cost_inputs(const f32x4 (&x)[4], float* v) {
  constexpr CostIdx ci = cost_idx(COST);
#pragma unroll
  for (int i = 0; i < ci.n; ++i) {
    const int xi = ci.idx[i];
    const int slot = xi < QP ? xi : 32 + (xi - QP);
    const float r = x[slot >> 4][slot & 3];
    switch ((slot >> 2) & 3) {  // compile-time after unrolling
      case 0: v[i] = group_bcast<0>(r); break;
      case 1: v[i] = group_bcast<1>(r); break;
      case 2: v[i] = group_bcast<2>(r); break;
      default: v[i] = group_bcast<3>(r); break;
    }
  }
}

// ------------------------------------------------------------------------------------------------ kernel

template <int ARCH, int PREC, int COST>
// waves_per_eu(1,1): the LDS weight image admits one block (<= 4 waves) per CU, so one wave per SIMD is the real
// occupancy; without it hipcc minimises VGPRs for occupancy and serialises every ds_read -> MFMA.
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void fc_rollout_kernel(SolveArgs a,
                                                                                                   FcArgs net) {
  using A = Arch<ARCH>;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  if constexpr (PREC == MPPI_PREC_BF16) {
    const int4* src = reinterpret_cast<const int4*>(net.img);
    int4* dst = reinterpret_cast<int4*>(lds);
    for (int i = threadIdx.x; i < (net.img_bytes >> 4); i += blockDim.x) dst[i] = src[i];
    __syncthreads();
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) *a.status = 0u;  // per-solve status word (read after the reduce)
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4;
  const int gw = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int waves_per_solve = a.Kp >> 4;
  if (gw >= a.B * waves_per_solve) return;
  const int b = gw / waves_per_solve;
  const int k = (gw - b * waves_per_solve) * 16 + (lane & 15);

  const char* img;
  if constexpr (PREC == MPPI_PREC_BF16)
    img = lds;
  else
    img = net.img;
  auto W = [&](int l) { return img + net.w_off[l]; };
  auto Bi = [&](int l) { return reinterpret_cast<const float*>(img + net.b_off[l]); };

  // initial state in slot layout
  f32x4 x[4];
  const float* x0 = a.x0 + (long)b * a.nx;
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int s = 16 * mt + 4 * g + r;
      const int src = s < 32 ? (s < net.qp ? s : -1) : (s - 32 < net.qv ? net.qp + s - 32 : -1);
      x[mt][r] = src >= 0 ? x0[src] : 0.0f;
    }

  float cx[MPPI_CTX_MAX];
#pragma unroll
  for (int i = 0; i < MPPI_CTX_MAX; ++i) cx[i] = a.ctx ? a.ctx[(long)b * MPPI_CTX_MAX + i] : a.ctx_default[i];
  const float* Ub = a.U + (long)b * a.nu * a.H;
  const float* eb = a.noise + (long)b * a.nu * a.H * a.Kp + k;
  const long ustride = (long)a.H * a.Kp;
  float cost = 0.0f;
  float v[kCostMaxIdx];

  // control slots of this lane group: {4g..4g+3, 16+4g..16+4g+3} (u tiles 0,1 of the D layout).
  // Loads are unconditional (pad slots read row nu-1 and are zeroed by a mask): a conditional load makes
  // hipcc branch around it and wait vmcnt(0) per element, serialising the prefetch.
  float umask[8];
  int urow[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int us = (j < 4) ? 4 * g + j : 16 + 4 * g + (j - 4);
    umask[j] = us < a.nu ? 1.0f : 0.0f;
    urow[j] = us < a.nu ? us : a.nu - 1;
  }
  auto load_u = [&](int t, f32x4 (&u)[2]) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float uv = Ub[urow[j] * a.H + t] + eb[urow[j] * ustride + (long)t * a.Kp];
      u[j >> 2][j & 3] = uv * umask[j];
    }
  };
  f32x4 un[2];
  load_u(0, un);

#ifdef MPPI_STAMPS
  unsigned long long st_[kNumStamps] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long tprev_ = __builtin_amdgcn_s_memtime();
#endif
  for (int t = 0; t < a.H; ++t) {
    STAMP(0);
    int ol = lane, og = g;  // opaque copies: weight/bias addresses are re-derived every step (no LICM)
    asm volatile("" : "+v"(ol), "+v"(og));
    f32x4 u[2] = {un[0], un[1]};
    load_u(t + 1 < a.H ? t + 1 : t, un);  // prefetch the next step's controls (unconditional: no vmcnt(0) at a join)
    if (a.ctrl_clamp > 0.0f) {
#pragma unroll
      for (int j = 0; j < 8; ++j) u[j >> 2][j & 3] = fminf(a.ctrl_clamp, fmaxf(-a.ctrl_clamp, u[j >> 2][j & 3]));
    }
    float usq = 0.0f;
#pragma unroll
    for (int j = 0; j < 8; ++j) usq = fmaf(u[j >> 2][j & 3], u[j >> 2][j & 3], usq);
    usq = group_sum(usq);

    STAMP(1);  // segment 1: control loads/prefetch, clamp, |u|^2
    // ---- network: dx = net([x, u])
    f32x4 in0[A::IN_T];
#pragma unroll
    for (int i = 0; i < 4; ++i) in0[i] = x[i];
    if constexpr (A::IN_T == 6) {
      in0[4] = u[0];
      in0[5] = u[1];
    }
    f32x4 h0[A::MT0];
    if constexpr (PREC == MPPI_PREC_BF16)
      layer_bf16<A::MT0, A::IN_T, A::BLOCKS0>(h0, in0, reinterpret_cast<const bf16x8*>(W(0)), Bi(0), ol, og);
    else
      layer_f32<A::MT0, A::IN_T, A::BLOCKS0>(h0, in0, reinterpret_cast<const float*>(W(0)), Bi(0), ol, og);
    STAMP(2);  // segment 2: layer 0 MFMAs
    if constexpr (A::LN0)
      layernorm_relu<A::MT0>(h0, reinterpret_cast<const float*>(img + net.lng_off),
                             reinterpret_cast<const float*>(img + net.lnb_off), og);
    else
      relu<A::MT0>(h0);
    STAMP(3);  // segment 3: LayerNorm/ReLU
    f32x4 h1[A::MT1];
    if constexpr (PREC == MPPI_PREC_BF16)
      layer_bf16<A::MT1, A::MT0, 1>(h1, h0, reinterpret_cast<const bf16x8*>(W(1)), Bi(1), ol, og);
    else
      layer_f32<A::MT1, A::MT0, 1>(h1, h0, reinterpret_cast<const float*>(W(1)), Bi(1), ol, og);
    STAMP(4);  // segment 4: layer 1
    f32x4 dx[4];
    relu<A::MT1>(h1);
    if constexpr (A::NL == 3) {
      if constexpr (PREC == MPPI_PREC_BF16)
        layer_bf16<4, A::MT1, 1>(dx, h1, reinterpret_cast<const bf16x8*>(W(2)), Bi(2), ol, og);
      else
        layer_f32<4, A::MT1, 1>(dx, h1, reinterpret_cast<const float*>(W(2)), Bi(2), ol, og);
    } else {
      f32x4 h2[A::MT2];
      if constexpr (PREC == MPPI_PREC_BF16)
        layer_bf16<A::MT2, A::MT1, 1>(h2, h1, reinterpret_cast<const bf16x8*>(W(2)), Bi(2), ol, og);
      else
        layer_f32<A::MT2, A::MT1, 1>(h2, h1, reinterpret_cast<const float*>(W(2)), Bi(2), ol, og);
      relu<A::MT2>(h2);
      if constexpr (PREC == MPPI_PREC_BF16)
        layer_bf16<4, A::MT2, 1>(dx, h2, reinterpret_cast<const bf16x8*>(W(3)), Bi(3), ol, og);
      else
        layer_f32<4, A::MT2, 1>(dx, h2, reinterpret_cast<const float*>(W(3)), Bi(3), ol, og);
    }
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) x[mt] += dx[mt];
    STAMP(5);  // segment 5: remaining layers + state update

    // ---- running cost on (x_{t+1}, u_t)
    gather_cost_inputs<COST, A::QP>(x, v);
    const float u0 = group_bcast<0>(u[0][0]);  // control 0 lives in lane group 0, slot 0
    cost += cost_eval_t<COST>(v, u0, usq, cx);
  }
  STAMP(6);  // segment 6: cost gather + eval (last step)
#ifdef MPPI_STAMPS
  if (lane == 0)
    for (int i = 0; i < kNumStamps; ++i) atomicAdd(&g_stamps[i], st_[i]);
#endif
  if (a.terminal_weight != 0.0f) cost += a.terminal_weight * cost_eval_t<COST>(v, 0.0f, 0.0f, cx);
  if (g == 0 && k < a.K) a.costs[(long)b * a.Kp + k] = isfinite(cost) ? cost : INFINITY;
}

#ifdef MPPI_STAMPS
extern "C" int mppi_debug_stamps(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * kNumStamps) != hipSuccess) return -2;
  if (reset) {
    unsigned long long z[kNumStamps] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), z, sizeof(z)) != hipSuccess) return -2;
  }
  return 0;
}
#endif

template <int ARCH, int PREC, int COST>
static hipError_t launch_t(const SolveArgs& a, const FcArgs& fa, int grid, int wpb, size_t lds, hipStream_t stream) {
  auto kern = fc_rollout_kernel<ARCH, PREC, COST>;
  // > 64 KiB of dynamic LDS must be opted into per kernel (gfx950 has 160 KiB per CU).
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * wpb), lds, stream, a, fa);
  return hipGetLastError();
}

template <int ARCH, int PREC>
static hipError_t launch_cost(const SolveArgs& a, const FcArgs& fa, int grid, int wpb, size_t lds, hipStream_t s) {
  switch (a.cost_kind) {
    case MPPI_COST_HUMANOID_V3: return launch_t<ARCH, PREC, MPPI_COST_HUMANOID_V3>(a, fa, grid, wpb, lds, s);
    case MPPI_COST_QUAD_JL: return launch_t<ARCH, PREC, MPPI_COST_QUAD_JL>(a, fa, grid, wpb, lds, s);
    case MPPI_COST_QUAD_EST: return launch_t<ARCH, PREC, MPPI_COST_QUAD_EST>(a, fa, grid, wpb, lds, s);
    case MPPI_COST_CARTPOLE_EST: return launch_t<ARCH, PREC, MPPI_COST_CARTPOLE_EST>(a, fa, grid, wpb, lds, s);
    case MPPI_COST_CARTPOLE: return launch_t<ARCH, PREC, MPPI_COST_CARTPOLE>(a, fa, grid, wpb, lds, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_fc_rollout(const SolveArgs& a, const FcNet& n, hipStream_t stream) {
  FcArgs fa;
  fa.img = reinterpret_cast<const char*>(n.d_img);
  fa.img_bytes = n.img_bytes;
  for (int i = 0; i < 4; ++i) {
    fa.w_off[i] = n.w_off[i];
    fa.b_off[i] = n.b_off[i];
  }
  fa.lng_off = n.lng_off;
  fa.lnb_off = n.lnb_off;
  fa.ln_n = n.ln_n;
  fa.qp = n.qp;
  fa.qv = n.qv;
  const int total_waves = a.B * (a.Kp >> 4);
  // bf16: one block per CU (the LDS weight image admits one); spread the waves over all CUs.
  int wpb = (total_waves + 255) / 256;
  wpb = wpb < 1 ? 1 : (wpb > 4 ? 4 : wpb);
  const int grid = (total_waves + wpb - 1) / wpb;
  const size_t lds = n.precision == MPPI_PREC_BF16 ? (size_t)n.img_bytes : 0;
  if (n.arch == kArchCA) {
    if (a.cost_kind != MPPI_COST_HUMANOID_V3) return hipErrorInvalidValue;  // CA is built for the humanoid
    return n.precision == MPPI_PREC_BF16
               ? launch_t<kArchCA, MPPI_PREC_BF16, MPPI_COST_HUMANOID_V3>(a, fa, grid, wpb, lds, stream)
               : launch_t<kArchCA, MPPI_PREC_FP32, MPPI_COST_HUMANOID_V3>(a, fa, grid, wpb, lds, stream);
  }
  if (n.arch == kArchMLP)
    return n.precision == MPPI_PREC_BF16 ? launch_cost<kArchMLP, MPPI_PREC_BF16>(a, fa, grid, wpb, lds, stream)
                                         : launch_cost<kArchMLP, MPPI_PREC_FP32>(a, fa, grid, wpb, lds, stream);
  return hipErrorInvalidValue;
}

}  // namespace mppi
