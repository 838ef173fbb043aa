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
#include <hip/hip_runtime.h>

#include "costs.h"
#include "mppi_internal.h"

namespace mppi {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

// Network shapes in m-tiles of 16 rows. IN_T input tiles = state slots (4) [+ control slots (2)].
template <int ARCH>
struct Arch;
template <>
struct Arch<kArchCA> {  // folded CrossAttentionStatePredictor(28, 27, 21, 128), learning/model.py:157-202
  static constexpr int NL = 3, IN_T = 4, MT0 = 16, MT1 = 8, MT2 = 4, MT3 = 4;
  static constexpr bool LN0 = true;
  static constexpr int BLOCKS0 = 2;  // block-diagonal: qpos slots -> rows [0,128), qvel slots -> [128,256)
};
template <>
struct Arch<kArchMLP> {  // MLPStatePredictor(nx, nu, 128, hidden_layers=2), learning/model.py:6-46
  static constexpr int NL = 4, IN_T = 6, MT0 = 8, MT1 = 8, MT2 = 8, MT3 = 4;
  static constexpr bool LN0 = false;
  static constexpr int BLOCKS0 = 1;
};

struct FcArgs {
  const char* img;  // packed image in global memory
  int img_bytes;
  int w_off[4], b_off[4];
  int lng_off, lnb_off, ln_n;
  // state slots: x[0, qp) -> slots [0, qp); x[qp, qp+qv) -> slots [32, 32+qv); other slots are 0.
  int qp, qv;
};

__device__ __forceinline__ int x_slot_of(const FcArgs& n, int i) { return i < n.qp ? i : 32 + (i - n.qp); }

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

// LayerNorm over the ln_n real features of each sample (two-pass, like torch), then ReLU.
// A sample's features are spread over its 4 lanes {n, n+16, n+32, n+48}.
template <int MT>
__device__ __forceinline__ void layernorm_relu(f32x4 (&h)[MT], const float* __restrict__ gam,
                                               const float* __restrict__ bet, int ln_n, int g) {
  float s = 0.0f;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) s += (h[mt][0] + h[mt][1]) + (h[mt][2] + h[mt][3]);
  s += __shfl_xor(s, 16);
  s += __shfl_xor(s, 32);
  const float inv_n = 1.0f / (float)ln_n;
  const float mean = s * inv_n;
  float v = 0.0f;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float d = (16 * mt + 4 * g + r < ln_n) ? h[mt][r] - mean : 0.0f;
      v = fmaf(d, d, v);
    }
  v += __shfl_xor(v, 16);
  v += __shfl_xor(v, 32);
  const float rstd = 1.0f / sqrtf(v * inv_n + 1e-5f);
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const f32x4 ga = *reinterpret_cast<const f32x4*>(gam + 16 * mt + 4 * g);
    const f32x4 be = *reinterpret_cast<const f32x4*>(bet + 16 * mt + 4 * g);
#pragma unroll
    for (int r = 0; r < 4; ++r) h[mt][r] = fmaxf(fmaf((h[mt][r] - mean) * rstd, ga[r], be[r]), 0.0f);
  }
}

// Register (mt, r) of x selected by a wave-uniform index (lowered to scalar branches, no scratch).
__device__ __forceinline__ float x_reg(const f32x4 (&x)[4], int mtr) {
  switch (mtr) {
    case 0: return x[0][0]; case 1: return x[0][1]; case 2: return x[0][2]; case 3: return x[0][3];
    case 4: return x[1][0]; case 5: return x[1][1]; case 6: return x[1][2]; case 7: return x[1][3];
    case 8: return x[2][0]; case 9: return x[2][1]; case 10: return x[2][2]; case 11: return x[2][3];
    case 12: return x[3][0]; case 13: return x[3][1]; case 14: return x[3][2]; default: return x[3][3];
  }
}

// Gather the state entries the cost reads (cost_idx order) into every lane of the sample.
__device__ __forceinline__ void gather_cost_inputs(const f32x4 (&x)[4], const CostIdx& ci, const FcArgs& net,
                                                   int lane, float* v) {
#pragma unroll
  for (int i = 0; i < kCostMaxIdx; ++i) {
    if (i < ci.n) {
      const int slot = x_slot_of(net, ci.idx[i]);
      const float r = x_reg(x, (slot >> 4) * 4 + (slot & 3));
      v[i] = __shfl(r, (lane & 15) + 16 * ((slot >> 2) & 3));
    }
  }
}

// ------------------------------------------------------------------------------------------------ kernel

template <int ARCH, int PREC>
__global__ __launch_bounds__(512) void fc_rollout_kernel(SolveArgs a, FcArgs net) {
  using A = Arch<ARCH>;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  if constexpr (PREC == MPPI_PREC_BF16) {
    const int4* src = reinterpret_cast<const int4*>(net.img);
    int4* dst = reinterpret_cast<int4*>(lds);
    for (int i = threadIdx.x; i < (net.img_bytes >> 4); i += blockDim.x) dst[i] = src[i];
    __syncthreads();
  }
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
  const CostIdx ci = cost_idx(a.cost_kind);
  const float* Ub = a.U + (long)b * a.nu * a.H;
  const float* eb = a.noise + (long)b * a.nu * a.H * a.Kp + k;
  const long ustride = (long)a.H * a.Kp;
  float cost = 0.0f;
  float v[kCostMaxIdx];

  // control slots of this lane group: {4g..4g+3, 16+4g..16+4g+3} (u tiles 0,1 of the D layout)
  auto load_u = [&](int t, f32x4 (&u)[2]) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int us = (j < 4) ? 4 * g + j : 16 + 4 * g + (j - 4);
      float uv = 0.0f;
      if (us < a.nu) uv = Ub[us * a.H + t] + eb[us * ustride + (long)t * a.Kp];
      u[j >> 2][j & 3] = uv;
    }
  };
  f32x4 un[2];
  load_u(0, un);

  for (int t = 0; t < a.H; ++t) {
    int ol = lane, og = g;  // opaque copies: weight/bias addresses are re-derived every step (no LICM)
    asm volatile("" : "+v"(ol), "+v"(og));
    f32x4 u[2] = {un[0], un[1]};
    if (t + 1 < a.H) load_u(t + 1, un);  // prefetch the next step's controls (noise rows)
    if (a.ctrl_clamp > 0.0f) {
#pragma unroll
      for (int j = 0; j < 8; ++j) u[j >> 2][j & 3] = fminf(a.ctrl_clamp, fmaxf(-a.ctrl_clamp, u[j >> 2][j & 3]));
    }
    float usq = 0.0f;
#pragma unroll
    for (int j = 0; j < 8; ++j) usq = fmaf(u[j >> 2][j & 3], u[j >> 2][j & 3], usq);
    usq += __shfl_xor(usq, 16);
    usq += __shfl_xor(usq, 32);

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
    if constexpr (A::LN0)
      layernorm_relu<A::MT0>(h0, reinterpret_cast<const float*>(img + net.lng_off),
                             reinterpret_cast<const float*>(img + net.lnb_off), net.ln_n, og);
    else
      relu<A::MT0>(h0);
    f32x4 h1[A::MT1];
    if constexpr (PREC == MPPI_PREC_BF16)
      layer_bf16<A::MT1, A::MT0, 1>(h1, h0, reinterpret_cast<const bf16x8*>(W(1)), Bi(1), ol, og);
    else
      layer_f32<A::MT1, A::MT0, 1>(h1, h0, reinterpret_cast<const float*>(W(1)), Bi(1), ol, og);
    f32x4 dx[4];
    if constexpr (A::NL == 3) {
      relu<A::MT1>(h1);
      if constexpr (PREC == MPPI_PREC_BF16)
        layer_bf16<4, A::MT1, 1>(dx, h1, reinterpret_cast<const bf16x8*>(W(2)), Bi(2), ol, og);
      else
        layer_f32<4, A::MT1, 1>(dx, h1, reinterpret_cast<const float*>(W(2)), Bi(2), ol, og);
    } else {
      relu<A::MT1>(h1);
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

    // ---- running cost on (x_{t+1}, u_t)
    gather_cost_inputs(x, ci, net, lane, v);
    float u0 = __shfl(u[0][0], lane & 15);  // control 0 lives in group 0, slot 0
    cost += cost_eval(a.cost_kind, v, u0, usq, cx);
  }
  if (a.terminal_weight != 0.0f) cost += a.terminal_weight * cost_eval(a.cost_kind, v, 0.0f, 0.0f, cx);
  if (g == 0 && k < a.K) a.costs[(long)b * a.Kp + k] = isfinite(cost) ? cost : INFINITY;
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
  wpb = wpb < 1 ? 1 : (wpb > 8 ? 8 : wpb);
  if (n.precision != MPPI_PREC_BF16) wpb = wpb > 4 ? 4 : wpb;
  const int grid = (total_waves + wpb - 1) / wpb;
  const size_t lds = n.precision == MPPI_PREC_BF16 ? (size_t)n.img_bytes : 0;
  const dim3 blk(64 * wpb);
  if (n.arch == kArchCA && n.precision == MPPI_PREC_BF16)
    hipLaunchKernelGGL((fc_rollout_kernel<kArchCA, MPPI_PREC_BF16>), dim3(grid), blk, lds, stream, a, fa);
  else if (n.arch == kArchCA)
    hipLaunchKernelGGL((fc_rollout_kernel<kArchCA, MPPI_PREC_FP32>), dim3(grid), blk, lds, stream, a, fa);
  else if (n.arch == kArchMLP && n.precision == MPPI_PREC_BF16)
    hipLaunchKernelGGL((fc_rollout_kernel<kArchMLP, MPPI_PREC_BF16>), dim3(grid), blk, lds, stream, a, fa);
  else if (n.arch == kArchMLP)
    hipLaunchKernelGGL((fc_rollout_kernel<kArchMLP, MPPI_PREC_FP32>), dim3(grid), blk, lds, stream, a, fa);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

}  // namespace mppi
