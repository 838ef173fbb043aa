// fc_wave_mlp_x3_kernel (round 5): the split-bf16 (MPPI_PREC_BF16X3, fp32-accurate) per-wave rollout of
// MLPStatePredictor(nx, nu, 128, hidden_layers = 2) (learning/model.py:6-46).  fc_wave_mlp_kernel's organisation
// (kernels_fc_wave.hip: one wave runs all four layers of its 16 samples on 16x16x32 MFMAs, every layer's output packed
// to bf16 as the next layer's B operand with no LDS round trip, 8 waves = 2 per SIMD) with every product as three
// bf16 MFMAs -- W_hi a_hi + W_hi a_lo + W_lo a_hi, fp32 accumulate, the a_lo W_lo term dropped -- and the operands
// (state, controls, activations) split into bf16 hi / lo pairs in registers.  The M-split split kernel it replaces for
// large batches holds its hi / lo weights in registers at one wave per SIMD (config #4 shape, humanoid MLP: 1.56 ms
// per 64-solve rollout).
//   * LDS (144 KiB): the hi fragments of all four layers and the lo fragments of layers 0 and 3 (mppi_nets.cpp
//     pack_image, mlp_x3); the lo fragments of the two hidden layers (64 KiB) stream from L2, LQ positions ahead.
//   * layer 0's bias rides in the MFMA (the b0 pair in pad state slots 62, 63, which hold 1.0: their lo parts are 0);
//     b1, b2, b3 initialise the accumulators.
//   * the running cost's state part through a one-step LDS ring (lane group 0 evaluates its 16 samples every step).
#include <cstdlib>

#include "x3_common.h"

namespace mppi {

namespace {

struct WaveMlpX3Lay {
  static constexpr int WH = 0;                 // hi: W0 (8 m-tiles x 3 k-steps) | W1 (8 x 4) | W2 (8 x 4) | W3 (4 x 4)
  static constexpr int W0L = WH + 104 * 1024;  // lo of W0
  static constexpr int W3L = W0L + 24 * 1024;  // lo of W3
  static constexpr int IMG = W3L + 16 * 1024;  // 144 KiB: one contiguous copy of the image at net.wmx3_off
  static constexpr int B1 = IMG;               // 128 f32
  static constexpr int B2 = B1 + 512;          // 128 f32
  static constexpr int B3 = B2 + 512;          // 64 f32
  static constexpr int RING = B3 + 256;
  static constexpr int WAVES = 8;
  template <int COST>
  static constexpr int ring_bytes() { return 16 * CostChunks<kArchMLP, COST>::HS * 4; }
  template <int COST>
  static constexpr int bytes() { return RING + WAVES * ring_bytes<COST>(); }
};
// hidden-layer lo fragments read this many stream positions ahead (position = one (layer, part, k-step, m-tile))
#ifndef X3M_LQ
#define X3M_LQ 8
#endif

__device__ __forceinline__ f32x4 mma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
// acc += W a, W = wh + wl, a = ah + al (the wl al term dropped)
__device__ __forceinline__ f32x4 mma16x3(const bf16x8& wh, const bf16x8& wl, const bf16x8& ah, const bf16x8& al,
                                         f32x4 acc) {
  acc = mma16(wl, ah, acc);
  acc = mma16(wh, al, acc);
  return mma16(wh, ah, acc);
}
// two 16x16 accumulator tiles (the k-step of the next layer: tile t0's 4 values then t1's) as bf16 hi and lo B operands
__device__ __forceinline__ void split16(const f32x4& t0, const f32x4& t1, bf16x8& hi, bf16x8& lo) {
  u32x4 hw, lw;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float x0 = q < 2 ? t0[2 * q] : t1[2 * q - 4], x1 = q < 2 ? t0[2 * q + 1] : t1[2 * q - 3];
    const unsigned p = pk_bf16(x0, x1);
    hw[q] = p;
    lw[q] = pk_bf16(x0 - __uint_as_float(p << 16), x1 - __uint_as_float(p & 0xFFFF0000u));
  }
  hi = __builtin_bit_cast(bf16x8, hw);
  lo = __builtin_bit_cast(bf16x8, lw);
}
__device__ __forceinline__ f32x4 relu4(f32x4 v) {
#pragma unroll
  for (int r = 0; r < 4; ++r) v[r] = __builtin_amdgcn_fmed3f(v[r], 0.0f, 3.402823466e38f);
  return v;
}

}  // namespace

template <int COST>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2))) void fc_wave_mlp_x3_kernel(SolveArgs a,
                                                                                                     FcArgs net) {
  using Y = WaveMlpX3Lay;
  using CC = CostChunks<kArchMLP, COST>;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const KClock kc = kclock_begin(a);
  if (blockIdx.x == 0 && threadIdx.x == 0) *a.status = 0u;
  const int lane = threadIdx.x & 63, g = lane >> 4, n = lane & 15;
  const int wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  {
    const int4* s0 = reinterpret_cast<const int4*>(net.img + net.wmx3_off);
    int4* d = reinterpret_cast<int4*>(lds);
    stage_lds<64 * Y::WAVES>(d, s0, Y::IMG / 16);
    float* v = reinterpret_cast<float*>(lds + Y::B1);
    if (threadIdx.x < 128) v[threadIdx.x] = reinterpret_cast<const float*>(net.img + net.b_off[1])[threadIdx.x];
    else if (threadIdx.x < 256)
      v[threadIdx.x] = reinterpret_cast<const float*>(net.img + net.b_off[2])[threadIdx.x - 128];
    else if (threadIdx.x < 320)
      v[threadIdx.x] = reinterpret_cast<const float*>(net.img + net.b_off[3])[threadIdx.x - 256];
  }
  __syncthreads();

  int fo = lane * 16;  // this lane's 16 B of a fragment; opaque per step (no hoisting of loop-invariant LDS reads)
  auto frag = [&](int base, int f) { return *reinterpret_cast<const bf16x8*>(lds + base + f * 1024 + fo); };
  const auto rW = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(net.img) + net.wmx3_lo_off, 0, 64 * 1024,
                                                    0x00020000);
  // hidden-layer lo fragment of stream position q: layer q / 32, part, k-step, m-tile in consumption order
  auto hlo_id = [](int q) {
    const int l = q >> 5, m = q & 31, hh = m >> 4, kk = (m >> 2) & 3, i = m & 3;
    return 32 * l + (4 * hh + i) * 4 + kk;
  };
  auto hlo = [&](int q) {
    return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rW, lane * 16, hlo_id(q) * 1024, 0));
  };
  const float* vb1 = reinterpret_cast<const float*>(lds + Y::B1) + 4 * g;
  const float* vb2 = reinterpret_cast<const float*>(lds + Y::B2) + 4 * g;
  const float* vb3 = reinterpret_cast<const float*>(lds + Y::B3) + 4 * g;
  float* ring = reinterpret_cast<float*>(lds + Y::RING + wib * Y::ring_bytes<COST>());

  const int H = a.H;
  const int wps = a.Kp / 16;
  const int total = a.B * wps;
  const float cl = a.ctrl_clamp > 0.0f ? a.ctrl_clamp : INFINITY;
  auto state_src = [&](int sl) {
    return sl < 32 ? (sl < net.qp ? sl : -1) : (sl - 32 < net.qv ? net.qp + sl - 32 : -1);
  };
  int chunk[4];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) {
    chunk[mt] = -1;
#pragma unroll
    for (int e = 0; e < 16; ++e)
      if (e == 4 * mt + g) chunk[mt] = CC::chunk(e / 4, e % 4);
  }

  for (int wt = blockIdx.x + gridDim.x * wib; wt < total; wt += gridDim.x * Y::WAVES) {
    const int b = __builtin_amdgcn_readfirstlane(wt / wps);
    const int k0 = (wt - b * wps) * 16;
    float cx[MPPI_CTX_MAX];
#pragma unroll
    for (int i = 0; i < MPPI_CTX_MAX; ++i) cx[i] = a.ctx ? a.ctx[(long)b * MPPI_CTX_MAX + i] : a.ctx_default[i];
    f32x4 x[4];  // the fp32 state, slot 16 mt + 4 g + r of sample n; 1.0 in the b0 pair's slots 62, 63
    {
      int go = g;
      asm volatile("" : "+v"(go));
      const auto rX = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.x0) + (long)b * a.nx, 0, a.nx * 4,
                                                        0x00020000);
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int sl = 16 * mt + 4 * go + r, src = state_src(sl);
          const float xv = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rX, src >= 0 ? 4 * src : 0x7FFFFFF0, 0, 0));
          x[mt][r] = (sl == kMlpBiasSlotHi || sl == kMlpBiasSlotLo) ? 1.0f : xv;
        }
    }
    const auto rU = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.U) + (long)b * a.nu * H, 0,
                                                      a.nu * H * 4, 0x00020000);
    const auto rE = __builtin_amdgcn_make_buffer_rsrc(a.noise + (long)b * a.nu * H * a.Kp, 0,
                                                      a.nu * H * a.Kp * 4, 0x00020000);
    // control slots of this lane group: 4g..4g+3, 16+4g..16+4g+3 (layer 0's third k-step); pads past nu read 0
    int uoff[8], eoff[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int us = (j < 4) ? 4 * g + j : 16 + 4 * g + (j - 4);
      uoff[j] = us < a.nu ? us * H * 4 : 0x7FFFFFF0;
      eoff[j] = us < a.nu ? (us * H * a.Kp + k0 + n) * 4 : 0x7FFFFFF0;
    }
    auto load_u = [&](int t, float (&c)[8]) {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        c[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rU, uoff[j], t * 4, 0)) +
               __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rE, eoff[j], t * a.Kp * 4, 0));
    };
    float un[8];
    load_u(0, un);
    float cost = 0.0f;
    auto ring_cost = [&](int t1) {
      const float* row = ring + n * CC::HS;
      f32x4 ch[CC::NCH];
#pragma unroll
      for (int c = 0; c < CC::NCH; ++c) ch[c] = *reinterpret_cast<const f32x4*>(row + 4 * c);
      constexpr CostIdx ci = cost_idx(COST);
      float v[kCostMaxIdx];
#pragma unroll
      for (int i = 0; i < ci.n; ++i) {
        const int sl = CC::slot(ci.idx[i]);
        v[i] = ch[CC::chunk(sl / 16, (sl % 16) / 4)][sl % 4];
      }
      return cost_eval_t<COST>(v, 0.0f, 0.0f, cx, t1);
    };

    for (int t = 0; t < H; ++t) {
      asm volatile("" : "+v"(fo));
      // ---- controls of step t (loaded a step ahead): clamp, the control part of the cost, layer 0's operands
      bf16x8 xh[3], xl[3];
      {
        f32x4 u0, u1;
        float usq = 0.0f;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          u0[j] = __builtin_amdgcn_fmed3f(un[j], -cl, cl);
          u1[j] = __builtin_amdgcn_fmed3f(un[4 + j], -cl, cl);
          usq = fmaf(u0[j], u0[j], usq);
          usq = fmaf(u1[j], u1[j], usq);
        }
        cost += ctrl_term_t<COST>(g == 0 ? u0[0] : 0.0f, usq);
        split16(x[0], x[1], xh[0], xl[0]);
        split16(x[2], x[3], xh[1], xl[1]);
        split16(u0, u1, xh[2], xl[2]);
      }
      load_u(t + 1 < H ? t + 1 : t, un);
      // the hidden layers' lo stream: the first X3M_LQ positions in flight during layer 0
      bf16x8 lq[X3M_LQ];
#pragma unroll
      for (int j = 0; j < X3M_LQ; ++j) lq[j] = hlo(j);

      // ---- layer 0 in 4 chunks of 2 m-tiles -> relu -> hi / lo, layer 1's operand of k-step c
      bf16x8 ah[4], al[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        f32x4 hv[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int mt = 2 * c + i;
          hv[i] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
          for (int kk = 0; kk < 3; ++kk)
            hv[i] = mma16x3(frag(Y::WH, 3 * mt + kk), frag(Y::W0L, 3 * mt + kk), xh[kk], xl[kk], hv[i]);
        }
        split16(relu4(hv[0]), relu4(hv[1]), ah[c], al[c]);
      }

      // ---- hidden layers 1 and 2 (128 -> 128), 2 parts of 4 m-tiles, bias from LDS as the accumulator's start
#pragma unroll
      for (int l = 0; l < 2; ++l) {
        const float* vb = l == 0 ? vb1 : vb2;
        bf16x8 oh[4], ol[4];
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          f32x4 z[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) z[i] = *reinterpret_cast<const f32x4*>(vb + 16 * (4 * hh + i));
#pragma unroll
          for (int kk = 0; kk < 4; ++kk)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int q = 32 * l + 16 * hh + 4 * kk + i;
              const bf16x8 lo = lq[q % X3M_LQ];
              if (q + X3M_LQ < 64) lq[q % X3M_LQ] = hlo(q + X3M_LQ);
              z[i] = mma16x3(frag(Y::WH, 24 + 32 * l + (4 * hh + i) * 4 + kk), lo, ah[kk], al[kk], z[i]);
            }
          split16(relu4(z[0]), relu4(z[1]), oh[2 * hh], ol[2 * hh]);
          split16(relu4(z[2]), relu4(z[3]), oh[2 * hh + 1], ol[2 * hh + 1]);
        }
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
          ah[kk] = oh[kk];
          al[kk] = ol[kk];
        }
      }

      // ---- last layer: x += b3 + W3 a (fp32 state)
      {
        f32x4 d[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) d[i] = *reinterpret_cast<const f32x4*>(vb3 + 16 * i);
#pragma unroll
        for (int kk = 0; kk < 4; ++kk)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            d[i] = mma16x3(frag(Y::WH, 88 + 4 * i + kk), frag(Y::W3L, 4 * i + kk), ah[kk], al[kk], d[i]);
#pragma unroll
        for (int i = 0; i < 4; ++i) x[i] += d[i];
      }

      // ---- the state part of the running cost of step t on x_{t+1} (1-based t + 1): one-step ring, lane group 0
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
        if (chunk[mt] >= 0) *reinterpret_cast<f32x4*>(ring + n * CC::HS + 4 * chunk[mt]) = x[mt];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (g == 0) cost += ring_cost(t + 1);
      __builtin_amdgcn_wave_barrier();
    }
    if (a.terminal_weight != 0.0f && g == 0) cost += a.terminal_weight * ring_cost(H);
    __builtin_amdgcn_wave_barrier();
    {
      const float c = group_sum(cost);
      const int k = k0 + n;
      if (g == 0 && k < a.K) a.costs[(long)b * a.Kp + k] = isfinite(c) ? c : INFINITY;
    }
    if (a.xout && k0 == 0 && n == 0) {
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int src = state_src(16 * mt + 4 * g + r);
          if (src >= 0) a.xout[(long)b * a.nx + src] = x[mt][r];
        }
    }
  }
  __syncthreads();
  kclock_record(a, kc);
}

static int x3m_device_cus() { return x3_device_cus(); }

// MPPI_X3M (read per launch): 0 = never, 1 = always (when the image carries it); unset = from one round of 8
// 16-sample wave-tiles per CU (the M-split split kernel below that: it spreads a tile's step over 4 SIMDs)
bool fc_wave_mlp_x3_wanted(const SolveArgs& a, const FcArgs& fa) {
  if (fa.wmx3_off < 0 || a.Kp < 16 || a.Kp % 16 != 0 || a.nx > kMlpBiasSlotHi || a.nu > 32) return false;
  const char* e = std::getenv("MPPI_X3M");
  if (e && e[0] == '0') return false;
  if (e && e[0] == '1') return true;
  return a.B * (a.Kp / 16) >= WaveMlpX3Lay::WAVES * x3m_device_cus();
}

hipError_t launch_fc_wave_mlp_x3(const SolveArgs& a, const FcArgs& fa, hipStream_t stream) {
  if (fa.wmx3_off < 0 || a.Kp <= 0 || a.Kp % 16 != 0) return hipErrorInvalidValue;
  const int wts = a.B * (a.Kp / 16);
  int grid = (wts + WaveMlpX3Lay::WAVES - 1) / WaveMlpX3Lay::WAVES;
  if (grid > x3m_device_cus()) grid = x3m_device_cus();
  auto go = [&](auto kern, int bytes) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * WaveMlpX3Lay::WAVES), bytes, stream, a, fa);
    return hipGetLastError();
  };
  note_kernel("fc_wave_mlp_x3_kernel");
#define MPPI_WAVE_MLP_X3_COST(K)                                                                    \
  case K:                                                                                           \
    static_assert(WaveMlpX3Lay::bytes<K>() <= 160 * 1024, "LDS per CU");                            \
    return go(fc_wave_mlp_x3_kernel<K>, WaveMlpX3Lay::bytes<K>());
  switch (a.cost_kind) {
    MPPI_WAVE_MLP_X3_COST(MPPI_COST_HUMANOID_V3)
    MPPI_WAVE_MLP_X3_COST(MPPI_COST_HUMANOID_V1)
    MPPI_WAVE_MLP_X3_COST(MPPI_COST_QUAD_EST)
    MPPI_WAVE_MLP_X3_COST(MPPI_COST_QUAD_JL)
    MPPI_WAVE_MLP_X3_COST(MPPI_COST_CARTPOLE_EST)
    MPPI_WAVE_MLP_X3_COST(MPPI_COST_CARTPOLE)
    default: return hipErrorInvalidValue;
  }
#undef MPPI_WAVE_MLP_X3_COST
}

}  // namespace mppi
