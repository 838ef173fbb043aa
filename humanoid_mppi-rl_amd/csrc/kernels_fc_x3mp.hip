// fc_wave32_mlp_x3_kernel (round 5): the split-bf16 (MPPI_PREC_BF16X3, fp32-accurate) per-wave rollout of
// MLPStatePredictor(nx, nu, 128, hidden_layers = 2) (learning/model.py:6-46) at 32 samples per wave on 32x32x16 MFMAs:
// fc_wave_mlp_x3_kernel's arithmetic (kernels_fc_x3m.hip: three bf16 products per product, hi / lo operands) in
// fc_wave32_x3p_kernel's organisation (kernels_fc_x3p.hip: two waves per SIMD, every layer streamed into the next one
// 32 rows at a time, so that only the accumulators of two layers are live).  Per wave-step 312 MFMAs of 32 cycles for
// 32 samples (the 16-sample kernel: 312 of 16 cycles for 16 samples), with each LDS fragment read feeding twice the
// samples and half the W1 / W2 lo stream from L2 per sample.
//   * LDS (144 KiB): hi of all four layers, lo of layers 0 and 3 (mppi_nets.cpp pack_image, mlp_x3); W1 / W2 lo from L2.
//   * layer 0's operand: the state as two 32x32 tiles (k-steps 0..3) and the controls laid out as a third tile (k-steps
//     4, 5: lane half h holds controls 8 i + 4 h + r, r < 4), so all six k-steps split like an accumulator tile.
//   * the running cost's state part from the registers (lane half 0; one v_permlane32_swap per slot that half 1 holds).
#include <cstdlib>

#include "x3_common.h"

namespace mppi {

namespace {

struct WaveMlp32X3Lay {
  static constexpr int W0H = 0;                // 24 fragments: T 6 + ks
  static constexpr int W1H = W0H + 24 * 1024;  // 32: T 8 + ks
  static constexpr int W2H = W1H + 32 * 1024;  // 32
  static constexpr int W3H = W2H + 32 * 1024;  // 16: T 8 + ks
  static constexpr int W0L = W3H + 16 * 1024;
  static constexpr int W3L = W0L + 24 * 1024;
  static constexpr int IMG = W3L + 16 * 1024;  // 144 KiB, one contiguous copy of the image at net.wm32x3_off
  static constexpr int B1 = IMG;               // 128 f32
  static constexpr int B2 = B1 + 512;          // 128 f32
  static constexpr int B3 = B2 + 512;          // 64 f32
  static constexpr int BYTES = B3 + 256;
  static constexpr int WAVES = 8;
};
#ifndef X3MP_LQ  // W1 / W2 lo fragments read this many stream positions ahead (position = one MFMA triple)
#define X3MP_LQ 8
#endif

// the hidden layers' lo fragment of stream position q: layer 1 in (T, kk, T1) order, layer 2 in (T1, kk, T2)
__device__ __forceinline__ int mlp32_lo_id(int q) {
  const int l = q >> 5, m = q & 31;
  return 32 * l + (m & 3) * 8 + 2 * (m >> 3) + ((m >> 2) & 1);
}
__device__ __forceinline__ f32x16 relu16(f32x16 v) {
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = __builtin_amdgcn_fmed3f(v[r], 0.0f, 3.402823466e38f);
  return v;
}

}  // namespace

template <int COST>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2))) void fc_wave32_mlp_x3_kernel(SolveArgs a,
                                                                                                       FcArgs net) {
  using Y = WaveMlp32X3Lay;
  using CC = CostChunks<kArchMLP, COST>;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const KClock kc = kclock_begin(a);
  if (blockIdx.x == 0 && threadIdx.x == 0) *a.status = 0u;
  const int lane = threadIdx.x & 63, h = lane >> 5, n = lane & 31;
  const int wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  {
    const int4* s0 = reinterpret_cast<const int4*>(net.img + net.wm32x3_off);
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
  const auto rW = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(net.img) + net.wm32x3_lo_off, 0, 64 * 1024,
                                                    0x00020000);
  auto hlo = [&](int q) {
    return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rW, lane * 16, mlp32_lo_id(q) * 1024, 0));
  };
  const float* vb1 = reinterpret_cast<const float*>(lds + Y::B1) + 4 * h;
  const float* vb2 = reinterpret_cast<const float*>(lds + Y::B2) + 4 * h;
  const float* vb3 = reinterpret_cast<const float*>(lds + Y::B3) + 4 * h;
  auto bias16 = [&](const float* vb, int T) {  // rows 32 T + 8 g8 + 4 h + r of a bias vector, accumulator layout
    f32x16 v;
#pragma unroll
    for (int g8 = 0; g8 < 4; ++g8) {
      const f32x4 b = *reinterpret_cast<const f32x4*>(vb + 32 * T + 8 * g8);
#pragma unroll
      for (int r = 0; r < 4; ++r) v[4 * g8 + r] = b[r];
    }
    return v;
  };

  const int H = a.H;
  const int wps = a.Kp / 32;
  const int total = a.B * wps;
  const float cl = a.ctrl_clamp > 0.0f ? a.ctrl_clamp : INFINITY;
  auto state_src = [&](int sl) {
    return sl < 32 ? (sl < net.qp ? sl : -1) : (sl - 32 < net.qv ? net.qp + sl - 32 : -1);
  };
  // the state part of the running cost from the registers: value i of the cost is slot sl = 32 T + r32, held by lane
  // half (r32 >> 2) & 1 at value (r32 & 3) + 4 (r32 >> 3); lane half 0 evaluates, a swap brings half 1's slots.
  // Called by EVERY lane (the swaps read the other half's lanes).
  auto state_cost = [&](const f32x16 (&xs)[2], const float* cx, int t1) {
    constexpr CostIdx ci = cost_idx(COST);
    float v[kCostMaxIdx];
#pragma unroll
    for (int i = 0; i < ci.n; ++i) {
      const int sl = CC::slot(ci.idx[i]), T = sl >> 5, r32 = sl & 31, hh = (r32 >> 2) & 1;
      const float own = xs[T][(r32 & 3) + 4 * (r32 >> 3)];
      if (hh == 0) {
        v[i] = own;
      } else {
        auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(own), __float_as_uint(own), false, false);
        v[i] = __uint_as_float(p[1]);  // lanes 0..31: the value of lane + 32
      }
    }
    return cost_eval_t<COST>(v, 0.0f, 0.0f, cx, t1);
  };

  for (int wt = blockIdx.x + gridDim.x * wib; wt < total; wt += gridDim.x * Y::WAVES) {
    const int b = __builtin_amdgcn_readfirstlane(wt / wps);
    const int k0 = (wt - b * wps) * 32;
    float cx[MPPI_CTX_MAX];
#pragma unroll
    for (int i = 0; i < MPPI_CTX_MAX; ++i) cx[i] = a.ctx ? a.ctx[(long)b * MPPI_CTX_MAX + i] : a.ctx_default[i];
    f32x16 x[2];  // the fp32 state, tiles 0 (slots 0..31) and 1 (32..63); 1.0 in the b0 pair's slots 62, 63
    int ho = h;
    asm volatile("" : "+v"(ho));
    {
      const auto rX = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.x0) + (long)b * a.nx, 0, a.nx * 4,
                                                        0x00020000);
#pragma unroll
      for (int T = 0; T < 2; ++T)
#pragma unroll
        for (int v = 0; v < 16; ++v) {
          const int sl = 32 * T + 8 * (v / 4) + 4 * ho + v % 4, src = state_src(sl);
          const float xv = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rX, src >= 0 ? 4 * src : 0x7FFFFFF0, 0, 0));
          x[T][v] = (sl == kMlpBiasSlotHi || sl == kMlpBiasSlotLo) ? 1.0f : xv;
        }
    }
    const auto rU = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.U) + (long)b * a.nu * H, 0,
                                                      a.nu * H * 4, 0x00020000);
    const auto rE = __builtin_amdgcn_make_buffer_rsrc(a.noise + (long)b * a.nu * H * a.Kp, 0,
                                                      a.nu * H * a.Kp * 4, 0x00020000);
    // controls of value v: slot (v & 3) + 8 (v >> 2) + 4 h (pads past nu read 0 through the buffer range); the
    // offsets are rebuilt per load from an opaque lane half (32 loop-invariant VGPRs otherwise)
    auto load_u = [&](int t, float (&c)[16]) {
      int hb = h;
      asm volatile("" : "+v"(hb));
      const int eb = k0 + n;
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int cs = (v & 3) + 8 * (v >> 2) + 4 * hb;
        const bool ok = cs < a.nu;
        const int uo = ok ? cs * H * 4 : 0x7FFFFFF0, eo = ok ? (cs * H * a.Kp + eb) * 4 : 0x7FFFFFF0;
        c[v] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rU, uo, t * 4, 0)) +
               __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rE, eo, t * a.Kp * 4, 0));
      }
    };
    float un[16];
    load_u(0, un);
    float cost = 0.0f;

    for (int t = 0; t < H; ++t) {
      asm volatile("" : "+v"(fo));
      // ---- controls of step t: clamp, the control part of the running cost, layer 0's k-steps 4, 5
      bf16x8 xh[6], xl[6];
      {
        f32x16 uc;
        float usq = 0.0f;
#pragma unroll
        for (int v = 0; v < 16; ++v) {
          uc[v] = __builtin_amdgcn_fmed3f(un[v], -cl, cl);
          usq = fmaf(uc[v], uc[v], usq);
        }
        cost += ctrl_term_t<COST>(h == 0 ? uc[0] : 0.0f, usq);  // control 0: value 0 of lane half 0
        split32<0>(x[0], xh[0], xl[0]);
        split32<1>(x[0], xh[1], xl[1]);
        split32<0>(x[1], xh[2], xl[2]);
        split32<1>(x[1], xh[3], xl[3]);
        split32<0>(uc, xh[4], xl[4]);
        split32<1>(uc, xh[5], xl[5]);
      }
      bf16x8 lq[X3MP_LQ];
#pragma unroll
      for (int j = 0; j < X3MP_LQ; ++j) lq[j] = hlo(j);

      // ---- layer 0, one 32-row tile at a time, ReLU'd and split: layer 1's k-steps 2 T, 2 T + 1, consumed at once
      f32x16 z1[4];
#pragma unroll
      for (int T1 = 0; T1 < 4; ++T1) z1[T1] = bias16(vb1, T1);
#pragma unroll
      for (int T = 0; T < 4; ++T) {
        f32x16 acc = {};
#pragma unroll
        for (int ks = 0; ks < 6; ++ks) acc = mma3(frag(Y::W0H, 6 * T + ks), frag(Y::W0L, 6 * T + ks), xh[ks], xl[ks], acc);
        acc = relu16(acc);
        bf16x8 ah[2], al[2];
        split32<0>(acc, ah[0], al[0]);
        split32<1>(acc, ah[1], al[1]);
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
          for (int T1 = 0; T1 < 4; ++T1) {
            const int q = 8 * T + 4 * kk + T1;
            const bf16x8 lo = lq[q % X3MP_LQ];
            if (q + X3MP_LQ < 64) lq[q % X3MP_LQ] = hlo(q + X3MP_LQ);
            z1[T1] = mma3(frag(Y::W1H, 8 * T1 + 2 * T + kk), lo, ah[kk], al[kk], z1[T1]);
          }
      }
      // ---- layer 1's output, one tile at a time, into layer 2
      f32x16 z2[4];
#pragma unroll
      for (int T2 = 0; T2 < 4; ++T2) z2[T2] = bias16(vb2, T2);
#pragma unroll
      for (int T1 = 0; T1 < 4; ++T1) {
        const f32x16 r = relu16(z1[T1]);
        bf16x8 ah[2], al[2];
        split32<0>(r, ah[0], al[0]);
        split32<1>(r, ah[1], al[1]);
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
          for (int T2 = 0; T2 < 4; ++T2) {
            const int q = 32 + 8 * T1 + 4 * kk + T2;
            const bf16x8 lo = lq[q % X3MP_LQ];
            if (q + X3MP_LQ < 64) lq[q % X3MP_LQ] = hlo(q + X3MP_LQ);
            z2[T2] = mma3(frag(Y::W2H, 8 * T2 + 2 * T1 + kk), lo, ah[kk], al[kk], z2[T2]);
          }
      }
      load_u(t + 1 < H ? t + 1 : t, un);  // the next step's controls, in flight through the last two layers
      // ---- layer 2's output, one tile at a time, into the last layer: x += b3 + W3 a (fp32 state)
      {
        f32x16 d[2] = {bias16(vb3, 0), bias16(vb3, 1)};
#pragma unroll
        for (int T2 = 0; T2 < 4; ++T2) {
          const f32x16 r = relu16(z2[T2]);
          bf16x8 ah[2], al[2];
          split32<0>(r, ah[0], al[0]);
          split32<1>(r, ah[1], al[1]);
#pragma unroll
          for (int kk = 0; kk < 2; ++kk)
#pragma unroll
            for (int T3 = 0; T3 < 2; ++T3) {
              const int f = 8 * T3 + 2 * T2 + kk;
              d[T3] = mma3(frag(Y::W3H, f), frag(Y::W3L, f), ah[kk], al[kk], d[T3]);
            }
        }
#pragma unroll
        for (int T = 0; T < 2; ++T) x[T] += d[T];
      }
      // ---- the state part of the running cost of step t on x_{t+1} (1-based t + 1), kept on lane half 0
      {
        float sc = state_cost(x, cx, t + 1);
        asm volatile("" : "+v"(sc));
        cost += h == 0 ? sc : 0.0f;
      }
    }
    if (a.terminal_weight != 0.0f) {
      float tc = state_cost(x, cx, H);
      asm volatile("" : "+v"(tc));
      cost += h == 0 ? a.terminal_weight * tc : 0.0f;
    }
    {
      auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(cost), __float_as_uint(cost), false, false);
      const float c = __uint_as_float(p[0]) + __uint_as_float(p[1]);
      const int k = k0 + n;
      if (h == 0 && k < a.K) a.costs[(long)b * a.Kp + k] = isfinite(c) ? c : INFINITY;
    }
    if (a.xout && k0 == 0 && n == 0) {
      int hs = h;
      asm volatile("" : "+v"(hs));
#pragma unroll
      for (int T = 0; T < 2; ++T)
#pragma unroll
        for (int v = 0; v < 16; ++v) {
          const int src = state_src(32 * T + 8 * (v / 4) + 4 * hs + v % 4);
          if (src >= 0) a.xout[(long)b * a.nx + src] = x[T][v];
        }
    }
  }
  __syncthreads();
  kclock_record(a, kc);
}

// MPPI_X3M32 (read per launch): 0 = never, 1 = always (when the image carries it); unset: from one round of 8
// 32-sample wave-tiles per CU (below it fc_wave_mlp_x3_kernel or the M-split split kernel)
bool fc_wave32_mlp_x3_wanted(const SolveArgs& a, const FcArgs& fa) {
  if (fa.wm32x3_off < 0 || a.Kp < 32 || a.Kp % 32 != 0 || a.nx > kMlpBiasSlotHi || a.nu > 32) return false;
  const char* e = std::getenv("MPPI_X3M32");
  if (e && e[0] == '0') return false;
  if (e && e[0] == '1') return true;
  return a.B * (a.Kp / 32) >= WaveMlp32X3Lay::WAVES * x3_device_cus();
}

hipError_t launch_fc_wave32_mlp_x3(const SolveArgs& a, const FcArgs& fa, hipStream_t stream) {
  if (fa.wm32x3_off < 0 || a.Kp <= 0 || a.Kp % 32 != 0) return hipErrorInvalidValue;
  const int wts = a.B * (a.Kp / 32);
  int grid = (wts + WaveMlp32X3Lay::WAVES - 1) / WaveMlp32X3Lay::WAVES;
  if (grid > x3_device_cus()) grid = x3_device_cus();
  auto go = [&](auto kern) {
    constexpr int bytes = WaveMlp32X3Lay::BYTES;
    static_assert(bytes <= 160 * 1024, "LDS per CU");
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       bytes);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * WaveMlp32X3Lay::WAVES), bytes, stream, a, fa);
    return hipGetLastError();
  };
  note_kernel("fc_wave32_mlp_x3_kernel");
  switch (a.cost_kind) {
    case MPPI_COST_HUMANOID_V3: return go(fc_wave32_mlp_x3_kernel<MPPI_COST_HUMANOID_V3>);
    case MPPI_COST_HUMANOID_V1: return go(fc_wave32_mlp_x3_kernel<MPPI_COST_HUMANOID_V1>);
    case MPPI_COST_QUAD_EST: return go(fc_wave32_mlp_x3_kernel<MPPI_COST_QUAD_EST>);
    case MPPI_COST_QUAD_JL: return go(fc_wave32_mlp_x3_kernel<MPPI_COST_QUAD_JL>);
    case MPPI_COST_CARTPOLE_EST: return go(fc_wave32_mlp_x3_kernel<MPPI_COST_CARTPOLE_EST>);
    case MPPI_COST_CARTPOLE: return go(fc_wave32_mlp_x3_kernel<MPPI_COST_CARTPOLE>);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace mppi
