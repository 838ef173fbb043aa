// The split-bf16 (MPPI_PREC_BF16X3) per-wave CA rollout, fc_wave32_x3_kernel: fc_wave32_kernel's organisation
// (kernels_fc_wave.hip) at fp32 accuracy.  Its own translation unit so that it builds with the MFMA accumulators in
// AGPRs (build.py: no -amdgpu-mfma-vgpr-form here): a lone wave per SIMD has the whole 512-entry register file, and
// with the accumulators in AccVGPRs the 256 ArchVGPRs hold the hi / lo activations and the fragments in flight
// (config #4 at 64 solves, same box: 1501 -> 977 us per rollout; profiles/r04_ab_x3_agpr.log).
#include <cstdlib>

#include "x3_common.h"

#ifndef X3_L0LO_QV0  // the fp16 form's layer 0: the qvel rows' first k-step (state slots 32..47) with its lo (1) or hi only
                     // (0: fc_wave32_x3p_kernel's form, which the engine's probe checks; kernels_fc_x3p.hip X3P_L0LO_QV0)
#define X3_L0LO_QV0 0
#endif

namespace mppi {

template <int COST, int L1T>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void fc_wave32_x3_kernel(SolveArgs a,
                                                                                                   FcArgs net) {
  using Y = WaveX3Lay;
  using CC = CostChunks<kArchCA, COST>;
  constexpr int R = 2;  // ring steps: lane half h evaluates ring step h of its sample at each flush
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const KClock kc = kclock_begin(a);
  if (blockIdx.x == 0 && threadIdx.x == 0) *a.status = 0u;
  const int lane = threadIdx.x & 63, h = lane >> 5, n = lane & 31;
  const int wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  {
    const int4* s0 = reinterpret_cast<const int4*>(net.img + (L1T <= 1 ? net.w32f16_off : net.w32x3_off));
    int4* d = reinterpret_cast<int4*>(lds);
    stage_lds<256>(d, s0, Y::IMG / 16);
    float* v = reinterpret_cast<float*>(lds + Y::B1);
    if (threadIdx.x < 128) v[threadIdx.x] = reinterpret_cast<const float*>(net.img + net.b_off[1])[threadIdx.x];
    else if (threadIdx.x < 192)
      v[threadIdx.x] = reinterpret_cast<const float*>(net.img + net.b_off[2])[threadIdx.x - 128];
  }
  __syncthreads();

  int fo = lane * 16;  // this lane's 16 B of a fragment; opaque per step (no hoisting of loop-invariant LDS reads)
  auto frag = [&](int base, int f) { return *reinterpret_cast<const bf16x8*>(lds + base + f * 1024 + fo); };
  // W1's lo fragments from L2 (buffer loads: a scalar offset per fragment, no per-lane 64-bit address)
  const auto rW = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(net.img) + net.w32x3_l1lo_off, 0, 64 * 1024,
                                                    0x00020000);
  auto w1lo = [&](int f) {
    return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rW, lane * 16, f * 1024, 0));
  };
  const float* vb1 = reinterpret_cast<const float*>(lds + Y::B1) + 4 * h;
  const float* vbx = reinterpret_cast<const float*>(lds + Y::BX) + 4 * h;
  float* ring = reinterpret_cast<float*>(lds + Y::RING + wib * Y::ring_bytes<COST>());

  const int H = a.H;
  const int wps = a.Kp / 32;
  const int total = a.B * wps;
  const float inv_n = 1.0f / (float)net.ln_n;
  const float cl = a.ctrl_clamp > 0.0f ? a.ctrl_clamp : INFINITY;
  auto state_src = [&](int sl) {
    return sl < 32 ? (sl < net.qp ? sl : -1) : (sl - 32 < net.qv ? net.qp + sl - 32 : -1);
  };
  int chunk[2][4];
#pragma unroll
  for (int T = 0; T < 2; ++T)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      chunk[T][i] = -1;
#pragma unroll
      for (int hh = 0; hh < 2; ++hh)
        if (hh == h) chunk[T][i] = CC::chunk(2 * T + i / 2, 2 * (i % 2) + hh);
    }
  constexpr int NJ = 11;  // controls c = 2 j + h (requires 20 <= nu <= 22: launch_fc_wave_x3)

  for (int wt = blockIdx.x + gridDim.x * wib; wt < total; wt += gridDim.x * Y::WAVES) {
    const int b = __builtin_amdgcn_readfirstlane(wt / wps);
    const int k0 = (wt - b * wps) * 32;
    float cx[MPPI_CTX_MAX];
#pragma unroll
    for (int i = 0; i < MPPI_CTX_MAX; ++i) cx[i] = a.ctx ? a.ctx[(long)b * MPPI_CTX_MAX + i] : a.ctx_default[i];
    f32x16 x[2];  // the fp32 state, D-tiles 0 (slots 0..31) and 1 (32..63); 1.0 in the b0c slots 28, 60
    int ho = h;
    asm volatile("" : "+v"(ho));
    const auto rX = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.x0) + (long)b * a.nx, 0, a.nx * 4, 0x00020000);
#pragma unroll
    for (int T = 0; T < 2; ++T)
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int sl = 32 * T + 8 * (v / 4) + 4 * ho + v % 4, src = state_src(sl);
        const float xv = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rX, src >= 0 ? 4 * src : 0x7FFFFFF0, 0, 0));
        x[T][v] = (sl == kCaBiasSlotHi || sl == kCaBdBiasSlotHi) ? 1.0f : xv;
      }
    const auto rU = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.U) + (long)b * a.nu * H, 0,
                                                      a.nu * H * 4, 0x00020000);
    const auto rE = __builtin_amdgcn_make_buffer_rsrc(a.noise + (long)b * a.nu * H * a.Kp, 0,
                                                      a.nu * H * a.Kp * 4, 0x00020000);
    const int cl_ = 2 * (NJ - 1) + h;
    const int uoff0 = h * H * 4, eoff0 = (h * H * a.Kp + k0 + n) * 4;
    const int uoffl = cl_ < a.nu ? cl_ * H * 4 : 0x7FFFFFF0;
    const int eoffl = cl_ < a.nu ? (cl_ * H * a.Kp + k0 + n) * 4 : 0x7FFFFFF0;
    auto load_u = [&](int t, float (&c)[NJ]) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const bool last = j == NJ - 1;
        c[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rU, last ? uoffl : uoff0,
                                                                    t * 4 + (last ? 0 : j * 8 * H), 0)) +
               __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
                   rE, last ? eoffl : eoff0, (t * a.Kp + (last ? 0 : j * 2 * H * a.Kp)) * 4, 0));
      }
    };
    float un[NJ];
    load_u(0, un);
    float cost = 0.0f;
    auto ring_cost = [&](int rs, int t1) {
      const float* row = ring + (rs * 32 + n) * CC::HS;
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
      // W1's first two k-steps of lo fragments in flight from L2 during the statistic and layer 0
      bf16x8 l1q[MPPI_X3_L1PF][4];
#pragma unroll
      for (int kk = 0; kk < MPPI_X3_L1PF; ++kk)
#pragma unroll
        for (int T = 0; T < 4; ++T) l1q[kk][T] = L1T <= 1 ? bf16x8{} : w1lo(T * 16 + kk);  // (fp16 form: no lo)
      // ---- control part of the running cost of step t
      {
        float usq = 0.0f;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const float u = __builtin_amdgcn_fmed3f(un[j], -cl, cl);
          usq = fmaf(u, u, usq);
        }
        cost += ctrl_term_t<COST>(h == 0 ? __builtin_amdgcn_fmed3f(un[0], -cl, cl) : 0.0f, usq);
      }
      // ---- layer-0 operand as hi / lo, the statistic |R x~|^2 / n and mu = m~ x~ (R's row 30)
      // (the fp16 form with MPPI_X3_F16_L0, mppi_internal.h: fp16 W hi + lo against the state rounded to fp16)
      constexpr bool L0H = L1T <= 1 && MPPI_X3_F16_L0;
      bf16x8 xh[4], xl[4];
      if constexpr (L0H) {
        (void)xl;
        xh[0] = h16<0>(x[0]);
        xh[1] = h16<1>(x[0]);
        xh[2] = h16<0>(x[1]);
        xh[3] = h16<1>(x[1]);
      } else {
        split32<0>(x[0], xh[0], xl[0]);
        split32<1>(x[0], xh[1], xl[1]);
        split32<0>(x[1], xh[2], xl[2]);
        split32<1>(x[1], xh[3], xl[3]);
      }
      auto mm0 = [&](const bf16x8& wh, const bf16x8& wl, int ks, const f32x16& c) {
        if constexpr (L0H)
          return mma32h(wh, xh[ks], mma32h(wl, xh[ks], c));
        else
          return mma3(wh, wl, xh[ks], xl[ks], c);
      };
      float rstd, mu;
      {
        f32x16 g0 = {}, g1 = {};
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) g0 = mm0(frag(Y::RH, ks), frag(Y::RL, ks), ks, g0);
#pragma unroll
        for (int ks = 2; ks < 4; ++ks) g1 = mm0(frag(Y::RH, 4 + ks), frag(Y::RL, 4 + ks), ks, g1);
        const float m14 = g0[14];
        g0[14] = h == 1 ? 0.0f : m14;
        {
          auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(m14), __float_as_uint(m14), false, false);
          mu = h == 1 ? m14 : __uint_as_float(p[1]);
        }
        float qa = 0.0f, qb = 0.0f;
#pragma unroll
        for (int v = 0; v < 16; v += 2) {
          qa = fmaf(g0[v], g0[v], qa);
          qb = fmaf(g0[v + 1], g0[v + 1], qb);
          qa = fmaf(g1[v], g1[v], qa);
          qb = fmaf(g1[v + 1], g1[v + 1], qb);
        }
        float q = qa + qb;
        {
          auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(q), __float_as_uint(q), false, false);
          q = __uint_as_float(p[0]) + __uint_as_float(p[1]);
        }
        const float v = fmaf(q, inv_n, 1e-5f);
        rstd = __builtin_amdgcn_rsqf(v);
        const float sc = v * rstd;  // s = sqrt(var + eps), split: s_hi into xh, s_lo into xl at slots 30, 62
        if constexpr (L0H) {  // s as fp16 at slots 30, 62 (31 / 63 stay 0; -mu through the accumulators)
          const unsigned s16 = pk_f16(sc, 0.0f);
          u32x4 h1 = __builtin_bit_cast(u32x4, xh[1]), h3 = __builtin_bit_cast(u32x4, xh[3]);
          h1[3] = h == 1 ? (h1[3] & 0xFFFF0000u) | (s16 & 0xFFFFu) : h1[3];
          h3[3] = h == 1 ? (h3[3] & 0xFFFF0000u) | (s16 & 0xFFFFu) : h3[3];
          xh[1] = __builtin_bit_cast(bf16x8, h1);
          xh[3] = __builtin_bit_cast(bf16x8, h3);
        } else {
        const unsigned shi = pk_bf16(sc, 0.0f);
        const unsigned slo = pk_bf16(sc - __uint_as_float(shi << 16), 0.0f);
        // slot 30: k-step 1, slot 62: k-step 3; lane half 1, element 6 (the low half of word 3; 31 / 63 stay 0)
        u32x4 h1 = __builtin_bit_cast(u32x4, xh[1]), l1 = __builtin_bit_cast(u32x4, xl[1]);
        u32x4 h3 = __builtin_bit_cast(u32x4, xh[3]), l3 = __builtin_bit_cast(u32x4, xl[3]);
        h1[3] = h == 1 ? (h1[3] & 0xFFFF0000u) | (shi & 0xFFFFu) : h1[3];
        l1[3] = h == 1 ? (l1[3] & 0xFFFF0000u) | (slo & 0xFFFFu) : l1[3];
        h3[3] = h == 1 ? (h3[3] & 0xFFFF0000u) | (shi & 0xFFFFu) : h3[3];
        l3[3] = h == 1 ? (l3[3] & 0xFFFF0000u) | (slo & 0xFFFFu) : l3[3];
        xh[1] = __builtin_bit_cast(bf16x8, h1);
        xl[1] = __builtin_bit_cast(bf16x8, l1);
        xh[3] = __builtin_bit_cast(bf16x8, h3);
        xl[3] = __builtin_bit_cast(bf16x8, l3);
        }
      }

      // ---- layer 0 (block-diagonal), two D-tiles at a time: relu(h + beta' s) -> hi / lo, layer 1's operand
      bf16x8 a1h[16], a1l[16];
      (void)a1l;
#pragma unroll
      for (int T = 0; T < 8; T += 2) {
        f32x16 acc[2];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int v = 0; v < 16; ++v) acc[i][v] = -mu;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            const int TT = T + i, ks = (TT < 4 ? 0 : 2) + kk, p = 2 * TT + kk;
            if (L0H && !X3_L0LO_QV0 && ks == 2)  // the qvel rows' first k-step: hi only (as fc_wave32_x3p_kernel)
              acc[i] = mma32h(frag(Y::W0H, p), xh[ks], acc[i]);
            else
              acc[i] = mm0(frag(Y::W0H, p), frag(Y::W0L, p), ks, acc[i]);
          }
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          if constexpr (L1T <= 1) {  // the fp16 form (fc_common.h x3_f16_on): ReLU'd fp16
            a1h[2 * (T + i)] = h16_relu<0>(acc[i]);
            a1h[2 * (T + i) + 1] = h16_relu<1>(acc[i]);
          } else if constexpr (L1T == 2) {  // layer 1 reads its operand's hi part only (x3_l1_terms), ReLU'd packed
            a1h[2 * (T + i)] = hi32_relu<0>(acc[i]);
            a1h[2 * (T + i) + 1] = hi32_relu<1>(acc[i]);
          } else {
#pragma unroll
            for (int v = 0; v < 16; ++v) acc[i][v] = __builtin_amdgcn_fmed3f(acc[i][v], 0.0f, 3.402823466e38f);  // v_med3: no NaN-quieting v_max
            split32<0>(acc[i], a1h[2 * (T + i)], a1l[2 * (T + i)]);
            split32<1>(acc[i], a1h[2 * (T + i) + 1], a1l[2 * (T + i) + 1]);
          }
        }
      }

      // ---- layer 1: z = rstd (W1 a) + b1, four D-tiles interleaved per k-step; W1 lo two k-steps ahead from L2
      bf16x8 a2h[8], a2l[8];
      {
        f32x16 z[4] = {{}, {}, {}, {}};
#pragma unroll
        for (int ks = 0; ks < 16; ++ks) {
#pragma unroll
          for (int T = 0; T < 4; ++T) {
            if constexpr (L1T <= 1) {  // one fp16 product (W1 in fp16 at W1H)
              z[T] = mma32h(frag(Y::W1H, T * 16 + ks), a1h[ks], z[T]);
              continue;
            }
            const bf16x8 lo = l1q[ks % MPPI_X3_L1PF][T];
            if (ks + MPPI_X3_L1PF < 16) l1q[ks % MPPI_X3_L1PF][T] = w1lo(T * 16 + ks + MPPI_X3_L1PF);
            if constexpr (L1T == 2)
              z[T] = mma32(frag(Y::W1H, T * 16 + ks), a1h[ks], mma32(lo, a1h[ks], z[T]));
            else
              z[T] = mma3(frag(Y::W1H, T * 16 + ks), lo, a1h[ks], a1l[ks], z[T]);
          }
        }
#pragma unroll
        for (int T = 0; T < 4; ++T) {
#pragma unroll
          for (int g8 = 0; g8 < 4; ++g8) {
            const f32x4 b1 = *reinterpret_cast<const f32x4*>(vb1 + 32 * T + 8 * g8);
#pragma unroll
            for (int r = 0; r < 4; ++r)
              z[T][4 * g8 + r] = L1T <= 1 ? fmaf(z[T][4 * g8 + r], rstd, b1[r])  // (ReLU after fp16 packing)
                                          : __builtin_amdgcn_fmed3f(fmaf(z[T][4 * g8 + r], rstd, b1[r]), 0.0f,
                                                                    3.402823466e38f);
          }
          if constexpr (L1T <= 1) {
            a2h[2 * T] = h16_relu<0>(z[T]);
            a2h[2 * T + 1] = h16_relu<1>(z[T]);
          } else {
            split32<0>(z[T], a2h[2 * T], a2l[2 * T]);
            split32<1>(z[T], a2h[2 * T + 1], a2l[2 * T + 1]);
          }
        }
      }
      load_u(t + 1 < H ? t + 1 : t, un);  // the next step's controls

      // ---- last layer: x += bx + Wx a2
      {
        f32x16 d[2];
#pragma unroll
        for (int T = 0; T < 2; ++T)
#pragma unroll
          for (int g8 = 0; g8 < 4; ++g8) {
            const f32x4 bx = *reinterpret_cast<const f32x4*>(vbx + 32 * T + 8 * g8);
#pragma unroll
            for (int r = 0; r < 4; ++r) d[T][4 * g8 + r] = bx[r];
          }
#pragma unroll
        for (int ks = 0; ks < 8; ++ks)
#pragma unroll
          for (int T = 0; T < 2; ++T)
            d[T] = L1T == 0   ? mma32h(frag(Y::WXH, T * 8 + ks), a2h[ks], d[T])  // fp16, one product
                   : L1T <= 1 ? mma32h(frag(Y::WXH, T * 8 + ks), a2h[ks], mma32h(frag(Y::WXL, T * 8 + ks), a2h[ks], d[T]))
                              : mma3(frag(Y::WXH, T * 8 + ks), frag(Y::WXL, T * 8 + ks), a2h[ks], a2l[ks], d[T]);
#pragma unroll
        for (int T = 0; T < 2; ++T) x[T] += d[T];
      }

      // ---- cost ring [2 steps][32 samples][HS]; flush every 2 steps: lane half h takes ring step h
#pragma unroll
      for (int T = 0; T < 2; ++T)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (chunk[T][i] >= 0)
            *reinterpret_cast<f32x4*>(ring + ((t % R) * 32 + n) * CC::HS + 4 * chunk[T][i]) =
                f32x4{x[T][4 * i], x[T][4 * i + 1], x[T][4 * i + 2], x[T][4 * i + 3]};
      if ((t + 1) % R == 0 || t + 1 == H) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const int ts = t - t % R + h;
        if (ts <= t) cost += ring_cost(h, ts + 1);
        __builtin_amdgcn_wave_barrier();
      }
    }
    if (a.terminal_weight != 0.0f && h == 0) cost += a.terminal_weight * ring_cost((H - 1) % R, H);
    __builtin_amdgcn_wave_barrier();
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

// MPPI_X3_PAIR (read per launch): unset = two waves per SIMD (kernels_fc_x3p.hip) once the wave-tiles exceed one per
// SIMD, 0 = never, 1 = always.  At <= 4 tiles per CU the pair kernel would run them on half the CUs (8 per block).
static bool x3_pair_on(int wts) {
  const char* e = std::getenv("MPPI_X3_PAIR");
  if (e && e[0] == '0') return false;
  if (e && e[0] == '1') return true;
  return wts > WaveX3Lay::WAVES * x3_device_cus();
}

// MPPI_X3_WAVE (read per launch): 0 = split bf16 always on the M-split kernels, 2 = always on the per-wave kernels
static int x3_wave_mode() {
  const char* e = std::getenv("MPPI_X3_WAVE");
  return e && e[0] == '0' ? 0 : (e && e[0] == '2' ? 2 : 1);
}

bool fc_wave_x3_wanted(const SolveArgs& a, const FcArgs& fa) {
  // whole 32-sample wave-tiles, the humanoid controls, and enough of them for every CU's 4 waves
  if (fa.w32x3_off < 0 || fa.ln_n != 256 || a.Kp < 32 || a.Kp % 32 != 0 || a.nu < 20 || a.nu > 22) return false;
  const int mode = x3_wave_mode();
  if (mode != 1) return mode == 2;
  return a.B * (a.Kp / 32) >= WaveX3Lay::WAVES * x3_device_cus();
}

hipError_t launch_fc_wave_x3(const SolveArgs& a, const FcArgs& fa, hipStream_t stream) {
  if (fa.w32x3_off < 0 || a.Kp <= 0 || a.Kp % 32 != 0 || a.nu < 20 || a.nu > 22) return hipErrorInvalidValue;
  const int wts = a.B * (a.Kp / 32);
  int grid = (wts + WaveX3Lay::WAVES - 1) / WaveX3Lay::WAVES;
  if (grid > x3_device_cus()) grid = x3_device_cus();
  auto go = [&](auto kern, int bytes) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       bytes);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * WaveX3Lay::WAVES), bytes, stream, a, fa);
    return hipGetLastError();
  };
  if (x3_pair_on(wts)) return launch_fc_wave_x3p(a, fa, stream);  // two waves per SIMD (kernels_fc_x3p.hip)
  const int form = x3_form(a.H, fa.x3_l1, fa.x3_f16, fa.w32f16_off);
  static const char* const names[4] = {
      MPPI_X3_F16_L0 ? "fc_wave32_x3_kernel<f16,l2=1>" : "fc_wave32_x3_kernel<l1=f16,l2=1>",
      MPPI_X3_F16_L0 ? "fc_wave32_x3_kernel<f16>" : "fc_wave32_x3_kernel<l1=f16>", "fc_wave32_x3_kernel<l1=2>",
      "fc_wave32_x3_kernel<l1=3>"};
  note_kernel(names[form]);
  auto by_form = [&](auto cost) {
    constexpr int C = decltype(cost)::value;
    constexpr int bytes = WaveX3Lay::bytes<C>();
    switch (form) {
      case 0: return go(fc_wave32_x3_kernel<C, 0>, bytes);
      case 1: return go(fc_wave32_x3_kernel<C, 1>, bytes);
      case 2: return go(fc_wave32_x3_kernel<C, 2>, bytes);
      default: return go(fc_wave32_x3_kernel<C, 3>, bytes);
    }
  };
  if (a.cost_kind == MPPI_COST_HUMANOID_V1) return by_form(std::integral_constant<int, MPPI_COST_HUMANOID_V1>{});
  return by_form(std::integral_constant<int, MPPI_COST_HUMANOID_V3>{});
}

}  // namespace mppi
