// fc_wave32_x3p_kernel (round 5): the split (MPPI_PREC_BF16X3, fp32-accurate) per-wave CA rollout at TWO waves per
// SIMD.  The same arithmetic as fc_wave32_x3_kernel (kernels_fc_x3.hip: split bf16, three 32x32x16 MFMAs per product,
// the same LDS image and W1 lo stream), 8 waves and 256 samples per CU, so that one wave's VALU phases (the hi / lo
// splits, the statistic, the cost) can run beside the other wave's MFMAs instead of stalling a lone wave's in-order
// stream (the one-wave kernel: MFMA pipe 0.625 busy, 0.61 of its wave cycles issuing; profiles/r05_pmc_x3*).  Two waves
// per SIMD leave 256 registers per wave, so every layer is STREAMED instead of materialised:
//   * layer 0 runs one D-tile (32 rows) at a time; its ReLU'd, split output -- two k-steps of layer 1's operand -- is
//     consumed by layer 1's 24 MFMAs for those k-steps at once (all four layer-1 D-tiles accumulate in 64 registers),
//     so 16 registers of layer-0 activations are live instead of 128;
//   * the last layer likewise consumes layer 1's output one D-tile (two k-steps) at a time;
//   * the state part of the running cost is evaluated from the registers at every step (lane half 0 of each sample,
//     after one v_permlane32_swap per slot 4..6), so there is no LDS cost ring: the LDS holds the 144 KiB image and
//     b1 / bx only.
// Its own translation unit, so that its machine-scheduler flags are its own (build.py PER_FILE_FLAGS).
#include <cstdlib>

#include "x3_common.h"

namespace mppi {

#define X3P_WAVES 8
#ifndef X3P_HQ  // W1 hi read-ahead (stream positions)
#define X3P_HQ 1
#endif
#ifndef X3P_LQ  // W1 lo read-ahead (stream positions; 4 = one k-step).  With layer 1 at two MFMAs per product one k-step
                // no longer covers the L2 latency: 6 positions 729.7 -> 723.7 us per 64-solve rollout (two same-box
                // pairs; 2 for hi, or 8 for lo (spills), slower: profiles/r05_ab_x3p_readahead.log)
#define X3P_LQ 6
#endif
#ifndef X3P_EPI_PF  // the last layer software-pipelined one D-tile ahead (its fragments and layer 1's epilogue), 2: with
                    // the scheduler told to interleave each MFMA with VALU (round 5's bf16 form: -0.8..-1.9 % over
                    // five same-box pairs against 1, which was erratic there), 1: the pipelining alone -- in the fp16
                    // form 1 is the faster (381 vs 395 us per rollout on one box, 398 vs 400 on another, two pairs each:
                    // profiles/r06_ab_x3p_knobs_f16.log), 0: the round-5 order that clumped ~56 VALU before each tile's
                    // 12 MFMAs; bit-identical (profiles/r05_ab_x3p_epi_pf.log)
#define X3P_EPI_PF 1
#endif
#ifndef X3P_MU_SLOT  // -mu through the layer-0 MFMA (an operand slot against a column of 1.0) instead of the accumulators
#define X3P_MU_SLOT 1
#endif
#ifndef X3P_STAGGER  // waves 4..7 (each SIMD's second wave) start this many x 64 cycles late (s_sleep), 0 = together
#define X3P_STAGGER 0
#endif
#ifndef X3P_PRIO  // waves 4..7 at s_setprio X3P_PRIO for the whole kernel (0: equal priority, age decides)
#define X3P_PRIO 0
#endif
#ifndef X3P_COST_PAIR  // the state cost evaluated every second step for two steps at once, lane half 1 taking the
                       // earlier one (its 9 values kept in registers): half the cost VALU (1), or every step on half 0 (0)
#define X3P_COST_PAIR 0
#endif
#ifndef X3P_L0LO_QV0  // the fp16 form's layer 0: W lo on the qvel rows' first k-step (state slots 32..47, qvel weights
                      // only) too (1), or hi only there (0: 4 MFMAs and 4 fragment reads fewer per wave-step; the CPU
                      // error budget puts the qvel block's lo at nothing measurable on model_cross --
                      // profiles/r06_x3_error_budget_f16.txt "f16x2wq" -- and the engine's probe checks this form; the
                      // second k-step, which carries b0 and beta' against 1.0 and s, keeps its lo)
#define X3P_L0LO_QV0 0
#endif
#ifndef MPPI_X3P_DIAG  // timing-only diagnostic builds (results wrong): 1 = no W1 lo stream, 2 = no hi / lo split VALU,
                       // 3 = both, 4 = 3 without the state cost
#define MPPI_X3P_DIAG 0
#endif
template <int HALF>
__device__ __forceinline__ void split32p(const f32x16& v, bf16x8& hi, bf16x8& lo) {
#if MPPI_X3P_DIAG >= 2
  constexpr int o = 8 * HALF;
  u32x4 hw;
#pragma unroll
  for (int q = 0; q < 4; ++q) hw[q] = pk_bf16(v[o + 2 * q], v[o + 2 * q + 1]);
  hi = __builtin_bit_cast(bf16x8, hw);
  lo = hi;
#else
  split32<HALF>(v, hi, lo);
#endif
}

template <int COST, int L1T>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2))) void fc_wave32_x3p_kernel(SolveArgs a,
                                                                                                    FcArgs net) {
  using Y = WaveX3Lay;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const KClock kc = kclock_begin(a);
  if (blockIdx.x == 0 && threadIdx.x == 0) *a.status = 0u;
  const int lane = threadIdx.x & 63, h = lane >> 5, n = lane & 31;
  const int wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  {
    const int4* s0 = reinterpret_cast<const int4*>(net.img + (L1T <= 1 ? net.w32f16_off : net.w32x3_off));
    int4* d = reinterpret_cast<int4*>(lds);
    stage_lds<64 * X3P_WAVES>(d, s0, Y::IMG / 16);
    float* v = reinterpret_cast<float*>(lds + Y::B1);
    if (threadIdx.x < 128) v[threadIdx.x] = reinterpret_cast<const float*>(net.img + net.b_off[1])[threadIdx.x];
    else if (threadIdx.x < 192)
      v[threadIdx.x] = reinterpret_cast<const float*>(net.img + net.b_off[2])[threadIdx.x - 128];
  }
  __syncthreads();
  if (wib >= 4) {
    if constexpr (X3P_PRIO > 0) __builtin_amdgcn_s_setprio(X3P_PRIO);
    if constexpr (X3P_STAGGER > 0) __builtin_amdgcn_s_sleep(X3P_STAGGER);
  }

  int fo = lane * 16;  // this lane's 16 B of a fragment; opaque per step (no hoisting of loop-invariant LDS reads)
  auto frag = [&](int base, int f) { return *reinterpret_cast<const bf16x8*>(lds + base + f * 1024 + fo); };
  const auto rW = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(net.img) + net.w32x3_l1lo_off, 0, 64 * 1024,
                                                    0x00020000);
  auto w1lo = [&](int f) {
    return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rW, lane * 16, f * 1024, 0));
  };
  const float* vb1 = reinterpret_cast<const float*>(lds + Y::B1) + 4 * h;
  const float* vbx = reinterpret_cast<const float*>(lds + Y::BX) + 4 * h;

  const int H = a.H;
  const int wps = a.Kp / 32;
  const int total = a.B * wps;
  const float inv_n = 1.0f / (float)net.ln_n;
  const float cl = a.ctrl_clamp > 0.0f ? a.ctrl_clamp : INFINITY;
  auto state_src = [&](int sl) {
    return sl < 32 ? (sl < net.qp ? sl : -1) : (sl - 32 < net.qv ? net.qp + sl - 32 : -1);
  };
  constexpr int NJ = 11;  // controls c = 2 j + h (requires 20 <= nu <= 22: launch_fc_wave_x3)
  constexpr CostIdx ci = cost_idx(COST);
  static_assert(ci.n == 9 && ci.idx[3] == 3 && ci.idx[7] == 28, "the humanoid costs' state slots");
  // the state part of the running cost at 1-based step t1 from the register state: lane half 0 holds slots 0..3 (tile
  // 0 values 0..3) and 32, 33 (tile 1 values 0, 1), half 1 slots 4..7; one swap per slot gives half 0 slots 4..6.
  // Called by EVERY lane (the swaps read the other half's lanes, which an EXEC mask of half 0 would hide).
  auto gather_cost = [&](const f32x16 (&xs)[2], float (&v)[kCostMaxIdx]) {
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(xs[0][i]), __float_as_uint(xs[0][i]), false, false);
      v[4 + i] = __uint_as_float(p[1]);  // lanes 0..31: the value of lane + 32 (slot 4 + i)
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = xs[0][i];
    v[7] = xs[1][0];
    v[8] = xs[1][1];
  };
  auto state_cost = [&](const f32x16 (&xs)[2], const float* cx, int t1) {
    float v[kCostMaxIdx];
    gather_cost(xs, v);
    return cost_eval_t<COST>(v, 0.0f, 0.0f, cx, t1);
  };

  for (int wt = blockIdx.x + gridDim.x * wib; wt < total; wt += gridDim.x * X3P_WAVES) {
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
    float pv[kCostMaxIdx] = {};  // X3P_COST_PAIR: the even step's cost values (lane half 0), for the next odd step

    for (int t = 0; t < H; ++t) {
      asm volatile("" : "+v"(fo));
      // ---- control part of the running cost of step t (lane half h: controls 2 j + h)
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
      // MPPI_X3_F16_L0 (mppi_internal.h): the fp16 form's layer 0 and statistic too, fp16 W hi + lo against ONE fp16
      // operand (the state rounded to fp16, -mu as an fp16 hi / lo pair in slots 29 / 31, s in slot 30)
      constexpr bool L0H = L1T <= 1 && MPPI_X3_F16_L0;
      bf16x8 xh[4], xl[4];
      if constexpr (L0H) {
        (void)xl;
        xh[0] = h16<0>(x[0]);
        xh[1] = h16<1>(x[0]);
        xh[2] = h16<0>(x[1]);
        xh[3] = h16<1>(x[1]);
      } else {
        split32p<0>(x[0], xh[0], xl[0]);
        split32p<1>(x[0], xh[1], xl[1]);
        split32p<0>(x[1], xh[2], xl[2]);
        split32p<1>(x[1], xh[3], xl[3]);
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
        if constexpr (L0H) {
          // word 2 = (1.0, -mu_hi) at slots 28, 29; word 3 = (s, -mu_lo) at slots 30, 31 (L0x: 1.0 in column 31)
          const unsigned mhi = pk_f16(0.0f, -mu);
          const unsigned w3 = pk_f16(sc, -mu - f16_hi_value(mhi));
          u32x4 h1 = __builtin_bit_cast(u32x4, xh[1]), h3 = __builtin_bit_cast(u32x4, xh[3]);
          h1[2] = h == 1 ? (h1[2] & 0xFFFFu) | (mhi & 0xFFFF0000u) : h1[2];
          h3[2] = h == 1 ? (h3[2] & 0xFFFFu) | (mhi & 0xFFFF0000u) : h3[2];
          h1[3] = h == 1 ? w3 : h1[3];
          h3[3] = h == 1 ? w3 : h3[3];
          xh[1] = __builtin_bit_cast(bf16x8, h1);
          xh[3] = __builtin_bit_cast(bf16x8, h3);
        } else {
        const unsigned shi = pk_bf16(sc, 0.0f);
        const unsigned slo = pk_bf16(sc - __uint_as_float(shi << 16), 0.0f);
        u32x4 h1 = __builtin_bit_cast(u32x4, xh[1]), l1 = __builtin_bit_cast(u32x4, xl[1]);
        u32x4 h3 = __builtin_bit_cast(u32x4, xh[3]), l3 = __builtin_bit_cast(u32x4, xl[3]);
        h1[3] = h == 1 ? (h1[3] & 0xFFFF0000u) | (shi & 0xFFFFu) : h1[3];
        l1[3] = h == 1 ? (l1[3] & 0xFFFF0000u) | (slo & 0xFFFFu) : l1[3];
        h3[3] = h == 1 ? (h3[3] & 0xFFFF0000u) | (shi & 0xFFFFu) : h3[3];
        l3[3] = h == 1 ? (l3[3] & 0xFFFF0000u) | (slo & 0xFFFFu) : l3[3];
#if X3P_MU_SLOT
        // -mu (hi / lo) into slots 29 / 61 (value 13 of lane half 1: word 2's upper half), against L0x's column of 1.0:
        // the layer-0 accumulators start at 0 instead of a broadcast -mu tile (16 moves and 16 live registers)
        const unsigned mhi = pk_bf16(0.0f, -mu);
        const unsigned mlo = pk_bf16(0.0f, -mu - __uint_as_float(mhi & 0xFFFF0000u));
        h1[2] = h == 1 ? (h1[2] & 0xFFFFu) | (mhi & 0xFFFF0000u) : h1[2];
        l1[2] = h == 1 ? (l1[2] & 0xFFFFu) | (mlo & 0xFFFF0000u) : l1[2];
        h3[2] = h == 1 ? (h3[2] & 0xFFFFu) | (mhi & 0xFFFF0000u) : h3[2];
        l3[2] = h == 1 ? (l3[2] & 0xFFFFu) | (mlo & 0xFFFF0000u) : l3[2];
#endif
        xh[1] = __builtin_bit_cast(bf16x8, h1);
        xl[1] = __builtin_bit_cast(bf16x8, l1);
        xh[3] = __builtin_bit_cast(bf16x8, h3);
        xl[3] = __builtin_bit_cast(bf16x8, l3);
        }
      }

      // ---- layer 0 one D-tile at a time, each streamed into layer 1: relu(h + beta' s) -> hi / lo = layer 1's k-steps
      // 2 T, 2 T + 1, consumed at once by the four layer-1 D-tiles.  Every fragment is read ahead of its MFMAs: W1's hi
      // (LDS) one MFMA triple ahead, its lo (L2) one k-step ahead, the next layer-0 tile's (LDS) during this tile's
      // layer-1 part -- at 256 registers per wave the compiler otherwise reads each just before its MFMA and waits.
      f32x16 z[4] = {{}, {}, {}, {}};
      // W1's fragments of stream position q = 8 T + 4 kk + T1 (fragment T1 * 16 + 2 T + kk) read ahead through
      // register rings: hi (LDS) X3P_HQ positions ahead, lo (L2) X3P_LQ positions ahead
      auto w1f = [](int q) { return (q & 3) * 16 + (q >> 2); };
      bf16x8 l1q[X3P_LQ], hq[X3P_HQ];
#pragma unroll
      for (int j = 0; j < X3P_LQ; ++j) l1q[j] = L1T <= 1 ? bf16x8{} : w1lo(w1f(j));
#pragma unroll
      for (int j = 0; j < X3P_HQ; ++j) hq[j] = frag(Y::W1H, w1f(j));
      bf16x8 w0h[2], w0l[2];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        w0h[kk] = frag(Y::W0H, kk);
        w0l[kk] = frag(Y::W0L, kk);
      }
#pragma unroll
      for (int T = 0; T < 8; ++T) {
        f32x16 acc;
#pragma unroll
        for (int v = 0; v < 16; ++v) acc[v] = X3P_MU_SLOT ? 0.0f : -mu;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          if (L0H && !X3P_L0LO_QV0 && T >= 4 && kk == 0)
            acc = mma32h(w0h[kk], xh[2], acc);  // the qvel rows' first k-step: hi only
          else
            acc = mm0(w0h[kk], w0l[kk], (T < 4 ? 0 : 2) + kk, acc);
        }
        if (T + 1 < 8) {
#pragma unroll
          for (int kk = 0; kk < 2; ++kk) {
            w0h[kk] = frag(Y::W0H, 2 * (T + 1) + kk);
            if (!(L0H && !X3P_L0LO_QV0 && T + 1 >= 4 && kk == 0)) w0l[kk] = frag(Y::W0L, 2 * (T + 1) + kk);
          }
        }
        bf16x8 ah[2], al[2];
        if constexpr (L1T <= 1) {  // the fp16 form: layer 1's operand as ReLU'd fp16 (fc_common.h x3_f16_on)
          (void)al;
          ah[0] = h16_relu<0>(acc);
          ah[1] = h16_relu<1>(acc);
        } else if constexpr (L1T == 2) {  // layer 1 reads its operand's hi part only (fc_common.h x3_l1_terms), ReLU'd packed
          (void)al;
          ah[0] = hi32_relu<0>(acc);
          ah[1] = hi32_relu<1>(acc);
        } else {
#pragma unroll
          for (int v = 0; v < 16; ++v) acc[v] = __builtin_amdgcn_fmed3f(acc[v], 0.0f, 3.402823466e38f);
          split32p<0>(acc, ah[0], al[0]);
          split32p<1>(acc, ah[1], al[1]);
        }
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
          for (int T1 = 0; T1 < 4; ++T1) {
            const int q = 8 * T + 4 * kk + T1;
            const bf16x8 hi = hq[q % X3P_HQ], lo = l1q[q % X3P_LQ];
            if (q + X3P_HQ < 64) hq[q % X3P_HQ] = frag(Y::W1H, w1f(q + X3P_HQ));
            if constexpr (L1T <= 1) {  // one fp16 product (W1 in fp16 at W1H), no lo stream
              (void)lo;
              z[T1] = mma32h(hi, ah[kk], z[T1]);
              continue;
            }
#if MPPI_X3P_DIAG == 1 || MPPI_X3P_DIAG >= 3  // timing only (wrong results): W1's lo fragments not streamed from L2
            (void)lo;
            z[T1] = mma3(hi, hi, ah[kk], al[kk], z[T1]);
#else
            if (q + X3P_LQ < 64) l1q[q % X3P_LQ] = w1lo(w1f(q + X3P_LQ));
            if constexpr (L1T == 2)
              z[T1] = mma32(hi, ah[kk], mma32(lo, ah[kk], z[T1]));  // W1_lo a_hi + W1_hi a_hi
            else
              z[T1] = mma3(hi, lo, ah[kk], al[kk], z[T1]);
#endif
          }
        }
      }
      load_u(t + 1 < H ? t + 1 : t, un);  // the next step's controls

      // ---- layer 1's output one D-tile at a time (z = rstd (W1 a) + b1, ReLU, hi / lo) streamed into the last layer
#if X3P_EPI_PF
      // software-pipelined (X3P_EPI_PF): the last layer's 8 fragments of tile T1 + 1 (LDS) and its epilogue (VALU) are
      // issued before tile T1's 12 MFMAs, so neither waits on the other (the registers of layers 0 / 1's rings are free)
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
        auto epi = [&](int T1, bf16x8 (&ah)[2], bf16x8 (&al)[2]) {
#pragma unroll
          for (int g8 = 0; g8 < 4; ++g8) {
            const f32x4 b1 = *reinterpret_cast<const f32x4*>(vb1 + 32 * T1 + 8 * g8);
#pragma unroll
            for (int r = 0; r < 4; ++r)
              z[T1][4 * g8 + r] = L1T <= 1 ? fmaf(z[T1][4 * g8 + r], rstd, b1[r])  // (ReLU after fp16 packing)
                                           : __builtin_amdgcn_fmed3f(fmaf(z[T1][4 * g8 + r], rstd, b1[r]), 0.0f,
                                                                     3.402823466e38f);
          }
          if constexpr (L1T <= 1) {
            ah[0] = h16_relu<0>(z[T1]);
            ah[1] = h16_relu<1>(z[T1]);
          } else {
            split32p<0>(z[T1], ah[0], al[0]);
            split32p<1>(z[T1], ah[1], al[1]);
          }
        };
        auto wx = [&](int T1, bf16x8 (&fh)[4], bf16x8 (&fl)[4]) {
#pragma unroll
          for (int kk = 0; kk < 2; ++kk)
#pragma unroll
            for (int T = 0; T < 2; ++T) {
              const int f = T * 8 + 2 * T1 + kk;
              fh[2 * kk + T] = frag(Y::WXH, f);
              fl[2 * kk + T] = frag(Y::WXL, f);
            }
        };
        bf16x8 ah[2][2], al[2][2], fh[4], fl[4];
        wx(0, fh, fl);
        epi(0, ah[0], al[0]);
#if X3P_EPI_PF >= 2
        __builtin_amdgcn_sched_barrier(0);
#endif
#pragma unroll
        for (int T1 = 0; T1 < 4; ++T1) {
          const int c = T1 & 1;
#pragma unroll
          for (int kk = 0; kk < 2; ++kk)
#pragma unroll
            for (int T = 0; T < 2; ++T)
              d[T] = L1T == 0 ? mma32h(fh[2 * kk + T], ah[c][kk], d[T])  // fp16, one product
                     : L1T <= 1 ? mma32h(fh[2 * kk + T], ah[c][kk], mma32h(fl[2 * kk + T], ah[c][kk], d[T]))  // hi + lo
                              : mma3(fh[2 * kk + T], fl[2 * kk + T], ah[c][kk], al[c][kk], d[T]);
          if (T1 + 1 < 4) {
            wx(T1 + 1, fh, fl);
            epi(T1 + 1, ah[c ^ 1], al[c ^ 1]);
#if X3P_EPI_PF >= 2  // the scheduler told to interleave: the LDS reads first, then each MFMA followed by VALU
            __builtin_amdgcn_sched_group_barrier(0x100, 12, 0);
            constexpr int nm = L1T <= 1 ? 8 : 12;  // MFMAs per tile; VALU per MFMA: fp16 ~32 / 8, bf16 ~56 / 12
#pragma unroll
            for (int i = 0; i < nm; ++i) {
              __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
              __builtin_amdgcn_sched_group_barrier(0x002, L1T <= 1 ? 4 : 5, 0);
            }
#endif
          }
#if X3P_EPI_PF >= 2
          __builtin_amdgcn_sched_barrier(0);
#endif
        }
#pragma unroll
        for (int T = 0; T < 2; ++T) x[T] += d[T];
      }
#else
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
        for (int T1 = 0; T1 < 4; ++T1) {
#pragma unroll
          for (int g8 = 0; g8 < 4; ++g8) {
            const f32x4 b1 = *reinterpret_cast<const f32x4*>(vb1 + 32 * T1 + 8 * g8);
#pragma unroll
            for (int r = 0; r < 4; ++r)
              z[T1][4 * g8 + r] = __builtin_amdgcn_fmed3f(fmaf(z[T1][4 * g8 + r], rstd, b1[r]), 0.0f, 3.402823466e38f);
          }
          bf16x8 ah[2], al[2];
          split32p<0>(z[T1], ah[0], al[0]);
          split32p<1>(z[T1], ah[1], al[1]);
#pragma unroll
          for (int kk = 0; kk < 2; ++kk)
#pragma unroll
            for (int T = 0; T < 2; ++T) {
              const int f = T * 8 + 2 * T1 + kk;
              d[T] = mma3(frag(Y::WXH, f), frag(Y::WXL, f), ah[kk], al[kk], d[T]);
            }
        }
#pragma unroll
        for (int T = 0; T < 2; ++T) x[T] += d[T];
      }
#endif
      // ---- state part of the running cost of step t (its post-step state x_{t+1}; 1-based t + 1), evaluated by every
      // lane (the opaque asm keeps the compiler from sinking it into a lane-half-0 branch, where the swaps would read
      // the masked half) and kept on lane half 0
#if MPPI_X3P_DIAG < 4
      if constexpr (X3P_COST_PAIR) {
        float v[kCostMaxIdx];
        gather_cost(x, v);  // lane half 0: x_{t+1}'s
        if ((t & 1) == 0 && t + 1 < H) {  // an even step with a successor: kept for the next step
#pragma unroll
          for (int i = 0; i < kCostMaxIdx; ++i) pv[i] = v[i];
        } else {  // an odd step: half 1 takes step t - 1's (pv, from half 0); or the last step alone
#pragma unroll
          for (int i = 0; i < kCostMaxIdx; ++i) {
            auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(pv[i]), __float_as_uint(pv[i]), false, false);
            v[i] = h == 0 ? v[i] : __uint_as_float(p[0]);  // lanes 32..63: the value of lane - 32
          }
          float sc = cost_eval_t<COST>(v, 0.0f, 0.0f, cx, h == 0 ? t + 1 : t);
          asm volatile("" : "+v"(sc));
          cost += (h == 0 || (t & 1)) ? sc : 0.0f;
        }
      } else {
        float sc = state_cost(x, cx, t + 1);
        asm volatile("" : "+v"(sc));
        cost += h == 0 ? sc : 0.0f;
      }
#endif
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

hipError_t launch_fc_wave_x3p(const SolveArgs& a, const FcArgs& fa, hipStream_t stream) {
  const int wts = a.B * (a.Kp / 32);
  int grid = (wts + X3P_WAVES - 1) / X3P_WAVES;  // 8 wave-tiles per CU and round
  if (grid > x3_device_cus()) grid = x3_device_cus();
  auto go = [&](auto kern) {
    const int bytes = WaveX3Lay::RING;  // the image + b1 / bx (no cost ring)
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       bytes);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * X3P_WAVES), bytes, stream, a, fa);
    return hipGetLastError();
  };
  const int form = x3_form(a.H, fa.x3_l1, fa.x3_f16, fa.w32f16_off);
  static const char* const names[4] = {
      MPPI_X3_F16_L0 ? "fc_wave32_x3p_kernel<f16,l2=1>" : "fc_wave32_x3p_kernel<l1=f16,l2=1>",
      MPPI_X3_F16_L0 ? "fc_wave32_x3p_kernel<f16>" : "fc_wave32_x3p_kernel<l1=f16>", "fc_wave32_x3p_kernel<l1=2>",
      "fc_wave32_x3p_kernel<l1=3>"};
  note_kernel(names[form]);
  auto by_form = [&](auto cost) {
    constexpr int C = decltype(cost)::value;
    switch (form) {
      case 0: return go(fc_wave32_x3p_kernel<C, 0>);
      case 1: return go(fc_wave32_x3p_kernel<C, 1>);
      case 2: return go(fc_wave32_x3p_kernel<C, 2>);
      default: return go(fc_wave32_x3p_kernel<C, 3>);
    }
  };
  if (a.cost_kind == MPPI_COST_HUMANOID_V1) return by_form(std::integral_constant<int, MPPI_COST_HUMANOID_V1>{});
  return by_form(std::integral_constant<int, MPPI_COST_HUMANOID_V3>{});
}

}  // namespace mppi
