// Per-wave rollout of the folded humanoid CrossAttention surrogate (bf16; BASELINE config #4 with many solves per
// GPU).  Same network and the same bf16-operand / fp32-accumulate arithmetic as fc_rollout_kernel<kArchCA>
// (fc_rollout.h), organised the other way round:
//
//   * ONE wave owns NS sample tiles of 16 samples (NS = 2: 32 consecutive samples of one solve) for the whole horizon
//     and runs every layer for them itself: the accumulator layout of layer l, packed to bf16, IS the B operand of
//     layer l+1 (the host permutes the weights' k order, mppi_nets.cpp::pack_image), so activations never leave the
//     wave's registers -- no LDS exchange, no barrier anywhere in the horizon loop;
//   * every weight fragment lives ONCE per CU, in LDS (one 512-thread block of 8 waves per CU, 2 per SIMD): each wave
//     streams the 112 A fragments of a step through ds_read_b128, and with NS = 2 each fragment feeds two MFMAs (one
//     per sample tile), so the LDS stream is half the matrix pipe's rate and the kernel is MFMA-bound;
//   * the folded LayerNorm needs rstd = rsqrt(mean(h^2) + eps) of the layer-0 output h, which the M-split kernel gets
//     from a cross-wave sum AFTER layer 0.  Here mean(h^2) = x~^T G x~ / n = |R x~|^2 / n comes first, from the
//     Cholesky factor R of the Gram matrix G of the bf16 layer-0 columns (upper triangular in slot order; hi + lo bf16
//     fragments: 12 MFMAs per tile, exact to ~2^-18 of mean(h^2)), so layer 0 then runs in
//     chunks whose outputs go straight to bf16: relu(h rstd + beta') = rstd relu(h + beta' s), s = 1/rstd, with
//     beta' s added by the MFMA itself (beta' as a bf16 hi / lo pair in the pad columns 30, 31, 59 of layer 0 against
//     s_hi, s_hi, s_lo in the operand) and rstd applied to layer 1's output: z1 = rstd (W1 a) + b1;
//   * layer 0's bias rides in the MFMA too (the b0 hi / lo pair in pad slots 28, 29, which hold 1.0 in the state);
//   * running cost: the control part every step (lane group g: controls g, g + 4, ...), the state part from a
//     per-wave LDS ring of 4 / NS steps, one (step, tile, sample) per lane at every flush.
// Used for batches with many tiles per CU (launch_fc_wave); small batches keep the M-split kernel, which spreads one
// tile's step over 4 SIMDs.
#include "fc_rollout.h"

#include <cstdlib>

namespace mppi {

typedef __attribute__((ext_vector_type(4))) unsigned u32x4;

// LDS image (bytes): the layers' A fragments [m-tile][k-step][64 lanes][16 B], G_hi, G_lo, b1, bx; then each wave's
// cost ring [4 / NS steps][NS tiles][16 samples][HS] fp32
struct WaveLay {
  static constexpr int W0 = 0;                  // 16 x 2 fragments
  static constexpr int W1 = W0 + 32 * 1024;     // 8 x 8
  static constexpr int WX = W1 + 64 * 1024;     // 4 x 4
  static constexpr int GH = WX + 16 * 1024;     // 4 x 2
  static constexpr int GL = GH + 8 * 1024;      // 4 x 2
  static constexpr int B1 = GL + 8 * 1024;      // 128 f32
  static constexpr int BX = B1 + 512;           // 64 f32
  static constexpr int B0 = BX + 256;           // 128 f32: layer 0's centred bias, qpos-fed rows (fc_wave32_kernel, BD 2)
  static constexpr int RING = B0 + 512;
  static constexpr int WAVES = 8;
  template <int COST>
  static constexpr int ring_bytes() { return 4 * 16 * CostChunks<kArchCA, COST>::HS * 4; }  // 4 (step, tile) slots
  template <int COST>
  static constexpr int bytes() { return RING + WAVES * ring_bytes<COST>(); }
};

__device__ __forceinline__ unsigned pk_bf16(float a, float b) {  // one v_cvt_pk_bf16_f32 (RNE)
  return __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{a, b}, bf16x2));
}
__device__ __forceinline__ unsigned pk_bf16_relu(float a, float b) {  // + one v_pk_max_i16 (see P::put_tile_relu)
  return __builtin_bit_cast(unsigned,
                            __builtin_elementwise_max(__builtin_bit_cast(i16x2, pk_bf16(a, b)), i16x2{0, 0}));
}
// B operand of k-step ks from the accumulator tiles 2 ks (elements 0..3) and 2 ks + 1 (elements 4..7)
__device__ __forceinline__ bf16x8 bop(const f32x4& lo, const f32x4& hi) {
  return __builtin_bit_cast(bf16x8, u32x4{pk_bf16(lo[0], lo[1]), pk_bf16(lo[2], lo[3]), pk_bf16(hi[0], hi[1]),
                                          pk_bf16(hi[2], hi[3])});
}
__device__ __forceinline__ bf16x8 bop_relu(const f32x4& lo, const f32x4& hi) {
  return __builtin_bit_cast(bf16x8, u32x4{pk_bf16_relu(lo[0], lo[1]), pk_bf16_relu(lo[2], lo[3]),
                                          pk_bf16_relu(hi[0], hi[1]), pk_bf16_relu(hi[2], hi[3])});
}
__device__ __forceinline__ f32x4 mma(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// The step's 128 A fragments in the order the step consumes them (sequence index j), as fragment indices into the LDS
// image (1 KiB each: W0 from 0, W1 from 32, WX from 96, G_hi from 112, G_lo from 120).  Layer 1 runs in parts of MP
// m-tiles.
#ifndef MPPI_WAVE_L1MP
#define MPPI_WAVE_L1MP 4
#endif
constexpr int kWaveL1MP = MPPI_WAVE_L1MP;
// BD = 0: the dense (centred) layer 0, 16 m-tiles x 2 k-steps, 124 fragments per step.  BD = 2 (mppi_nets.cpp,
// w32_bd 2, the same image form as fc_wave32_kernel's): m-tiles 0..7 (qpos-fed rows) read k-step 0, 8..15 (qvel-fed)
// k-step 1, 108 fragments.
template <int BD>
struct WaveSeq {
  static constexpr int L0 = BD ? 16 : 32, L1 = 12 + L0, LX = L1 + 64, FRAGS = LX + 16;
  static constexpr int frag(int j) {
    // Cholesky factor R of the Gram matrix: m-tiles 0, 1 read both k-steps (R_hi, R_hi, R_lo, R_lo), m-tiles 2, 3 only
    // k-step 1 (R is upper triangular in slot order: its rows 32.. touch slots 32.. only)
    if (j < 8) return (j % 4 < 2 ? 112 : 120) + (j / 4) * 2 + (j % 2);
    if (j < 12) return ((j - 8) % 2 == 0 ? 112 : 120) + (2 + (j - 8) / 2) * 2 + 1;
    if (j < L1) return BD ? 2 * (j - 12) + ((j - 12) >= 8 ? 1 : 0) : j - 12;  // W0: (m-tile, k-step) in order
    if (j < LX) {  // W1: part p, k-step kk, m-tile MP p + i
      const int m = j - L1, p = m / (8 * kWaveL1MP), kk = (m / kWaveL1MP) % 8, i = m % kWaveL1MP;
      return 32 + (kWaveL1MP * p + i) * 8 + kk;
    }
    const int m = j - LX;  // WX: k-step kk, m-tile i
    return 96 + (m % 4) * 4 + m / 4;
  }
};

template <int COST, int NS, int BD>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2))) void fc_wave_kernel(SolveArgs a,
                                                                                              FcArgs net) {
  using Y = WaveLay;
  using Q = WaveSeq<BD>;
  using CC = CostChunks<kArchCA, COST>;
  constexpr int R = 4 / NS;  // ring steps: every lane evaluates one (step, tile, sample) per flush
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const KClock kc = kclock_begin(a);
  if (blockIdx.x == 0 && threadIdx.x == 0) *a.status = 0u;
  const int lane = threadIdx.x & 63, g = lane >> 4, n = lane & 15;
  const int wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);

  // ---- the weight image into LDS, once per block: W0 | W1 | WX are contiguous in the global image
  {
    const int4* s0 = reinterpret_cast<const int4*>(net.img + net.w_off[0]);
    const int4* sg = reinterpret_cast<const int4*>(net.img + (BD ? net.gbd_off : net.g_off));
    const int4* sb = reinterpret_cast<const int4*>(net.img + net.w0bd_off);  // BD: the block-diagonal layer 0
    int4* d = reinterpret_cast<int4*>(lds);
    constexpr int NW = (Y::GH - Y::W0) / 16, NG = (Y::B1 - Y::GH) / 16, N0 = (Y::W1 - Y::W0) / 16;
    if (BD) {
      stage_lds<512>(d, sb, N0);
      stage_lds<512>(d + N0, s0 + N0, NW - N0);
    } else {
      stage_lds<512>(d, s0, NW);
    }
    stage_lds<512>(d + Y::GH / 16, sg, NG);
    float* v = reinterpret_cast<float*>(lds + Y::B1);
    if (threadIdx.x < 128) v[threadIdx.x] = reinterpret_cast<const float*>(net.img + net.b_off[1])[threadIdx.x];
    else if (threadIdx.x < 192)
      v[threadIdx.x] = reinterpret_cast<const float*>(net.img + net.b_off[2])[threadIdx.x - 128];
    else if (threadIdx.x < 320)  // B0 follows BX: layer 0's centred bias, rows 0..127
      v[threadIdx.x] = reinterpret_cast<const float*>(net.img + net.b_off[0])[threadIdx.x - 192];
  }
  __syncthreads();

#ifdef MPPI_WAVE_PRIO  // A/B variant: static issue priority for the second wave of each SIMD (waves 4..7)
  if (wib >= 4) __builtin_amdgcn_s_setprio(1);
#endif
#ifdef MPPI_WAVE_STAGGER  // A/B variant: waves 4..7 start MPPI_WAVE_STAGGER x 8128 cycles later
  if (wib >= 4)
    for (int i = 0; i < MPPI_WAVE_STAGGER; ++i) __builtin_amdgcn_s_sleep(127);
#endif
  static_assert(Y::W1 == 32 * 1024 && Y::WX == 96 * 1024 && Y::GH == 112 * 1024 && Y::GL == 120 * 1024, "wave_frag");
  // LDS byte offsets of this lane's 16 B of fragment 0 and fragment 64 (fragments 64.. lie past ds_read's 16-bit
  // offset field: a second base register), made opaque once per step (opaque_bases) so hipcc neither folds them into
  // one base plus a v_add per read nor hoists the loop-invariant reads out of the horizon loop into (spilled) registers
  int fo_lo = lane * 16, fo_hi = lane * 16 + 64 * 1024;
  auto opaque_bases = [&]() { asm volatile("" : "+v"(fo_lo), "+v"(fo_hi)); };
  auto frag_at = [&](int f) {
    return *reinterpret_cast<const bf16x8*>(lds + (f < 64 ? fo_lo + f * 1024 : fo_hi + (f - 64) * 1024));
  };
#ifndef MPPI_WAVE_RING
#define MPPI_WAVE_RING 4
#endif
#if MPPI_WAVE_RING > 0
  // fragments read MPPI_WAVE_RING ahead of their MFMAs, through a register ring that runs on across phases, steps and
  // wave-tiles (the sequence repeats every step).  Same-box A/B, config #4 at 64 solves: no ring (the compiler's own
  // schedule reads 4 fragments, waits, issues their 8 MFMAs) 441 us per rollout, ring of 4 412 us, ring of 8 (layer 1
  // in parts of 2 m-tiles to make room; 6 VGPRs spilled) 422 us
  constexpr int D = MPPI_WAVE_RING;
  static_assert(Q::FRAGS % D == 0, "ring");
  bf16x8 F[D];
#pragma unroll
  for (int j = 0; j < D; ++j) F[j] = frag_at(Q::frag(j));
  auto take = [&](int j) {
    const bf16x8 f = F[j % D];
    F[j % D] = frag_at(Q::frag((j + D) % Q::FRAGS));
    return f;
  };
#else
  auto take = [&](int j) { return frag_at(Q::frag(j)); };
#endif
  const float* vb1 = reinterpret_cast<const float*>(lds + Y::B1) + 4 * g;
  const float* vb0 = reinterpret_cast<const float*>(lds + Y::B0) + 4 * g;
  const float* vbx = reinterpret_cast<const float*>(lds + Y::BX) + 4 * g;
  float* ring = reinterpret_cast<float*>(lds + Y::RING + wib * Y::ring_bytes<COST>());

  const int H = a.H;
  const int wps = a.Kp / (16 * NS);  // wave-tiles per solve
  const int total = a.B * wps;
  const float inv_n = 1.0f / (float)net.ln_n;
  const float cl = a.ctrl_clamp > 0.0f ? a.ctrl_clamp : INFINITY;
  auto state_src = [&](int sl) {
    return sl < 32 ? (sl < net.qp ? sl : -1) : (sl - 32 < net.qv ? net.qp + sl - 32 : -1);
  };
  // ring chunks this lane stores: state tile mt, lane group g (only the slots the cost reads)
  int chunk[4];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) {
    chunk[mt] = -1;
#pragma unroll
    for (int e = 0; e < 16; ++e)
      if (e == 4 * mt + g) chunk[mt] = CC::chunk(e / 4, e % 4);
  }
  // this lane's controls u = g + 4 j (j < 6), pad slots past nu read 0 through the buffer range
  constexpr int NJ = (kMaxNu + 3) / 4 < 6 ? (kMaxNu + 3) / 4 : 6;
  static_assert(NJ * 4 >= 21, "the humanoid's 21 controls over 4 lane groups");

  for (int wt = blockIdx.x + gridDim.x * wib; wt < total; wt += gridDim.x * Y::WAVES) {
    const int b = __builtin_amdgcn_readfirstlane(wt / wps);
    const int k0 = (wt - b * wps) * 16 * NS;  // first sample of tile 0
    float cx[MPPI_CTX_MAX];
#pragma unroll
    for (int i = 0; i < MPPI_CTX_MAX; ++i) cx[i] = a.ctx ? a.ctx[(long)b * MPPI_CTX_MAX + i] : a.ctx_default[i];
    // fp32 state in the accumulator layout (slot 16 mt + 4 g + r of sample n); 1.0 in the b0 slots (their rows of the
    // last layer are 0, so they stay 1.0), 0 in the other pads
    f32x4 x[NS][4];
    {
      // per-wave-tile x0 offsets from an opaque lane group (see fc_wave32_kernel: not hoisted out of the tile loop)
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
          const bool one = sl == kCaBiasSlotHi || sl == kCaBiasSlotLo ||
                           (BD != 0 && (sl == kCaBdBiasSlotHi || sl == kCaBdBiasSlotLo));
          const float v = one ? 1.0f : xv;
#pragma unroll
          for (int s = 0; s < NS; ++s) x[s][mt][r] = v;
        }
    }
    const auto rU = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.U) + (long)b * a.nu * H, 0,
                                                      a.nu * H * 4, 0x00020000);
    const auto rE = __builtin_amdgcn_make_buffer_rsrc(a.noise + (long)b * a.nu * H * a.Kp, 0,
                                                      a.nu * H * a.Kp * 4, 0x00020000);
    // per-lane offsets of control u = g (j = 0) and u = g + 4 (NJ - 1) (a pad slot past nu: out of the buffer's range,
    // which reads 0); controls g + 4 j in between add j 16 H (Kp) bytes through the scalar offset
    const int ul = g + 4 * (NJ - 1);
    const int uoff0 = g * H * 4, eoff0 = (g * H * a.Kp + k0 + n) * 4;
    const int uoffl = ul < a.nu ? ul * H * 4 : 0x7FFFFFF0;
    const int eoffl = ul < a.nu ? (ul * H * a.Kp + k0 + n) * 4 : 0x7FFFFFF0;
    static_assert(NJ >= 2, "");
    auto load_u = [&](int t, float (&c)[NS][NJ]) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const bool last = j == NJ - 1;
        const float uv = __uint_as_float(
            __builtin_amdgcn_raw_buffer_load_b32(rU, last ? uoffl : uoff0, t * 4 + (last ? 0 : j * 16 * H), 0));
#pragma unroll
        for (int s = 0; s < NS; ++s)
          c[s][j] = uv + __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
                             rE, last ? eoffl : eoff0, (t * a.Kp + 16 * s + (last ? 0 : j * 4 * H * a.Kp)) * 4, 0));
      }
    };
    float un[NS][NJ];
    load_u(0, un);
    float cost[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) cost[s] = 0.0f;
    // state part of the cost of (ring slot rs, tile s, sample n) from the ring
    auto ring_cost = [&](int rs, int s, int t1) {
      const float* row = ring + ((rs * NS + s) * 16 + n) * CC::HS;
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
      opaque_bases();
      // ---- layer-0 operand (bf16 state; b0 slots 1.0) and mean(h^2) from the Gram matrix
      bf16x8 xb[NS][2];
      float rstd[NS], mu[NS];
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        xb[s][0] = bop(x[s][0], x[s][1]);
        xb[s][1] = bop(x[s][2], x[s][3]);
      }
      {
        f32x4 gx[NS][4];  // R x~ (R: the Gram matrix's Cholesky factor, hi + lo)
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
          if (mt < 2) {
            const bf16x8 h0 = take(4 * mt), h1 = take(4 * mt + 1), l0 = take(4 * mt + 2), l1 = take(4 * mt + 3);
#pragma unroll
            for (int s = 0; s < NS; ++s) {
              gx[s][mt] = mma(h0, xb[s][0], f32x4{0.0f, 0.0f, 0.0f, 0.0f});
              gx[s][mt] = mma(h1, xb[s][1], gx[s][mt]);
#ifndef MPPI_WAVE_GRAM1  // A/B timing variant only (numerics differ): R_hi alone
              gx[s][mt] = mma(l0, xb[s][0], gx[s][mt]);
              gx[s][mt] = mma(l1, xb[s][1], gx[s][mt]);
#endif
            }
          } else {
            const bf16x8 h1 = take(8 + 2 * (mt - 2)), l1 = take(9 + 2 * (mt - 2));
#pragma unroll
            for (int s = 0; s < NS; ++s) {
              gx[s][mt] = mma(h1, xb[s][1], f32x4{0.0f, 0.0f, 0.0f, 0.0f});
#ifndef MPPI_WAVE_GRAM1
              gx[s][mt] = mma(l1, xb[s][1], gx[s][mt]);
#endif
            }
          }
        }
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          mu[s] = 0.0f;
          if constexpr (BD != 0) {  // R's pad row 30 (m-tile 1, lane group 3, value 2) is the row mean m~: mu = m~ x~
            const float m30 = g == 3 ? gx[s][1][2] : 0.0f;
            gx[s][1][2] = g == 3 ? 0.0f : gx[s][1][2];
            mu[s] = group_sum(m30);
          }
          // q = |R x~|^2: this lane's 16 rows, then the 4 lane groups
          float qa = 0.0f, qb = 0.0f;
#pragma unroll
          for (int mt = 0; mt < 4; ++mt) {
            qa = fmaf(gx[s][mt][0], gx[s][mt][0], qa);
            qb = fmaf(gx[s][mt][1], gx[s][mt][1], qb);
            qa = fmaf(gx[s][mt][2], gx[s][mt][2], qa);
            qb = fmaf(gx[s][mt][3], gx[s][mt][3], qb);
          }
          const float q = group_sum(qa + qb);
          const float v = fmaf(q, inv_n, 1e-5f);  // >= 1e-5: no denormal
          rstd[s] = __builtin_amdgcn_rsqf(v);
          const float sc = v * rstd[s];  // s = sqrt(var + eps)
          const unsigned shi = pk_bf16(sc, sc);
          const float lo = sc - __uint_as_float(shi << 16);
          const unsigned slo = pk_bf16(lo, lo);
          // s into the beta' slots of the operand: 30, 31 (k-step 0, lane group 3, elements 6, 7) = s_hi; 59 (k-step
          // 1, lane group 2, element 7) = s_lo (element 6 there is the state slot 58)
          u32x4 w0 = __builtin_bit_cast(u32x4, xb[s][0]), w1 = __builtin_bit_cast(u32x4, xb[s][1]);
          w0[3] = g == 3 ? shi : w0[3];
          w1[3] = g == 2 ? ((w1[3] & 0xFFFFu) | (slo & 0xFFFF0000u)) : w1[3];
          if constexpr (BD != 0) {  // slot 29 (lane group 3, element 5) = s_lo; 62, 63 (k-step 1, group 3) = s_hi
            w0[2] = g == 3 ? ((w0[2] & 0xFFFFu) | (slo & 0xFFFF0000u)) : w0[2];
            w1[3] = g == 3 ? shi : w1[3];
          }
          xb[s][0] = __builtin_bit_cast(bf16x8, w0);
          xb[s][1] = __builtin_bit_cast(bf16x8, w1);
        }
      }

      // ---- layer 0 in 8 chunks of 2 m-tiles: relu(h + beta' s) -> bf16, the layer-1 operand of k-step c
      bf16x8 a1[NS][8];
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        f32x4 h[NS][2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          if constexpr (BD != 0) {  // one k-step per m-tile; the accumulators start at (qpos rows: b0c) - mu
            const int mt = 2 * c + i;
            const bf16x8 f = take(12 + mt);
            const f32x4 bb = mt < 8 ? *reinterpret_cast<const f32x4*>(vb0 + 16 * mt) : f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
            for (int s = 0; s < NS; ++s) {
              const f32x4 c0 = bb - f32x4{mu[s], mu[s], mu[s], mu[s]};
              h[s][i] = mma(f, xb[s][mt < 8 ? 0 : 1], c0);
            }
          } else {
            const bf16x8 f0 = take(12 + (2 * c + i) * 2), f1 = take(12 + (2 * c + i) * 2 + 1);
#pragma unroll
            for (int s = 0; s < NS; ++s) {
              h[s][i] = mma(f0, xb[s][0], f32x4{0.0f, 0.0f, 0.0f, 0.0f});
              h[s][i] = mma(f1, xb[s][1], h[s][i]);
            }
          }
        }
#pragma unroll
        for (int s = 0; s < NS; ++s) a1[s][c] = bop_relu(h[s][0], h[s][1]);
      }

      // ---- control part of the running cost of step t (loaded during the previous step's last layer)
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        float usq = 0.0f;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const float u = __builtin_amdgcn_fmed3f(un[s][j], -cl, cl);
          usq = fmaf(u, u, usq);
        }
        cost[s] += ctrl_term_t<COST>(g == 0 ? __builtin_amdgcn_fmed3f(un[s][0], -cl, cl) : 0.0f, usq);
      }

      // ---- layer 1 in parts of MP m-tiles: z = rstd (W1 a) + b1, relu -> bf16, the last layer's operand
      constexpr int MP = kWaveL1MP;
      bf16x8 a2[NS][4];
#pragma unroll
      for (int hh = 0; hh < 8 / MP; ++hh) {
        f32x4 z[NS][MP];
#pragma unroll
        for (int kk = 0; kk < 8; ++kk)
#pragma unroll
          for (int i = 0; i < MP; ++i) {
            const bf16x8 f = take(Q::L1 + hh * 8 * MP + kk * MP + i);
#pragma unroll
            for (int s = 0; s < NS; ++s)
              z[s][i] = mma(f, a1[s][kk], kk == 0 ? f32x4{0.0f, 0.0f, 0.0f, 0.0f} : z[s][i]);
          }
#pragma unroll
        for (int i = 0; i < MP; ++i) {
          const f32x4 b1 = *reinterpret_cast<const f32x4*>(vb1 + 16 * (MP * hh + i));
#pragma unroll
          for (int s = 0; s < NS; ++s) {
#ifdef MPPI_WAVE_PK
            const f32x2 r2 = {rstd[s], rstd[s]};
            const f32x2 lo = f32x2{z[s][i][0], z[s][i][1]} * r2 + f32x2{b1[0], b1[1]};
            const f32x2 hi = f32x2{z[s][i][2], z[s][i][3]} * r2 + f32x2{b1[2], b1[3]};
            z[s][i] = f32x4{lo.x, lo.y, hi.x, hi.y};
#else
#pragma unroll
            for (int r = 0; r < 4; ++r) z[s][i][r] = fmaf(z[s][i][r], rstd[s], b1[r]);
#endif
          }
        }
#pragma unroll
        for (int s = 0; s < NS; ++s)
#pragma unroll
          for (int i = 0; i < MP; i += 2) a2[s][(MP * hh + i) / 2] = bop_relu(z[s][i], z[s][i + 1]);
      }

      // the next step's controls, issued after layer 1 (the register peak) and consumed after its layer 0
      load_u(t + 1 < H ? t + 1 : t, un);

      // ---- last layer: x += bx + Wx a2 (fp32 state)
      {
        f32x4 d[NS][4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const f32x4 bx = *reinterpret_cast<const f32x4*>(vbx + 16 * i);
#pragma unroll
          for (int s = 0; s < NS; ++s) d[s][i] = bx;
        }
#pragma unroll
        for (int kk = 0; kk < 4; ++kk)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const bf16x8 f = take(Q::LX + kk * 4 + i);
#pragma unroll
            for (int s = 0; s < NS; ++s) d[s][i] = mma(f, a2[s][kk], d[s][i]);
          }
#pragma unroll
        for (int s = 0; s < NS; ++s)
#pragma unroll
          for (int i = 0; i < 4; ++i) x[s][i] += d[s][i];
      }

      // ---- the state slots the cost reads into the ring; flush every R steps (and after the last step)
#pragma unroll
      for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
          if (chunk[mt] >= 0)
            *reinterpret_cast<f32x4*>(ring + (((t % R) * NS + s) * 16 + n) * CC::HS + 4 * chunk[mt]) = x[s][mt];
      if ((t + 1) % R == 0 || t + 1 == H) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the ring rows this wave just wrote
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const int rs = g % R, s = g / R;  // this lane: ring step rs of tile s
        const int ts = t - t % R + rs;
        if (ts <= t) {
          const float c = ring_cost(rs, s, ts + 1);
#pragma unroll
          for (int s2 = 0; s2 < NS; ++s2) cost[s2] += s == s2 ? c : 0.0f;
        }
        __builtin_amdgcn_wave_barrier();  // reads done before the next steps overwrite the ring
      }
    }
    // terminal cost on x_H (the ring slot of step H - 1), once per (tile, sample): lanes of ring step 0
    if (a.terminal_weight != 0.0f && g % R == 0) {
      const int s = g / R;
      const float c = a.terminal_weight * ring_cost((H - 1) % R, s, H);
#pragma unroll
      for (int s2 = 0; s2 < NS; ++s2) cost[s2] += s == s2 ? c : 0.0f;
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const float c = group_sum(cost[s]);
      const int k = k0 + 16 * s + n;
      if (g == 0 && k < a.K) a.costs[(long)b * a.Kp + k] = isfinite(c) ? c : INFINITY;
    }
    if (a.xout && k0 == 0 && n == 0) {  // env step: final state of sample 0 of the solve
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int src = state_src(16 * mt + 4 * g + r);
          if (src >= 0) a.xout[(long)b * a.nx + src] = x[0][mt][r];
        }
    }
  }
  __syncthreads();
  kclock_record(a, kc);
}

// ------------------------------------------------------------------------------------------ 32x32x16 variant

// fc_wave_kernel with v_mfma_f32_32x32x16_bf16: one wave's 32 samples are ONE MFMA column block, so a step issues half
// as many MFMA instructions (124 instead of 248) for the same matrix-pipe time.  An MFMA holds its SIMD's vector issue
// for 8 cycles (MI355X_MICROARCH.md, constants table), 8 of 16 for 16x16x32 but 8 of 32 here: the VALU work of the step
// (bf16 conversions, the LayerNorm statistic and scale, the costs) gets three times the issue room beside the MFMAs.
// Layouts: a 32x32 accumulator tile (D-tile T, 32 rows) holds in lane l the 16 values v = 4 i + r of rows
// 32 T + 8 i + 4 (l >> 5) + r for sample l & 31; its values 0..7 / 8..15 packed to bf16 are the next layer's B operand
// of k-steps 2 T / 2 T + 1 (the host packs the A fragments in that k order: mppi_nets.cpp, w32_off).  The image holds
// the same fragment indices as fc_wave_kernel's (W0 0.., W1 32.., WX 96.., R_hi 112.., R_lo 120..).
typedef __attribute__((ext_vector_type(16))) float f32x16;
__device__ __forceinline__ f32x16 mma32(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
template <int HALF>
__device__ __forceinline__ bf16x8 bop32(const f32x16& v) {
  constexpr int o = 8 * HALF;
  return __builtin_bit_cast(bf16x8, u32x4{pk_bf16(v[o], v[o + 1]), pk_bf16(v[o + 2], v[o + 3]),
                                          pk_bf16(v[o + 4], v[o + 5]), pk_bf16(v[o + 6], v[o + 7])});
}
template <int HALF>
__device__ __forceinline__ bf16x8 bop32_relu(const f32x16& v) {
  constexpr int o = 8 * HALF;
  return __builtin_bit_cast(bf16x8, u32x4{pk_bf16_relu(v[o], v[o + 1]), pk_bf16_relu(v[o + 2], v[o + 3]),
                                          pk_bf16_relu(v[o + 4], v[o + 5]), pk_bf16_relu(v[o + 6], v[o + 7])});
}
#ifndef MPPI_WAVE32_RING
#define MPPI_WAVE32_RING 4
#endif
// software-pipelined conversions (1: layer 0, 2: and layer 1); same-box A/B, config #4 at 64 solves
// (profiles/r03_ab_wave.log [swp]): 364.9 / 364.2 us per rollout -> 1: 364.5 / 362.2 -> 2: 359.5 / 360.3
#ifndef MPPI_WAVE32_SWP
#define MPPI_WAVE32_SWP 2
#endif
// The step's fragment sequence.  BD = 0: the dense (centred) layer 0, every (D-tile, k-step): 124 MFMAs per
// wave-step.  BD = 1, 2: the block-diagonal layer 0 (mppi_nets.cpp, w32_bd): D-tiles 0..3 (qpos-fed rows) read
// k-steps 0, 1 and, for BD = 1, the pad k-step 3 (its beta' s_lo column), D-tiles 4..7 (qvel-fed) k-steps 2, 3: 112
// MFMAs; BD = 2 takes the qpos rows' bias through their accumulators instead, 108.
template <int BD>
struct W32Seq {
  static constexpr bool use(int T, int ks) { return BD == 0 || (T < 4 ? (ks < 2 || (BD == 1 && ks == 3)) : ks >= 2); }
  static constexpr int pos(int T, int ks) {  // sequence position of (T, ks) among layer 0's MFMAs
    int p = 0;
    for (int t = 0; t < T; ++t)
      for (int k = 0; k < 4; ++k) p += use(t, k) ? 1 : 0;
    for (int k = 0; k < ks; ++k) p += use(T, k) ? 1 : 0;
    return p;
  }
  static constexpr int L1 = 12 + pos(8, 0), LX = L1 + 64, USED = LX + 16;  // dense: 44, 108, 124
  // padded to a multiple of 8 positions for an 8-deep ring (the padding positions are never used: dead reads)
  static constexpr int FRAGS = MPPI_WAVE32_RING == 8 ? (USED + 7) / 8 * 8 : USED;
  static constexpr int frag(int j) {
    if (j >= USED) return 0;
    if (j < 4) return 112 + j;              // R_hi, D-tile 0, k-steps 0..3
    if (j < 8) return 120 + (j - 4);        // R_lo, D-tile 0
    if (j < 10) return 116 + 2 + (j - 8);   // R_hi, D-tile 1, k-steps 2, 3 (R is upper triangular)
    if (j < 12) return 124 + 2 + (j - 10);  // R_lo, D-tile 1
    if (j < L1) {                           // W0: (D-tile, k-step) in order
      for (int T = 0; T < 8; ++T)
        for (int ks = 0; ks < 4; ++ks)
          if (use(T, ks) && 12 + pos(T, ks) == j) return 4 * T + ks;
      return 0;
    }
    if (j < LX) {  // W1: parts of 2 D-tiles, k-step ks, D-tile 2 p + i
#if MPPI_WAVE32_SWP >= 2
      const int m = j - L1, p = m / 32, i = (m / 16) % 2, ks = m % 16;  // D-tile-major within a part
#else
      const int m = j - L1, p = m / 32, ks = (m / 2) % 16, i = m % 2;
#endif
      return 32 + (2 * p + i) * 16 + ks;
    }
    const int m = j - LX;  // WX: k-step ks, D-tile T
    return 96 + (m % 2) * 8 + m / 2;
  }
};

template <int COST, int BD>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2))) void fc_wave32_kernel(SolveArgs a,
                                                                                                FcArgs net) {
  using Y = WaveLay;
  using Q = W32Seq<BD>;
  using CC = CostChunks<kArchCA, COST>;
  constexpr int R = 2;  // ring steps: lane half h evaluates ring step h of its sample at each flush
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const KClock kc = kclock_begin(a);
  if (blockIdx.x == 0 && threadIdx.x == 0) *a.status = 0u;
  const int lane = threadIdx.x & 63, h = lane >> 5, n = lane & 31;
  const int wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  {
    const int4* s0 = reinterpret_cast<const int4*>(net.img + net.w32_off);
    int4* d = reinterpret_cast<int4*>(lds);
    stage_lds<512>(d, s0, Y::B1 / 16);
    float* v = reinterpret_cast<float*>(lds + Y::B1);
    if (threadIdx.x < 128) v[threadIdx.x] = reinterpret_cast<const float*>(net.img + net.b_off[1])[threadIdx.x];
    else if (threadIdx.x < 192)
      v[threadIdx.x] = reinterpret_cast<const float*>(net.img + net.b_off[2])[threadIdx.x - 128];
    else if (threadIdx.x < 320)  // B0 follows BX: layer 0's centred bias, rows 0..127
      v[threadIdx.x] = reinterpret_cast<const float*>(net.img + net.b_off[0])[threadIdx.x - 192];
  }
  __syncthreads();

  int fo_lo = lane * 16, fo_hi = lane * 16 + 64 * 1024;  // see fc_wave_kernel
  auto opaque_bases = [&]() { asm volatile("" : "+v"(fo_lo), "+v"(fo_hi)); };
  auto frag_at = [&](int f) {
    return *reinterpret_cast<const bf16x8*>(lds + (f < 64 ? fo_lo + f * 1024 : fo_hi + (f - 64) * 1024));
  };
  constexpr int D = MPPI_WAVE32_RING;
  static_assert(Q::FRAGS % D == 0, "ring");
  bf16x8 F[D];
#pragma unroll
  for (int j = 0; j < D; ++j) F[j] = frag_at(Q::frag(j));
  auto take = [&](int j) {
    const bf16x8 f = F[j % D];
    F[j % D] = frag_at(Q::frag((j + D) % Q::FRAGS));
    return f;
  };
  // row 32 T + 8 i + 4 h + r of a bias vector: this lane's 4 values of value group i
  const float* vb1 = reinterpret_cast<const float*>(lds + Y::B1) + 4 * h;
  const float* vbx = reinterpret_cast<const float*>(lds + Y::BX) + 4 * h;
  const float* vb0 = reinterpret_cast<const float*>(lds + Y::B0) + 4 * h;
  float* ring = reinterpret_cast<float*>(lds + Y::RING + wib * Y::ring_bytes<COST>());

  const int H = a.H;
  const int wps = a.Kp / 32;
  const int total = a.B * wps;
  const float inv_n = 1.0f / (float)net.ln_n;
  const float cl = a.ctrl_clamp > 0.0f ? a.ctrl_clamp : INFINITY;
  auto state_src = [&](int sl) {
    return sl < 32 ? (sl < net.qp ? sl : -1) : (sl - 32 < net.qv ? net.qp + sl - 32 : -1);
  };
  // ring chunks of this lane half: D-tile T, value group i  <->  16-row tile 2 T + i / 2, lane group 2 (i % 2) + h
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
  constexpr int NJ = 11;  // controls c = 2 j + h (requires 20 <= nu <= 22: launch_fc_wave32)

  for (int wt = blockIdx.x + gridDim.x * wib; wt < total; wt += gridDim.x * Y::WAVES) {
    const int b = __builtin_amdgcn_readfirstlane(wt / wps);
    const int k0 = (wt - b * wps) * 32;
    float cx[MPPI_CTX_MAX];
#pragma unroll
    for (int i = 0; i < MPPI_CTX_MAX; ++i) cx[i] = a.ctx ? a.ctx[(long)b * MPPI_CTX_MAX + i] : a.ctx_default[i];
    f32x16 x[2];  // the state, D-tiles 0 (slots 0..31) and 1 (32..63); 1.0 in the b0 slots
    // the lane half through an opaque copy, so the 16 per-lane x0 offsets are derived here, per wave-tile: hoisted out of
    // the tile loop (loop-invariant) they were 16 64-bit addresses live across the whole horizon, 9 of them spilled at
    // 256 VGPRs: one scratch store of 72 B per lane per wave at kernel start, the 9.4 MB of WRITE_SIZE per config-#4
    // launch (2048 waves x 64 lanes x 72 B); buffer loads take a 32-bit offset and read 0 past the solve's row
    int ho = h;
    asm volatile("" : "+v"(ho));
    const auto rX = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.x0) + (long)b * a.nx, 0, a.nx * 4, 0x00020000);
#pragma unroll
    for (int T = 0; T < 2; ++T)
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int sl = 32 * T + 8 * (v / 4) + 4 * ho + v % 4, src = state_src(sl);
        const float xv = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rX, src >= 0 ? 4 * src : 0x7FFFFFF0, 0, 0));
        const bool one = sl == kCaBiasSlotHi || sl == kCaBiasSlotLo || (BD != 0 && (sl == kCaBdBiasSlotHi || sl == kCaBdBiasSlotLo));
        x[T][v] = one ? 1.0f : xv;
      }
    const auto rU = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.U) + (long)b * a.nu * H, 0,
                                                      a.nu * H * 4, 0x00020000);
    const auto rE = __builtin_amdgcn_make_buffer_rsrc(a.noise + (long)b * a.nu * H * a.Kp, 0,
                                                      a.nu * H * a.Kp * 4, 0x00020000);
    const int cl_ = 2 * (NJ - 1) + h;  // the last control slot of this lane half (a pad past nu reads 0)
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
      opaque_bases();
#ifndef MPPI_WAVE32_CTRL_LATE
      // ---- control part of the running cost of step t (loaded during the previous step's last layer)
      {
        float usq = 0.0f;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const float u = __builtin_amdgcn_fmed3f(un[j], -cl, cl);
          usq = fmaf(u, u, usq);
        }
        cost += ctrl_term_t<COST>(h == 0 ? __builtin_amdgcn_fmed3f(un[0], -cl, cl) : 0.0f, usq);
      }

#endif
      // ---- layer-0 operand and mean(h^2) = |R x~|^2 / n
      bf16x8 xb[4] = {bop32<0>(x[0]), bop32<1>(x[0]), bop32<0>(x[1]), bop32<1>(x[1])};
      float rstd, mu = 0.0f;
      {
        f32x16 g0 = {}, g1 = {};
#pragma unroll
        for (int j = 0; j < 8; ++j) g0 = mma32(take(j), xb[j % 4], g0);  // R_hi then R_lo, D-tile 0
#pragma unroll
        for (int j = 8; j < 12; ++j) g1 = mma32(take(j), xb[2 + j % 2], g1);  // D-tile 1: k-steps 2, 3
        if constexpr (BD != 0) {  // R's pad row 30 (value 14 of lane half 1) is the row mean m~: mu = m~ x~, not squared
          const float m14 = g0[14];
          g0[14] = h == 1 ? 0.0f : m14;
          auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(m14), __float_as_uint(m14), false, false);
          mu = h == 1 ? m14 : __uint_as_float(p[1]);  // p[1]: lanes 0..31 receive lanes 32..63's value
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
        {  // + the other lane half (rows 4..7 of each group of 8)
          auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(q), __float_as_uint(q), false, false);
          q = __uint_as_float(p[0]) + __uint_as_float(p[1]);
        }
        const float v = fmaf(q, inv_n, 1e-5f);
        rstd = __builtin_amdgcn_rsqf(v);
        const float sc = v * rstd;
        const unsigned shi = pk_bf16(sc, sc);
        const float lo = sc - __uint_as_float(shi << 16);
        const unsigned slo = pk_bf16(lo, lo);
        // beta' slots: 30, 31 (k-step 1, lane half 1, elements 6, 7) = s_hi; 59 (k-step 3, lane half 0, element 7) = s_lo
        u32x4 w1 = __builtin_bit_cast(u32x4, xb[1]), w3 = __builtin_bit_cast(u32x4, xb[3]);
        w1[3] = h == 1 ? shi : w1[3];
        // BD 2: s_lo in slot 29 (k-step 1, lane half 1, element 5) for the qpos rows' beta'_hi s_lo term (the
        // statistic above read the 1.0 there)
        if constexpr (BD == 2) w1[2] = h == 1 ? ((w1[2] & 0xFFFFu) | (slo & 0xFFFF0000u)) : w1[2];
        // BD: the qvel rows' beta' pair against s_hi in slots 62, 63 (k-step 3, lane half 1, elements 6, 7)
        w3[3] = h == 0 ? ((w3[3] & 0xFFFFu) | (slo & 0xFFFF0000u)) : (BD != 0 ? shi : w3[3]);
        xb[1] = __builtin_bit_cast(bf16x8, w1);
        xb[3] = __builtin_bit_cast(bf16x8, w3);
      }

      // ---- layer 0, one D-tile (32 rows) at a time -> relu -> bf16: layer 1's k-steps 2 T, 2 T + 1
#ifdef MPPI_WAVE32_SGB
      __builtin_amdgcn_sched_barrier(0);  // the interleave groups below start at layer 0
#endif
      bf16x8 a1[16];
#if MPPI_WAVE32_SWP >= 1
      // tile T's conversion issued after tile T+1's MFMAs (program order pinned by scheduling barriers), so the
      // wave's in-order issue does not wait on tile T's last MFMA before it can start tile T+1
      {
        f32x16 acc2[2];
        f32x16 c0 = {};  // BD: the LayerNorm centring -mu rides in every layer-0 tile's accumulator
        if constexpr (BD != 0) {
#pragma unroll
          for (int v = 0; v < 16; ++v) c0[v] = -mu;
        }
#pragma unroll
        for (int T = 0; T <= 8; ++T) {
          if (T < 8) {
            acc2[T & 1] = c0;
            if constexpr (BD == 2) {  // qpos rows: + their centred bias b0c (fp32, LDS)
              if (T < 4) {
#pragma unroll
                for (int g8 = 0; g8 < 4; ++g8) {
                  const f32x4 bb = *reinterpret_cast<const f32x4*>(vb0 + 32 * T + 8 * g8);
#pragma unroll
                  for (int r = 0; r < 4; ++r) acc2[T & 1][4 * g8 + r] = bb[r] - mu;
                }
              }
            }
#pragma unroll
            for (int ks = 0; ks < 4; ++ks)
              if (Q::use(T, ks)) acc2[T & 1] = mma32(take(12 + Q::pos(T, ks)), xb[ks], acc2[T & 1]);
          }
          __builtin_amdgcn_sched_barrier(0);
          if (T > 0) {
            a1[2 * (T - 1)] = bop32_relu<0>(acc2[(T - 1) & 1]);
            a1[2 * (T - 1) + 1] = bop32_relu<1>(acc2[(T - 1) & 1]);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      }
#else
#pragma unroll
      for (int T = 0; T < 8; ++T) {
        f32x16 acc = {};
        if constexpr (BD != 0) {
#pragma unroll
          for (int v = 0; v < 16; ++v) acc[v] = -mu;
        }
        if constexpr (BD == 2) {
          if (T < 4) {
#pragma unroll
            for (int g8 = 0; g8 < 4; ++g8) {
              const f32x4 bb = *reinterpret_cast<const f32x4*>(vb0 + 32 * T + 8 * g8);
#pragma unroll
              for (int r = 0; r < 4; ++r) acc[4 * g8 + r] = bb[r] - mu;
            }
          }
        }
#pragma unroll
        for (int ks = 0; ks < 4; ++ks)
          if (Q::use(T, ks)) acc = mma32(take(12 + Q::pos(T, ks)), xb[ks], acc);
        a1[2 * T] = bop32_relu<0>(acc);
        a1[2 * T + 1] = bop32_relu<1>(acc);
#ifdef MPPI_WAVE32_SGB  // A/B: the previous tile's conversion interleaved between this tile's MFMAs
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);
        }
#endif
      }
#endif
#ifdef MPPI_WAVE32_CTRL_LATE
      // ---- control part of the running cost of step t (loaded during the previous step)
      {
        float usq = 0.0f;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const float u = __builtin_amdgcn_fmed3f(un[j], -cl, cl);
          usq = fmaf(u, u, usq);
        }
        cost += ctrl_term_t<COST>(h == 0 ? __builtin_amdgcn_fmed3f(un[0], -cl, cl) : 0.0f, usq);
      }

#endif

      // ---- layer 1 in two parts of 2 D-tiles: z = rstd (W1 a) + b1, relu -> bf16
      bf16x8 a2[8];
#if MPPI_WAVE32_SWP >= 2
      // D-tile-major within a part; D-tile 0's bias + relu + bf16 issued after D-tile 1's first MFMAs
      auto conv1 = [&](f32x16& zz, int T) {
#pragma unroll
        for (int g8 = 0; g8 < 4; ++g8) {
          const f32x4 b1 = *reinterpret_cast<const f32x4*>(vb1 + 32 * T + 8 * g8);
#pragma unroll
          for (int r = 0; r < 4; ++r) zz[4 * g8 + r] = fmaf(zz[4 * g8 + r], rstd, b1[r]);
        }
        a2[2 * T] = bop32_relu<0>(zz);
        a2[2 * T + 1] = bop32_relu<1>(zz);
      };
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        f32x16 z0 = {}, z1 = {};
#pragma unroll
        for (int ks = 0; ks < 16; ++ks) z0 = mma32(take(Q::L1 + 32 * p + ks), a1[ks], z0);
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) z1 = mma32(take(Q::L1 + 32 * p + 16 + ks), a1[ks], z1);
        __builtin_amdgcn_sched_barrier(0);
        conv1(z0, 2 * p);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int ks = 2; ks < 16; ++ks) z1 = mma32(take(Q::L1 + 32 * p + 16 + ks), a1[ks], z1);
        conv1(z1, 2 * p + 1);
      }
#else
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        f32x16 z[2] = {{}, {}};
#pragma unroll
        for (int ks = 0; ks < 16; ++ks)
#pragma unroll
          for (int i = 0; i < 2; ++i) z[i] = mma32(take(Q::L1 + 32 * p + 2 * ks + i), a1[ks], z[i]);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int T = 2 * p + i;
#pragma unroll
          for (int g8 = 0; g8 < 4; ++g8) {
            const f32x4 b1 = *reinterpret_cast<const f32x4*>(vb1 + 32 * T + 8 * g8);
#pragma unroll
            for (int r = 0; r < 4; ++r) z[i][4 * g8 + r] = fmaf(z[i][4 * g8 + r], rstd, b1[r]);
          }
          a2[2 * T] = bop32_relu<0>(z[i]);
          a2[2 * T + 1] = bop32_relu<1>(z[i]);
        }
#if defined(MPPI_WAVE32_SGB) && MPPI_WAVE32_SGB >= 2  // A/B: part 0's conversion between part 1's MFMAs
        if (p == 1) {
#pragma unroll
          for (int k = 0; k < 32; ++k) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
          }
        }
#endif
      }
#endif
      load_u(t + 1 < H ? t + 1 : t, un);  // the next step's controls, consumed after its layer 0

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
          for (int T = 0; T < 2; ++T) d[T] = mma32(take(Q::LX + 2 * ks + T), a2[ks], d[T]);
#if defined(MPPI_WAVE32_SGB) && MPPI_WAVE32_SGB >= 2  // A/B: part 1's conversion between the last layer's MFMAs
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);
        }
#endif
#pragma unroll
        for (int T = 0; T < 2; ++T) x[T] += d[T];
      }
#pragma unroll
      for (int j = Q::USED; j < Q::FRAGS; ++j) (void)take(j);  // the padding positions (8-deep ring)

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
      int hs = h;  // opaque as for the x0 loads
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

// ------------------------------------------------------------------------------------------ MLP (hidden 128 x 2)

// The same per-wave organisation for MLPStatePredictor(nx, nu, 128, hidden_layers = 2) (learning/model.py:6-46): one
// wave runs all 4 layers of NS tiles, every weight fragment once per CU in LDS, read through the register ring.  No
// LayerNorm; the controls u = clamp(U + eps) are layer 0's third k-step (lane group g: controls 4g..4g+3, 16+4g..,
// the M-split kernel's slots), and their squares the running cost's control part; layer 0's bias rides in the MFMA
// (the image's b0 pair in pad slots 62, 63, which hold 1.0 here); b1, b2, b3 initialise the accumulators from LDS.
struct WaveMlpLay {
  static constexpr int W0 = 0;                // 8 m-tiles x 3 k-steps (state, state, controls)
  static constexpr int W1 = W0 + 24 * 1024;   // 8 x 4
  static constexpr int W2 = W1 + 32 * 1024;   // 8 x 4
  static constexpr int W3 = W2 + 32 * 1024;   // 4 x 4
  static constexpr int B1 = W3 + 16 * 1024;   // 128 f32
  static constexpr int B2 = B1 + 512;         // 128 f32
  static constexpr int B3 = B2 + 512;         // 64 f32
  static constexpr int RING = B3 + 256;
  static constexpr int WAVES = 8;
  template <int COST>
  static constexpr int ring_bytes() { return 4 * 16 * CostChunks<kArchMLP, COST>::HS * 4; }
  template <int COST>
  static constexpr int bytes() { return RING + WAVES * ring_bytes<COST>(); }
};
constexpr int kWaveMlpFrags = 104;  // 24 + 32 + 32 + 16
__host__ __device__ constexpr int wave_mlp_frag(int j) {
  if (j < 24) return j;  // W0 in (m-tile, k-step) order
  if (j < 88) {          // W1 (j < 56), W2: part p of MP m-tiles, k-step kk, m-tile MP p + i
    const int l = j < 56 ? 0 : 1, m = j - (l ? 56 : 24), p = m / (4 * kWaveL1MP), kk = (m / kWaveL1MP) % 4,
              i = m % kWaveL1MP;
    return 24 + 32 * l + (kWaveL1MP * p + i) * 4 + kk;
  }
  const int m = j - 88;  // W3: k-step kk, m-tile i
  return 88 + (m % 4) * 4 + m / 4;
}

template <int COST, int NS>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2))) void fc_wave_mlp_kernel(SolveArgs a,
                                                                                                  FcArgs net) {
  using Y = WaveMlpLay;
  using CC = CostChunks<kArchMLP, COST>;
  constexpr int R = 4 / NS;
  constexpr int MP = kWaveL1MP;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const KClock kc = kclock_begin(a);
  if (blockIdx.x == 0 && threadIdx.x == 0) *a.status = 0u;
  const int lane = threadIdx.x & 63, g = lane >> 4, n = lane & 15;
  const int wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  {  // the 4 layers' fragments are contiguous in the global image from w_off[0]; then b1, b2, b3
    const int4* s0 = reinterpret_cast<const int4*>(net.img + net.w_off[0]);
    int4* d = reinterpret_cast<int4*>(lds);
    stage_lds<512>(d, s0, Y::B1 / 16);
    float* v = reinterpret_cast<float*>(lds + Y::B1);
    if (threadIdx.x < 128) v[threadIdx.x] = reinterpret_cast<const float*>(net.img + net.b_off[1])[threadIdx.x];
    else if (threadIdx.x < 256)
      v[threadIdx.x] = reinterpret_cast<const float*>(net.img + net.b_off[2])[threadIdx.x - 128];
    else if (threadIdx.x < 320)
      v[threadIdx.x] = reinterpret_cast<const float*>(net.img + net.b_off[3])[threadIdx.x - 256];
  }
  __syncthreads();

  static_assert(Y::B1 == 104 * 1024, "wave_mlp_frag");
  int fo_lo = lane * 16, fo_hi = lane * 16 + 64 * 1024;  // fragments 0..63 / 64.. (see fc_wave_kernel)
  auto opaque_bases = [&]() { asm volatile("" : "+v"(fo_lo), "+v"(fo_hi)); };
  auto frag_at = [&](int f) {
    return *reinterpret_cast<const bf16x8*>(lds + (f < 64 ? fo_lo + f * 1024 : fo_hi + (f - 64) * 1024));
  };
  constexpr int D = MPPI_WAVE_RING > 0 ? MPPI_WAVE_RING : 4;
  static_assert(kWaveMlpFrags % D == 0, "ring");
  bf16x8 F[D];
#pragma unroll
  for (int j = 0; j < D; ++j) F[j] = frag_at(wave_mlp_frag(j));
  auto take = [&](int j) {
    const bf16x8 f = F[j % D];
    F[j % D] = frag_at(wave_mlp_frag((j + D) % kWaveMlpFrags));
    return f;
  };
  const float* vb1 = reinterpret_cast<const float*>(lds + Y::B1) + 4 * g;
  const float* vb2 = reinterpret_cast<const float*>(lds + Y::B2) + 4 * g;
  const float* vb3 = reinterpret_cast<const float*>(lds + Y::B3) + 4 * g;
  float* ring = reinterpret_cast<float*>(lds + Y::RING + wib * Y::ring_bytes<COST>());

  const int H = a.H;
  const int wps = a.Kp / (16 * NS);
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
    const int k0 = (wt - b * wps) * 16 * NS;
    float cx[MPPI_CTX_MAX];
#pragma unroll
    for (int i = 0; i < MPPI_CTX_MAX; ++i) cx[i] = a.ctx ? a.ctx[(long)b * MPPI_CTX_MAX + i] : a.ctx_default[i];
    f32x4 x[NS][4];
    {
      // per-wave-tile x0 offsets from an opaque lane group (see fc_wave32_kernel: not hoisted out of the tile loop)
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
          const float v = (sl == kMlpBiasSlotHi || sl == kMlpBiasSlotLo) ? 1.0f : xv;
#pragma unroll
          for (int s = 0; s < NS; ++s) x[s][mt][r] = v;
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
    auto load_u = [&](int t, float (&c)[NS][8]) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float uv = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rU, uoff[j], t * 4, 0));
#pragma unroll
        for (int s = 0; s < NS; ++s)
          c[s][j] = uv + __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rE, eoff[j], (t * a.Kp + 16 * s) * 4, 0));
      }
    };
    float un[NS][8];
    load_u(0, un);
    float cost[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) cost[s] = 0.0f;
    auto ring_cost = [&](int rs, int s, int t1) {
      const float* row = ring + ((rs * NS + s) * 16 + n) * CC::HS;
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
      opaque_bases();
      // ---- controls of step t (loaded a step ahead): clamp, the control part of the cost, layer 0's operand
      bf16x8 xb[NS][3];
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        f32x4 u0, u1;
        float usq = 0.0f;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          u0[j] = __builtin_amdgcn_fmed3f(un[s][j], -cl, cl);
          u1[j] = __builtin_amdgcn_fmed3f(un[s][4 + j], -cl, cl);
          usq = fmaf(u0[j], u0[j], usq);
          usq = fmaf(u1[j], u1[j], usq);
        }
        cost[s] += ctrl_term_t<COST>(g == 0 ? u0[0] : 0.0f, usq);
        xb[s][0] = bop(x[s][0], x[s][1]);
        xb[s][1] = bop(x[s][2], x[s][3]);
        xb[s][2] = bop(u0, u1);
      }
      load_u(t + 1 < H ? t + 1 : t, un);

      // ---- layer 0 in 4 chunks of 2 m-tiles -> relu -> bf16, layer 1's operand of k-step c
      bf16x8 a1[NS][4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        f32x4 h[NS][2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const bf16x8 f0 = take(6 * c + 3 * i), f1 = take(6 * c + 3 * i + 1), f2 = take(6 * c + 3 * i + 2);
#pragma unroll
          for (int s = 0; s < NS; ++s) {
            h[s][i] = mma(f0, xb[s][0], f32x4{0.0f, 0.0f, 0.0f, 0.0f});
            h[s][i] = mma(f1, xb[s][1], h[s][i]);
            h[s][i] = mma(f2, xb[s][2], h[s][i]);
          }
        }
#pragma unroll
        for (int s = 0; s < NS; ++s) a1[s][c] = bop_relu(h[s][0], h[s][1]);
      }

      // ---- hidden layers 1 and 2 (128 -> 128, bias from LDS as the accumulator's start, relu)
      bf16x8 a2[NS][4];
#pragma unroll
      for (int l = 0; l < 2; ++l) {
        const float* vb = l == 0 ? vb1 : vb2;
        const int j0 = l == 0 ? 24 : 56;
#pragma unroll
        for (int hh = 0; hh < 8 / MP; ++hh) {
          f32x4 z[NS][MP];
#pragma unroll
          for (int i = 0; i < MP; ++i) {
            const f32x4 bias = *reinterpret_cast<const f32x4*>(vb + 16 * (MP * hh + i));
#pragma unroll
            for (int s = 0; s < NS; ++s) z[s][i] = bias;
          }
#pragma unroll
          for (int kk = 0; kk < 4; ++kk)
#pragma unroll
            for (int i = 0; i < MP; ++i) {
              const bf16x8 f = take(j0 + hh * 4 * MP + kk * MP + i);
#pragma unroll
              for (int s = 0; s < NS; ++s) z[s][i] = mma(f, l == 0 ? a1[s][kk] : a2[s][kk], z[s][i]);
            }
#pragma unroll
          for (int s = 0; s < NS; ++s)
#pragma unroll
            for (int i = 0; i < MP; i += 2) {
              const bf16x8 o = bop_relu(z[s][i], z[s][i + 1]);
              if (l == 0) a2[s][(MP * hh + i) / 2] = o;
              else a1[s][(MP * hh + i) / 2] = o;  // layer 2's output reuses a1 (layer 1's input is dead)
            }
        }
      }

      // ---- last layer: x += b3 + W3 a (fp32 state)
      {
        f32x4 d[NS][4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const f32x4 b3 = *reinterpret_cast<const f32x4*>(vb3 + 16 * i);
#pragma unroll
          for (int s = 0; s < NS; ++s) d[s][i] = b3;
        }
#pragma unroll
        for (int kk = 0; kk < 4; ++kk)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const bf16x8 f = take(88 + kk * 4 + i);
#pragma unroll
            for (int s = 0; s < NS; ++s) d[s][i] = mma(f, a1[s][kk], d[s][i]);
          }
#pragma unroll
        for (int s = 0; s < NS; ++s)
#pragma unroll
          for (int i = 0; i < 4; ++i) x[s][i] += d[s][i];
      }

      // ---- cost ring (as fc_wave_kernel)
#pragma unroll
      for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
          if (chunk[mt] >= 0)
            *reinterpret_cast<f32x4*>(ring + (((t % R) * NS + s) * 16 + n) * CC::HS + 4 * chunk[mt]) = x[s][mt];
      if ((t + 1) % R == 0 || t + 1 == H) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const int rs = g % R, s = g / R;
        const int ts = t - t % R + rs;
        if (ts <= t) {
          const float c = ring_cost(rs, s, ts + 1);
#pragma unroll
          for (int s2 = 0; s2 < NS; ++s2) cost[s2] += s == s2 ? c : 0.0f;
        }
        __builtin_amdgcn_wave_barrier();
      }
    }
    if (a.terminal_weight != 0.0f && g % R == 0) {
      const int s = g / R;
      const float c = a.terminal_weight * ring_cost((H - 1) % R, s, H);
#pragma unroll
      for (int s2 = 0; s2 < NS; ++s2) cost[s2] += s == s2 ? c : 0.0f;
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const float c = group_sum(cost[s]);
      const int k = k0 + 16 * s + n;
      if (g == 0 && k < a.K) a.costs[(long)b * a.Kp + k] = isfinite(c) ? c : INFINITY;
    }
    if (a.xout && k0 == 0 && n == 0) {
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int src = state_src(16 * mt + 4 * g + r);
          if (src >= 0) a.xout[(long)b * a.nx + src] = x[0][mt][r];
        }
    }
  }
  __syncthreads();
  kclock_record(a, kc);
}

// MPPI_FC_WAVE: 0 never, 1 / 2 always with NS = 1 / 2 sample tiles per wave, 3 the 32x32x16 variant (read per launch,
// so a test can switch it); unset: by 16-sample tiles per CU, from a same-box sweep over config #4 batches (scripts/gpu_sweep_wave.sh,
// DESIGN.md §4): NS = 2 from 12 tiles per CU (48 solves and up), NS = 1 from 6 (24, 32 solves), below that the
// M-split kernel (16 solves: 153 us vs 185 us for NS = 1), which spreads one tile's step over 4 SIMDs
static int fc_wave_mode() {
  const char* e = std::getenv("MPPI_FC_WAVE");
  return e ? std::atoi(e) : -1;
}

static int wave_device_cus() { return current_device_cus(); }

int fc_wave_ns(const SolveArgs& a, const FcArgs& fa) {
  // a wave owns 32 samples of one solve (NS = 2, 32x32): only for Kp a multiple of 32.  The env-step launch (Kp = 16,
  // one sample) always takes the M-split kernel, also when MPPI_FC_WAVE forces these kernels.
  if (fa.g_off < 0 || fa.ln_n != 256 || a.Kp < 32 || a.Kp % 32 != 0) return 0;
  const int mode = fc_wave_mode();
  if (mode == 0) return 0;
  if (mode == 1 || mode == 2) return mode;
  const bool w32 = fa.w32_off >= 0 && a.nu >= 20 && a.nu <= 22;  // the 32x32x16 variant (fc_wave32_kernel)
  if (mode == 3) return w32 ? 3 : 2;
  const int tiles = a.B * (a.Kp >> 4), cus = wave_device_cus();
  // two tiles per wave: the 32x32x16 variant where it applies (two boxes, config #4 64 solves: 384.7-389.8 ->
  // 365.9-370.5 us; 378.5/378.8 -> 371.1/366.5 us)
  return tiles >= 12 * cus ? (w32 ? 3 : 2) : (tiles >= 6 * cus ? 1 : 0);
}

hipError_t launch_fc_wave(const SolveArgs& a, const FcArgs& fa, int ns, hipStream_t stream) {
  if (a.Kp <= 0 || a.Kp % (ns == 3 ? 32 : 16 * ns) != 0) return hipErrorInvalidValue;  // whole wave-tiles only
  if (ns == 3) {  // the 32x32x16 variant (32 samples per wave)
    if (fa.w32_off < 0 || a.nu < 20 || a.nu > 22) return hipErrorInvalidValue;
    const int wts = a.B * (a.Kp / 32);
    int grid = (wts + WaveLay::WAVES - 1) / WaveLay::WAVES;
    if (grid > wave_device_cus()) grid = wave_device_cus();
    auto go32 = [&](auto kern, int bytes) {
      hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
      if (e != hipSuccess) return e;
      hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * WaveLay::WAVES), bytes, stream, a, fa);
      return hipGetLastError();
    };
    const int b1 = WaveLay::bytes<MPPI_COST_HUMANOID_V1>(), b3 = WaveLay::bytes<MPPI_COST_HUMANOID_V3>();
    note_kernel("fc_wave32_kernel");
    if (a.cost_kind == MPPI_COST_HUMANOID_V1)
      return fa.w32_bd == 2   ? go32(fc_wave32_kernel<MPPI_COST_HUMANOID_V1, 2>, b1)
             : fa.w32_bd == 1 ? go32(fc_wave32_kernel<MPPI_COST_HUMANOID_V1, 1>, b1)
                              : go32(fc_wave32_kernel<MPPI_COST_HUMANOID_V1, 0>, b1);
    return fa.w32_bd == 2   ? go32(fc_wave32_kernel<MPPI_COST_HUMANOID_V3, 2>, b3)
           : fa.w32_bd == 1 ? go32(fc_wave32_kernel<MPPI_COST_HUMANOID_V3, 1>, b3)
                            : go32(fc_wave32_kernel<MPPI_COST_HUMANOID_V3, 0>, b3);
  }
  const int wts = a.B * (a.Kp / (16 * ns));
  const int cus = wave_device_cus();
  int grid = (wts + WaveLay::WAVES - 1) / WaveLay::WAVES;
  if (grid > cus) grid = cus;  // persistent: a wave takes wave-tiles wt, wt + 8 grid, ...
  const bool bd = fa.w32_bd == 2 && fa.w0bd_off >= 0 && fa.gbd_off >= 0;  // the block-diagonal layer 0 (form 2)
  auto go = [&](auto kern, int bytes) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * WaveLay::WAVES), bytes, stream, a, fa);
    return hipGetLastError();
  };
  constexpr int V1 = MPPI_COST_HUMANOID_V1, V3 = MPPI_COST_HUMANOID_V3;
  static_assert(WaveLay::bytes<V3>() <= 160 * 1024 && WaveLay::bytes<V1>() <= 160 * 1024, "LDS per CU");
  note_kernel(ns == 1 ? "fc_wave_kernel<ns=1>" : "fc_wave_kernel<ns=2>");
  if (a.cost_kind == V1)
    return bd ? (ns == 1 ? go(fc_wave_kernel<V1, 1, 2>, WaveLay::bytes<V1>()) : go(fc_wave_kernel<V1, 2, 2>, WaveLay::bytes<V1>()))
              : (ns == 1 ? go(fc_wave_kernel<V1, 1, 0>, WaveLay::bytes<V1>()) : go(fc_wave_kernel<V1, 2, 0>, WaveLay::bytes<V1>()));
  return bd ? (ns == 1 ? go(fc_wave_kernel<V3, 1, 2>, WaveLay::bytes<V3>()) : go(fc_wave_kernel<V3, 2, 2>, WaveLay::bytes<V3>()))
            : (ns == 1 ? go(fc_wave_kernel<V3, 1, 0>, WaveLay::bytes<V3>()) : go(fc_wave_kernel<V3, 2, 0>, WaveLay::bytes<V3>()));
}

}  // namespace mppi

namespace mppi {

// MLP: the same rule as the CA kernel (fc_wave_ns), to be confirmed by its own sweep
int fc_wave_mlp_ns(const SolveArgs& a, const FcArgs& fa) {
  if (!fa.wave || a.nx > kMlpBiasSlotHi || a.nu > 32 || a.Kp < 32 || a.Kp % 32 != 0) return 0;  // as fc_wave_ns
  const int mode = fc_wave_mode();
  if (mode == 0) return 0;
  if (mode == 1 || mode == 2) return mode;
  const int tiles = a.B * (a.Kp >> 4), cus = wave_device_cus();
  return tiles >= 12 * cus ? 2 : (tiles >= 6 * cus ? 1 : 0);
}

hipError_t launch_fc_wave_mlp(const SolveArgs& a, const FcArgs& fa, int ns, hipStream_t stream) {
  if (a.Kp <= 0 || a.Kp % (16 * ns) != 0) return hipErrorInvalidValue;  // whole wave-tiles only
  const int wts = a.B * (a.Kp / (16 * ns));
  int grid = (wts + WaveMlpLay::WAVES - 1) / WaveMlpLay::WAVES;
  if (grid > wave_device_cus()) grid = wave_device_cus();
  auto go = [&](auto kern, int bytes) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * WaveMlpLay::WAVES), bytes, stream, a, fa);
    return hipGetLastError();
  };
  note_kernel(ns == 1 ? "fc_wave_mlp_kernel<ns=1>" : "fc_wave_mlp_kernel<ns=2>");
#define MPPI_WAVE_MLP_COST(K)                                                                       \
  case K:                                                                                           \
    static_assert(WaveMlpLay::bytes<K>() <= 160 * 1024, "LDS per CU");                              \
    return ns == 1 ? go(fc_wave_mlp_kernel<K, 1>, WaveMlpLay::bytes<K>())                           \
                   : go(fc_wave_mlp_kernel<K, 2>, WaveMlpLay::bytes<K>());
  switch (a.cost_kind) {
    MPPI_WAVE_MLP_COST(MPPI_COST_HUMANOID_V3)
    MPPI_WAVE_MLP_COST(MPPI_COST_HUMANOID_V1)
    MPPI_WAVE_MLP_COST(MPPI_COST_QUAD_EST)
    MPPI_WAVE_MLP_COST(MPPI_COST_QUAD_JL)
    MPPI_WAVE_MLP_COST(MPPI_COST_CARTPOLE_EST)
    MPPI_WAVE_MLP_COST(MPPI_COST_CARTPOLE)
    default: return hipErrorInvalidValue;
  }
#undef MPPI_WAVE_MLP_COST
}

}  // namespace mppi
