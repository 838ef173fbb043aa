// fc_rollout_kernel_x3d (round 6): the split (MPPI_PREC_BF16X3, fp32-accurate) M-split CA rollout for the few-tiles
// regime -- the 8- and 16-solve shards of config #4 at N = 8 and N = 4 -- at TWO waves per SIMD.
//
// fc_rollout_kernel_x3w (fc_rollout.h) spreads one 16-sample group's step over 4 waves (M split) and gives every wave
// two groups (NS = 2) at ONE wave per SIMD, because each wave keeps all of its rows' hi / lo fragments in registers
// (224 of them).  Its step is the latency of a dependent chain -- layer 0, the LayerNorm statistic exchange, act0,
// layer 1, act1, the last layer, the state exchange: 4 barriers -- in which one in-order wave interleaves its two
// groups statically; the MFMA pipe was ~46 % busy (136 MFMAs per wave-step in ~2.3 us).
//
// Here a 512-thread block holds TWO groups of 4 waves (waves 0..3 = group 0, 4..7 = group 1: one wave of each group per
// SIMD), each wave one 16-sample tile (NS = 1), so the SIMD's two waves are independent instruction streams that the
// hardware interleaves dynamically.  To fit 256 registers per wave and keep both groups on one LDS:
//   * layer 1's hi / lo fragments (the largest layer, 128 registers) stay in registers (AGPRs, read by the asm MFMAs of
//     P<BF16X3>::mma_a2, the two-product layer 1);
//   * layers 0 and 2 (the last layer) live in LDS ONCE per block as separate hi and lo planes (96 KiB, conflict-free
//     ds_read_b128 per fragment), shared by both groups, read where they are used every step;
//   * the layer-0 bias and the folded LayerNorm's beta' are read from LDS too (registers), act0 is stored as its hi
//     plane only (the two-product layer 1 reads nothing else), and the cost ring holds 8 steps.
// The two groups share the block's s_barrier and step in lockstep: the SIMD's two waves run the same phase, and the
// hardware interleaves their MFMA chains, LDS round trips and VALU.  (X3D_OFFSET = 1 -- group 1 passing one barrier
// before its first step and group 0 one after its last, so every barrier interval pairs one group's MFMA phase with the
// other's exchange -- measured 9 % slower: each interval then lasts as long as the longer of two unequal phases.)
// PMC at 8 solves (profiles/r06_pmc_mfma_x3d_8.txt): 194 VALU, 68 MFMA, 61 LDS instructions per wave-step; MFMA busy
// 0.31; wave cycles 0.24 issuing, 0.33 dependency-stalled, 0.43 waiting (barriers, LDS) -- the per-step chain's latency.
//
// Only the two-product layer 1 (x3_l1_terms == 2) and the fp16 form (F16; fc_common.h x3_f16_on: layer 1 one fp16
// product from 64 AGPRs of fp16 fragments, act0 / act1 and (MPPI_X3_F16_L0) the state as single fp16 planes, layer 0
// and the last layer fp16 hi + lo against them) are built here; three products keep fc_rollout_kernel_x3w.  Its own
// translation unit (build.py PER_FILE_FLAGS).
#include "fc_rollout.h"

namespace mppi {

#ifndef X3D_OFFSET  // group 1's phase lag in barrier intervals: 0 = lockstep (the default).  8 solves, same box: 1 =
                    // 166-167 us per rollout against 152.5 us in lockstep (profiles/r06_ab_x3d.log)
#define X3D_OFFSET 0
#endif
#ifndef X3D_PD  // control loads this many steps ahead (the step loop unrolled by it, <= 3).  8 solves, same box: 1 =
                // 147.7 us, 2 = 145.2, 3 = 145.1 per rollout
#define X3D_PD 2
#endif

template <int COST>
struct X3dLay {
  using CC = CostChunks<kArchCA, COST>;
  static constexpr int RING = 8;  // cost-ring steps (lane groups ls = 4 wv + g < RING evaluate one (step, sample) each)
  // shared by both groups: layer 0 / layer 2 fragments as hi and lo planes, [fragment (mt, kk)][lane] x 16 B
  static constexpr int F0H = 0;                // 32 fragments: m-tile mt 0..15, k-step kk 0..1 at mt * 2 + kk
  static constexpr int F0L = F0H + 32 * 1024;
  static constexpr int F2H = F0L + 32 * 1024;  // 16 fragments: mt 0..3, kk 0..3 at mt * 4 + kk
  static constexpr int F2L = F2H + 16 * 1024;
  static constexpr int B0 = F2L + 16 * 1024;   // layer-0 bias, 256 fp32 (padded rows)
  static constexpr int LNB = B0 + 1024;        // beta' of the folded LayerNorm, 256 fp32
  static constexpr int GRP = LNB + 1024;       // the two groups' exchanges
  // per group
  static constexpr int XB = 0;                 // state: 2 k-steps x (hi plane 1 KiB, lo plane 1 KiB)
  static constexpr int ACT0 = XB + 4096;       // act0 hi: 8 k-steps x 1 KiB (P<BF16> layout)
  static constexpr int ACT1 = ACT0 + 8192;     // act1: 4 k-steps x (hi, lo)
  static constexpr int HIST = ACT1 + 8192;     // cost ring [RING][16 samples][HS] fp32
  static constexpr int ST = HIST + RING * 16 * CC::HS * 4;
  static constexpr int CP = ST + 4 * 16 * 4;
  static constexpr int GBYTES = (CP + 4 * 16 * 4 + 15) / 16 * 16;
  static constexpr int BYTES = GRP + 2 * GBYTES;
  static_assert(BYTES <= 160 * 1024, "LDS per CU");
};

// the fp16 form's operands (F16): v as one fp16 tile in the bf16 exchange layout, relu(v) as one fp16 tile in the bf16 exchange layout (P<BF16>::put_tile_relu's
// packed ReLU on v_cvt_pk_f16_f32 output), and the 16x16x32 fp16 MFMA on fragments carried in bf16x8 containers
__device__ __forceinline__ void put_tile_f16(char* buf, int mt, int lane, const f32x4& v) {
  typedef __attribute__((ext_vector_type(2))) _Float16 f16x2_;
  auto pk = [](float a, float b) { return __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{a, b}, f16x2_)); };
  *reinterpret_cast<uint2*>(buf + (mt >> 1) * 1024 + lane * 16 + (mt & 1) * 8) = make_uint2(pk(v[0], v[1]), pk(v[2], v[3]));
}
__device__ __forceinline__ void put_tile_relu_f16(char* buf, int mt, int lane, const f32x4& v) {
  typedef __attribute__((ext_vector_type(2))) _Float16 f16x2_;
  auto pk = [](float a, float b) {
    const f16x2_ p = __builtin_convertvector(f32x2{a, b}, f16x2_);
    return __builtin_bit_cast(unsigned, __builtin_elementwise_max(__builtin_bit_cast(i16x2, p), i16x2{0, 0}));
  };
  *reinterpret_cast<uint2*>(buf + (mt >> 1) * 1024 + lane * 16 + (mt & 1) * 8) = make_uint2(pk(v[0], v[1]), pk(v[2], v[3]));
}
__device__ __forceinline__ f32x4 mma16h(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  typedef __attribute__((ext_vector_type(8))) _Float16 f16x8_;
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8_, a), __builtin_bit_cast(f16x8_, b), c, 0, 0, 0);
}
// ... layer 1's: the fragment from an AGPR (asm, like P<BF16X3>::mma_a2; the accumulators then pass mma_fence)
__device__ __forceinline__ f32x4 mma16h_a(const bf16x8& a, const bf16x8& b, f32x4 c) {
  asm volatile(
      "s_nop 1\n\t"
      "v_mfma_f32_16x16x32_f16 %0, %1, %2, %0"
      : "+v"(c)
      : "a"(a), "v"(b));
  return c;
}

template <int COST, bool F16, bool L2X1 = false>  // L2X1: the fp16 form's last layer as one product (x3_f16_l2x1)
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2))) void fc_rollout_kernel_x3d(SolveArgs a,
                                                                                                      FcArgs net) {
  using Y = X3dLay<COST>;
  using PR = P<MPPI_PREC_BF16X3>;
  using PB = P<MPPI_PREC_BF16>;
  using CC = typename Y::CC;
  constexpr bool L0H = F16 && MPPI_X3_F16_L0;  // layer 0 on the fp16 state plane (fp16 W hi + lo)
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const KClock kc = kclock_begin(a);
  if (blockIdx.x == 0 && threadIdx.x == 0) *a.status = 0u;
  const int lane = threadIdx.x & 63, g = lane >> 4, n = lane & 15;
  const int wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wv = wib & 3, gi = wib >> 2;  // wave in group, group in block
  constexpr int N0 = 4, N1 = 2;           // own m-tiles of layers 0 (16) and 1 (8); the last layer: m-tile wv
  // ---- stage layers 0 / 2 as hi / lo planes, the layer-0 bias and beta'
  {
    const int4* s0 = reinterpret_cast<const int4*>(net.img + (L0H ? net.wmf16_0_off : net.w_off[0]));  // 32 B / lane
    const int4* s2 = reinterpret_cast<const int4*>(net.img + (F16 ? net.wmf16_x_off : net.w_off[2]));
    int4 t0[8], t2[4];  // every load before any store (one memory round trip, not one per unit)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      t0[2 * j] = s0[2 * (threadIdx.x + 512 * j)];
      t0[2 * j + 1] = s0[2 * (threadIdx.x + 512 * j) + 1];
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      t2[2 * j] = s2[2 * (threadIdx.x + 512 * j)];
      t2[2 * j + 1] = s2[2 * (threadIdx.x + 512 * j) + 1];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      *reinterpret_cast<int4*>(lds + Y::F0H + (threadIdx.x + 512 * j) * 16) = t0[2 * j];
      *reinterpret_cast<int4*>(lds + Y::F0L + (threadIdx.x + 512 * j) * 16) = t0[2 * j + 1];
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      *reinterpret_cast<int4*>(lds + Y::F2H + (threadIdx.x + 512 * j) * 16) = t2[2 * j];
      *reinterpret_cast<int4*>(lds + Y::F2L + (threadIdx.x + 512 * j) * 16) = t2[2 * j + 1];
    }
    if (threadIdx.x < 256) {
      reinterpret_cast<float*>(lds + Y::B0)[threadIdx.x] =
          reinterpret_cast<const float*>(net.img + net.b_off[0])[threadIdx.x];
      reinterpret_cast<float*>(lds + Y::LNB)[threadIdx.x] =
          reinterpret_cast<const float*>(net.img + net.lnb_off)[threadIdx.x];
    }
  }
  const int gps = a.Kp >> 4, total = a.B * gps;
  const int grp = blockIdx.x * 2 + gi;
  // a group past the end still runs the loop (the barriers are block-wide) on a clamped copy and writes nothing
  const bool live = grp < total;
  const int gc = live ? grp : total - 1;
  const int b = __builtin_amdgcn_readfirstlane(gc / gps);
  const int k = (gc - b * gps) * 16 + n;
  char* ex = lds + Y::GRP + gi * Y::GBYTES;

  // layer 1's fragments of this wave's rows in registers (AGPRs: read by the asm MFMAs), loaded once
  using Wt = std::conditional_t<F16, bf16x8, typename PR::Wt>;  // fp16 form: one 16 B fp16 fragment
  Wt w1r[N1][8];
  load_frags<F16 ? MPPI_PREC_BF16 : MPPI_PREC_BF16X3>(
      w1r, reinterpret_cast<const Wt*>(net.img + (F16 ? net.wmf16_off : net.w_off[1])), wv * N1, lane);
  auto ld4 = [&](const float* p, int row) { return *reinterpret_cast<const f32x4*>(p + row); };
  f32x4 bias1[N1], biasx;
#pragma unroll
  for (int i = 0; i < N1; ++i) bias1[i] = ld4(reinterpret_cast<const float*>(net.img + net.b_off[1]), 16 * (wv * N1 + i) + 4 * g);
  biasx = ld4(reinterpret_cast<const float*>(net.img + net.b_off[2]), 16 * wv + 4 * g);
  int ol = lane;  // opaque per step: LDS fragment / operand reads are not hoisted out of the horizon loop
  auto frag = [&](int plane, int f) { return *reinterpret_cast<const bf16x8*>(lds + plane + f * 1024 + ol * 16); };

  // own state tile (m-tile wv), initial value from x0 of solve b
  f32x4 x;
  const float* x0 = a.x0 + (long)b * a.nx;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int sl = 16 * wv + 4 * g + r;
    const int src = sl < 32 ? (sl < net.qp ? sl : -1) : (sl - 32 < net.qv ? net.qp + sl - 32 : -1);
    x[r] = src >= 0 ? x0[src] : 0.0f;
  }
  if constexpr (L0H)
    put_tile_f16(ex + Y::XB, wv, lane, x);
  else
    PR::put_tile(ex + Y::XB, wv, lane, x);
  float cx[MPPI_CTX_MAX];
#pragma unroll
  for (int i = 0; i < MPPI_CTX_MAX; ++i) cx[i] = a.ctx ? a.ctx[(long)b * MPPI_CTX_MAX + i] : a.ctx_default[i];

  // control part of the running cost: lane (wv, g) of sample n accounts for controls {4g + wv, 16 + 4g + wv}, loaded
  // PD steps ahead (fc_rollout.h)
  const auto rU = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.U) + (long)b * a.nu * a.H, 0,
                                                    a.nu * a.H * 4, 0x00020000);
  const auto rE = __builtin_amdgcn_make_buffer_rsrc(a.noise + (long)b * a.nu * a.H * a.Kp, 0,
                                                    a.nu * a.H * a.Kp * 4, 0x00020000);
  const float cl = a.ctrl_clamp > 0.0f ? a.ctrl_clamp : INFINITY;
  constexpr int PD = X3D_PD;
  int cuoff[2], ceoff[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int us = 16 * i + 4 * g + wv;
    cuoff[i] = us < a.nu ? us * a.H * 4 : 0x7FFFFFF0;
    ceoff[i] = us < a.nu ? (us * a.H * a.Kp + k) * 4 : 0x7FFFFFF0;
  }
  auto load_cu = [&](int t, float (&cu)[2], float (&ce)[2]) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      cu[i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rU, cuoff[i], t * 4, 0));
      ce[i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rE, ceoff[i], t * a.Kp * 4, 0));
    }
  };
  float cuu[PD][2], cue[PD][2];
#pragma unroll
  for (int j = 0; j < PD; ++j) {
    asm volatile("" ::: "memory");  // issue order step 0, 1, ..., PD - 1 (the loop's wait counts assume it)
    load_cu(j < a.H ? j : a.H - 1, cuu[j], cue[j]);
  }
  float cost = 0.0f;
  constexpr CostIdx ci = cost_idx(COST);
  float* hist = reinterpret_cast<float*>(ex + Y::HIST);
  int my_chunk = -1;  // this lane's ring chunk (tile wv, lane group g), -1: the cost reads none of its slots
#pragma unroll
  for (int e = 0; e < 16; ++e)
    if (e == 4 * wv + g) my_chunk = CC::chunk(e / 4, e % 4);
  const int ls = 4 * wv + g;
  auto ring_cost = [&](int r, int t1) {
    f32x4 ch[CC::NCH];
#pragma unroll
    for (int c = 0; c < CC::NCH; ++c) ch[c] = *reinterpret_cast<const f32x4*>(hist + (r * 16 + n) * CC::HS + 4 * c);
    float v[kCostMaxIdx];
#pragma unroll
    for (int i = 0; i < ci.n; ++i) {
      const int sl = CC::slot(ci.idx[i]);
      v[i] = ch[CC::chunk(sl / 16, (sl % 16) / 4)][sl % 4];
    }
    return cost_eval_t<COST>(v, 0.0f, 0.0f, cx, t1);
  };
  __syncthreads();  // the LDS image and the initial state exchanges visible
  // group 1 runs X3D_OFFSET barrier intervals behind group 0 (group 0 passes the same number after its last step)
  if (gi == 1)
    for (int i = 0; i < X3D_OFFSET; ++i) __syncthreads();

  auto step = [&](const int t, auto PAR) __attribute__((always_inline)) {
    constexpr int PP = decltype(PAR)::value;
    asm volatile("" : "+v"(ol));
    {
      const float c0 = __builtin_amdgcn_fmed3f(cuu[PP][0] + cue[PP][0], -cl, cl);
      const float c1 = __builtin_amdgcn_fmed3f(cuu[PP][1] + cue[PP][1], -cl, cl);
      float cc0 = c0, cc1 = c1;
      asm volatile("" : "+v"(cc0), "+v"(cc1)::"memory");
      load_cu(t + PD < a.H ? t + PD : a.H - 1, cuu[PP], cue[PP]);
      cost += ctrl_term_t<COST>((g == 0 && wv == 0) ? cc0 : 0.0f, fmaf(cc0, cc0, cc1 * cc1));
    }
    // ---- layer 0 (dense, centred: the LayerNorm fold), fragments from the LDS planes -> statistic -> act0 (hi)
    f32x4 h[N0];
    {
      const float* b0 = reinterpret_cast<const float*>(lds + Y::B0);
#pragma unroll
      for (int i = 0; i < N0; ++i) h[i] = *reinterpret_cast<const f32x4*>(b0 + 16 * (wv * N0 + i) + 4 * g);
      if constexpr (L0H) {
        bf16x8 bin[2];
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) bin[ks] = PB::get_ks(ex + Y::XB, ks, ol);
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
          for (int i = 0; i < N0; ++i) {
            const int f = (wv * N0 + i) * 2 + kk;
            h[i] = mma16h(frag(Y::F0H, f), bin[kk], mma16h(frag(Y::F0L, f), bin[kk], h[i]));
          }
      } else {
        typename PR::Bop bin[2];
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) bin[ks] = PR::get_ks(ex + Y::XB, ks, ol);
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
          for (int i = 0; i < N0; ++i) {
            const int f = (wv * N0 + i) * 2 + kk;
            h[i] = PR::mma(BX3{frag(Y::F0H, f), frag(Y::F0L, f)}, bin[kk], h[i]);
          }
      }
      f32x2 q2[N0];
#pragma unroll
      for (int i = 0; i < N0; ++i) {
        const f32x2 lo = {h[i][0], h[i][1]}, hi = {h[i][2], h[i][3]};
        q2[i] = hi * hi + lo * lo;
      }
      q2[0] = (q2[0] + q2[1]) + (q2[2] + q2[3]);
      reinterpret_cast<float*>(ex + Y::ST)[wv * 16 + n] = group_sum(q2[0].x + q2[0].y);
    }
    __syncthreads();
    {
      const float* st = reinterpret_cast<const float*>(ex + Y::ST);
      float q = st[n];
#pragma unroll
      for (int w2 = 1; w2 < 4; ++w2) q += st[w2 * 16 + n];  // fixed order
      const float rstd = __builtin_amdgcn_rsqf(q * (1.0f / 256.0f) + 1e-5f);
      const f32x2 r2 = {rstd, rstd};
      const float* lb = reinterpret_cast<const float*>(lds + Y::LNB);
#pragma unroll
      for (int i = 0; i < N0; ++i) {
        const f32x4 be = *reinterpret_cast<const f32x4*>(lb + 16 * (wv * N0 + i) + 4 * g);
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          const f32x2 y = f32x2{h[i][2 * hh], h[i][2 * hh + 1]} * r2 + f32x2{be[2 * hh], be[2 * hh + 1]};
          h[i][2 * hh] = y.x;
          h[i][2 * hh + 1] = y.y;
        }
        if constexpr (F16)
          put_tile_relu_f16(ex + Y::ACT0, wv * N0 + i, lane, h[i]);
        else
          PB::put_tile_relu(ex + Y::ACT0, wv * N0 + i, lane, h[i]);  // the hi plane only
      }
    }
    __syncthreads();
    // ---- layer 1: two products (W1_lo a_hi + W1_hi a_hi) from the register-resident fragments -> act1 (hi / lo)
    {
      bf16x8 bin[8];
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) bin[ks] = PB::get_ks(ex + Y::ACT0, ks, ol);
      f32x4 h1[N1];
#pragma unroll
      for (int i = 0; i < N1; ++i) h1[i] = bias1[i];
      __builtin_amdgcn_sched_barrier(0);  // every B read before the first MFMA (each MFMA waits for its own read only)
#pragma unroll
      for (int kk = 0; kk < 8; ++kk)
#pragma unroll
        for (int i = 0; i < N1; ++i) {
          if constexpr (F16)
            h1[i] = mma16h_a(w1r[i][kk], bin[kk], h1[i]);
          else
            h1[i] = PR::mma_a2(w1r[i][kk], bin[kk], h1[i]);
        }
      mma_fence(h1);
#pragma unroll
      for (int i = 0; i < N1; ++i) {
        if constexpr (F16)
          put_tile_relu_f16(ex + Y::ACT1, wv * N1 + i, lane, h1[i]);  // one fp16 plane
        else
          PR::put_tile_relu(ex + Y::ACT1, wv * N1 + i, lane, h1[i]);
      }
    }
    __syncthreads();
    // ---- last layer (m-tile wv), fragments from the LDS planes, two accumulation chains; x += dx -> xb, cost ring
    {
      f32x4 d0 = biasx, d1 = {0.0f, 0.0f, 0.0f, 0.0f};
      if constexpr (F16) {  // fp16 W hi + lo against the fp16 plane
        bf16x8 bin[4];
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) bin[ks] = PB::get_ks(ex + Y::ACT1, ks, ol);
#pragma unroll
        for (int kk = 0; kk < 4; kk += 2) {
          const int f = wv * 4 + kk;
          if constexpr (L2X1) {
            d0 = mma16h(frag(Y::F2H, f), bin[kk], d0);
            d1 = mma16h(frag(Y::F2H, f + 1), bin[kk + 1], d1);
          } else {
            d0 = mma16h(frag(Y::F2H, f), bin[kk], mma16h(frag(Y::F2L, f), bin[kk], d0));
            d1 = mma16h(frag(Y::F2H, f + 1), bin[kk + 1], mma16h(frag(Y::F2L, f + 1), bin[kk + 1], d1));
          }
        }
      } else {
        typename PR::Bop bin[4];
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) bin[ks] = PR::get_ks(ex + Y::ACT1, ks, ol);
#pragma unroll
        for (int kk = 0; kk < 4; kk += 2) {
          const int f = wv * 4 + kk;
          d0 = PR::mma(BX3{frag(Y::F2H, f), frag(Y::F2L, f)}, bin[kk], d0);
          d1 = PR::mma(BX3{frag(Y::F2H, f + 1), frag(Y::F2L, f + 1)}, bin[kk + 1], d1);
        }
      }
      x += d0 + d1;
      if constexpr (L0H)
        put_tile_f16(ex + Y::XB, wv, lane, x);
      else
        PR::put_tile(ex + Y::XB, wv, lane, x);
      if (my_chunk >= 0)
        *reinterpret_cast<f32x4*>(hist + ((t % Y::RING) * 16 + n) * CC::HS + 4 * my_chunk) = x;
    }
    __syncthreads();
    if ((t + 1) % Y::RING == 0 || t + 1 == a.H) {  // ring full (or horizon done): one (step, sample) per lane group
      const int ts = t - t % Y::RING + ls;
      if (ls < Y::RING && ts <= t) cost += ring_cost(ls, ts + 1);
    }
  };
  int t0 = 0;
  for (; t0 + PD <= a.H; t0 += PD) {
    step(t0, std::integral_constant<int, 0>{});
    if constexpr (PD > 1) step(t0 + 1, std::integral_constant<int, 1 % PD>{});
    if constexpr (PD > 2) step(t0 + 2, std::integral_constant<int, 2 % PD>{});
  }
  if constexpr (PD > 1) if (t0 < a.H) step(t0, std::integral_constant<int, 0>{});
  if constexpr (PD > 2) if (t0 + 1 < a.H) step(t0 + 1, std::integral_constant<int, 1 % PD>{});
  if (gi == 0)
    for (int i = 0; i < X3D_OFFSET; ++i) __syncthreads();
  if (a.terminal_weight != 0.0f && ls == 0) cost += a.terminal_weight * ring_cost((a.H - 1) % Y::RING, a.H);
  cost = group_sum(cost);
  float* cp = reinterpret_cast<float*>(ex + Y::CP);
  if (g == 0) cp[wv * 16 + n] = cost;
  __syncthreads();
  kclock_record(a, kc);
  if (wv == 0 && g == 0 && live && k < a.K) {
    float c = cp[n];
#pragma unroll
    for (int w2 = 1; w2 < 4; ++w2) c += cp[w2 * 16 + n];
    a.costs[(long)b * a.Kp + k] = isfinite(c) ? c : INFINITY;
  }
  if (a.xout && live && k == 0) {  // env step: final state of sample 0 (lane n = 0 of the solve's first group)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int sl = 16 * wv + 4 * g + r;
      const int src = sl < 32 ? (sl < net.qp ? sl : -1) : (sl - 32 < net.qv ? net.qp + sl - 32 : -1);
      if (src >= 0) a.xout[(long)b * a.nx + src] = x[r];
    }
  }
}

// MPPI_X3D (read per launch): unset = this kernel for the split CA with the two-product layer 1 below the per-wave
// kernels' batch threshold; 0 = never (fc_rollout_kernel_x3w); 1 = always where it applies
bool fc_x3d_wanted(const SolveArgs& a, const FcArgs& fa) {
  if (fa.w_off[1] < 0 || fa.ln_n != 256 || a.Kp % 64 != 0) return false;
  if (x3_l1_terms(a.H, fa.x3_l1) != 2 && !x3_f16_on(a.H, fa.x3_f16, fa.wmf16_off)) return false;
  const char* e = std::getenv("MPPI_X3D");
  return !(e && e[0] == '0');
}

hipError_t launch_fc_x3d(const SolveArgs& a, const FcArgs& fa, hipStream_t stream) {
  const int groups = a.B * (a.Kp >> 4);
  if (a.Kp % 64 != 0 || groups < 1) return hipErrorInvalidValue;
  const int grid = (groups + 1) / 2;
  auto go = [&](auto kern, int bytes) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(512), bytes, stream, a, fa);
    return hipGetLastError();
  };
  const int form = x3_form(a.H, fa.x3_l1, fa.x3_f16, fa.wmf16_off);
  if (form == 3) return hipErrorInvalidValue;
  static const char* const names[3] = {
      MPPI_X3_F16_L0 ? "fc_rollout_kernel_x3d<f16,l2=1>" : "fc_rollout_kernel_x3d<l1=f16,l2=1>",
      MPPI_X3_F16_L0 ? "fc_rollout_kernel_x3d<f16>" : "fc_rollout_kernel_x3d<l1=f16>", "fc_rollout_kernel_x3d<l1=2>"};
  note_kernel(names[form]);
  auto by_form = [&](auto cost) {
    constexpr int C = decltype(cost)::value;
    switch (form) {
      case 0: return go(fc_rollout_kernel_x3d<C, true, true>, X3dLay<C>::BYTES);
      case 1: return go(fc_rollout_kernel_x3d<C, true>, X3dLay<C>::BYTES);
      default: return go(fc_rollout_kernel_x3d<C, false>, X3dLay<C>::BYTES);
    }
  };
  if (a.cost_kind == MPPI_COST_HUMANOID_V1) return by_form(std::integral_constant<int, MPPI_COST_HUMANOID_V1>{});
  return by_form(std::integral_constant<int, MPPI_COST_HUMANOID_V3>{});
}

}  // namespace mppi
