// fc_rollout_kernel_x3h (round 6, late): the fp16 form of the split (MPPI_PREC_BF16X3, fp32-accurate) M-split CA
// rollout with ONE group per block and TWO blocks per CU -- the few-tiles shards (8 / 16 solves of config #4 at N = 8 /
// N = 4).
//
// fc_rollout_kernel_x3d puts two 16-sample groups in one 512-thread block because the bf16x3 form's hi / lo weight
// images do not fit twice in the CU: the groups share one LDS copy of layers 0 and 2 (hi and lo planes, 96 KiB) and
// the block's barriers, so they step in lockstep and both read every fragment from LDS every step (24 KiB per
// wave-step).  In the fp16 form the HI weights of every layer take exactly the registers the bf16 M-split kernel
// (fc_rollout_kernel<CA, BF16>, fc_rollout.h) holds its bf16 weights in -- layer 0 32, layer 1 64 (AGPRs), last layer
// 16 -- so this kernel is that kernel's organisation in the fp16 form:
//   * a 256-thread block = one group (4 waves, one per SIMD, one 16-sample tile per wave), two blocks per CU with their
//     own barriers: the two groups drift, so one's barrier and LDS waits overlap the other's issue (odd blocks at
//     s_setprio 1, as in the bf16 kernel);
//   * the HI fragments of layers 0 and 2 and layer 1's fp16 fragments in registers for the whole horizon;
//   * only the LO planes of layers 0 and 2 (48 KiB) in LDS, per block, read by their own wave every step (12 fragments
//     per wave-step instead of 24);
//   * the layer-0 bias and beta' in LDS (registers are the limit at two waves per SIMD), an 8-step cost ring.
// The arithmetic is x3d's fp16 form term for term and in the same order (layer 0: lo then hi per k-step; the last
// layer: two chains, lo then hi), so the costs equal fc_rollout_kernel_x3d<f16>'s bitwise
// (tests/test_gpu_fullsize.py test_split_x3d_kernel_matches_x3w_and_oracle).  Its own translation unit (build.py PER_FILE_FLAGS).
#include "fc_rollout.h"

namespace mppi {

#ifndef X3H_PD  // control loads this many steps ahead (the step loop unrolled by it, <= 3)
#define X3H_PD 2
#endif
#ifndef X3H_ASM  // layers 0 and 2 as asm MFMAs reading the hi fragments from AGPRs (0: the builtin, and hipcc copies
                 // the AGPR-resident fragments to VGPRs before their MFMAs)
#define X3H_ASM 1
#endif
// timing-only diagnostic builds (results wrong): X3H_DIAG = 1 drops the lo products of layers 0 and 2 (no LDS read, no
// MFMA), 2 keeps their MFMAs on the hi fragment instead of the LDS lo plane (no LDS read)
#ifndef X3H_DIAG
#define X3H_DIAG 0
#endif
#ifndef X3H_B0MMA  // layer 0's bias through the MFMA chain (FcNet::wmf16_0b_off: b0 in the pad column kCaX3hBiasSlot
                   // against a state slot of 1.0) instead of an accumulator initialised from LDS
#define X3H_B0MMA 1
#endif
#ifndef X3H_BEPRE  // beta' read from LDS before the statistic barrier (its latency under the barrier wait)
#define X3H_BEPRE 1
#endif
#ifndef X3H_BEREG  // beta' of the own rows in registers for the horizon (16 VGPRs; needs the room X3H_B0MMA frees)
#define X3H_BEREG 1
#endif
#ifndef X3H_L0LO_QV  // layer 0's lo on the qvel k-step (state slots 32..63) too (1), or hi only there (0: 4 MFMAs and 4
                     // fragment reads fewer per wave-step; the CPU error budget puts the qvel columns' lo at nothing
                     // measurable on model_cross, profiles/r06_x3_error_budget_f16.txt "f16x2wq", and the engine's probe
                     // runs this kernel's form on the loaded net: mppi_api.hip x3_probe)
#define X3H_L0LO_QV 0
#endif
#ifndef X3H_L2LOREG  // the last layer's lo fragments in registers (AGPRs) instead of LDS reads every step (NS = 1)
#define X3H_L2LOREG 1
#endif
#ifndef X3H_PRIO  // odd blocks at s_setprio 1 (the bf16 M-split kernel's tie-break between the CU's two blocks)
#define X3H_PRIO 1
#endif

template <int COST, int NS>
struct X3hLay {
  using CC = CostChunks<kArchCA, COST>;
  static constexpr int RING = 8;                // cost-ring steps (lane groups ls = 4 wv + g < RING: one (step, sample))
  // shared by the block's NS tiles
  static constexpr int F0L = 0;                 // layer-0 lo plane: 32 fragments (mt 0..15, kk 0..1 at mt * 2 + kk)
  static constexpr int F2L = F0L + 32 * 1024;   // last-layer lo plane: 16 fragments (mt 0..3, kk 0..3 at mt * 4 + kk)
  static constexpr int B0 = F2L + 16 * 1024;    // layer-0 bias, 256 fp32
  static constexpr int LNB = B0 + 1024;         // beta' of the folded LayerNorm, 256 fp32
  static constexpr int TILES = LNB + 1024;      // the tiles' exchanges
  // per tile
  static constexpr int XB = 0;                  // state: one fp16 plane, 2 k-steps x 1 KiB
  static constexpr int ACT0 = XB + 2048;        // act0: one fp16 plane, 8 k-steps x 1 KiB
  static constexpr int ACT1 = ACT0 + 8192;      // act1: one fp16 plane, 4 k-steps x 1 KiB
  static constexpr int HIST = ACT1 + 4096;      // cost ring [RING][16 samples][HS] fp32
  static constexpr int ST = HIST + RING * 16 * CC::HS * 4;
  static constexpr int CP = ST + 4 * 16 * 4;
  static constexpr int TBYTES = (CP + 4 * 16 * 4 + 15) / 16 * 16;
  static constexpr int BYTES = TILES + NS * TBYTES;
  static_assert((NS == 1 ? 2 : 1) * BYTES <= 160 * 1024, "NS = 1: two blocks per CU; else one");
};

namespace {
typedef __attribute__((ext_vector_type(2))) _Float16 f16x2_;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8_;
// v as one fp16 tile in the bf16 exchange layout; relu(v) the same with the packed ReLU on v_cvt_pk_f16_f32's output
__device__ __forceinline__ void put_f16(char* buf, int mt, int lane, const f32x4& v) {
  auto pk = [](float a, float b) { return __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{a, b}, f16x2_)); };
  *reinterpret_cast<uint2*>(buf + (mt >> 1) * 1024 + lane * 16 + (mt & 1) * 8) = make_uint2(pk(v[0], v[1]), pk(v[2], v[3]));
}
__device__ __forceinline__ void put_relu_f16(char* buf, int mt, int lane, const f32x4& v) {
  auto pk = [](float a, float b) {
    const f16x2_ p = __builtin_convertvector(f32x2{a, b}, f16x2_);
    return __builtin_bit_cast(unsigned, __builtin_elementwise_max(__builtin_bit_cast(i16x2, p), i16x2{0, 0}));
  };
  *reinterpret_cast<uint2*>(buf + (mt >> 1) * 1024 + lane * 16 + (mt & 1) * 8) = make_uint2(pk(v[0], v[1]), pk(v[2], v[3]));
}
// the 16x16x32 fp16 MFMA on fragments carried in bf16x8 containers (the images' fp16 bits)
__device__ __forceinline__ f32x4 mmh(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8_, a), __builtin_bit_cast(f16x8_, b), c, 0, 0, 0);
}
// ... layer 1's: the fragment read from an AGPR (asm; the accumulators then pass mma_fence, tests/test_hazard_check.py)
__device__ __forceinline__ f32x4 mmh_a(const bf16x8& a, const bf16x8& b, f32x4 c) {
  asm volatile(
      "s_nop 1\n\t"
      "v_mfma_f32_16x16x32_f16 %0, %1, %2, %0"
      : "+v"(c)
      : "a"(a), "v"(b));
  return c;
}
// ... layers 0 and 2: W_lo b + W_hi b into one accumulator, lo from a VGPR (LDS), hi from an AGPR (same padding rules)
__device__ __forceinline__ f32x4 mmh2_a(const bf16x8& lo, const bf16x8& hi, const bf16x8& b, f32x4 c) {
  asm volatile(
      "s_nop 1\n\t"
      "v_mfma_f32_16x16x32_f16 %0, %1, %3, %0\n\t"
      "v_mfma_f32_16x16x32_f16 %0, %2, %3, %0"
      : "+v"(c)
      : "v"(lo), "a"(hi), "v"(b));
  return c;
}
// ... both fragments from AGPRs (the last layer with X3H_L2LOREG)
__device__ __forceinline__ f32x4 mmh2_aa(const bf16x8& lo, const bf16x8& hi, const bf16x8& b, f32x4 c) {
  asm volatile(
      "s_nop 1\n\t"
      "v_mfma_f32_16x16x32_f16 %0, %1, %3, %0\n\t"
      "v_mfma_f32_16x16x32_f16 %0, %2, %3, %0"
      : "+v"(c)
      : "a"(lo), "a"(hi), "v"(b));
  return c;
}
// ... the first k-step of a chain that starts from zero (the bias through the MFMA: X3H_B0MMA)
__device__ __forceinline__ f32x4 mmh2_a0(const bf16x8& lo, const bf16x8& hi, const bf16x8& b) {
  f32x4 c;
  asm volatile(
      "s_nop 1\n\t"
      "v_mfma_f32_16x16x32_f16 %0, %1, %3, 0\n\t"
      "v_mfma_f32_16x16x32_f16 %0, %2, %3, %0"
      : "=&v"(c)
      : "v"(lo), "a"(hi), "v"(b));
  return c;
}
}  // namespace

// The body; NS = sample tiles per wave (16 samples each, consecutive groups of one solve).  NS = 1: one group per block,
// two blocks per CU (256 registers per wave); NS > 1: one block per CU at one wave per SIMD (512 registers), every
// fragment feeding NS independent MFMA chains, the lo fragments read once per wave-step for all NS tiles.
template <int COST, bool L2X1, int NS>  // L2X1: the last layer as one fp16 product (the opt-in x3_f16_l2x1)
__device__ __forceinline__ void fc_x3h_body(const SolveArgs& a, const FcArgs& net, char* lds) {
  using Y = X3hLay<COST, NS>;
  using PB = P<MPPI_PREC_BF16>;
  using CC = typename Y::CC;
  const KClock kc = kclock_begin(a);
  if (blockIdx.x == 0 && threadIdx.x == 0) *a.status = 0u;
  if (NS == 1 && X3H_PRIO && (blockIdx.x & 1)) __builtin_amdgcn_s_setprio(1);
  const int lane = threadIdx.x & 63, g = lane >> 4, n = lane & 15;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  constexpr int N0 = 4, N1 = 2;  // own m-tiles of layers 0 (16) and 1 (8); the last layer: m-tile wv
  constexpr bool B0M = X3H_B0MMA && X3H_ASM && X3H_DIAG == 0;
  // [fragment][lane] x (hi, lo) 16 B each
  const int4* s0 = reinterpret_cast<const int4*>(net.img + (B0M ? net.wmf16_0b_off : net.wmf16_0_off));
  const int4* s2 = reinterpret_cast<const int4*>(net.img + net.wmf16_x_off);
  // ---- the lo planes of layers 0 / 2, the layer-0 bias and beta' into LDS (every load before any store)
  {
    int4 t0[8], t2[4];
#pragma unroll
    for (int j = 0; j < 8; ++j) t0[j] = s0[2 * (threadIdx.x + 256 * j) + 1];
#pragma unroll
    for (int j = 0; j < 4; ++j) t2[j] = s2[2 * (threadIdx.x + 256 * j) + 1];
    const float b0v = reinterpret_cast<const float*>(net.img + net.b_off[0])[threadIdx.x];
    const float lbv = reinterpret_cast<const float*>(net.img + net.lnb_off)[threadIdx.x];
#pragma unroll
    for (int j = 0; j < 8; ++j) *reinterpret_cast<int4*>(lds + Y::F0L + (threadIdx.x + 256 * j) * 16) = t0[j];
#pragma unroll
    for (int j = 0; j < 4; ++j) *reinterpret_cast<int4*>(lds + Y::F2L + (threadIdx.x + 256 * j) * 16) = t2[j];
    reinterpret_cast<float*>(lds + Y::B0)[threadIdx.x] = b0v;
    reinterpret_cast<float*>(lds + Y::LNB)[threadIdx.x] = lbv;
  }
  // ---- this wave's hi fragments: layer 0 (4 m-tiles x 2 k-steps), the last layer (m-tile wv, 4 k-steps), and layer
  // 1's fp16 fragments (AGPRs: read by the asm MFMAs), all loaded once
  bf16x8 w0h[N0][2], w2h[4], w1r[N1][8];
#pragma unroll
  for (int i = 0; i < N0; ++i)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
      w0h[i][kk] = __builtin_bit_cast(bf16x8, s0[2 * (((wv * N0 + i) * 2 + kk) * 64 + lane)]);
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) w2h[kk] = __builtin_bit_cast(bf16x8, s2[2 * ((wv * 4 + kk) * 64 + lane)]);
  constexpr bool L2R = X3H_L2LOREG && NS == 1 && X3H_ASM && X3H_DIAG == 0;
  bf16x8 w2l[L2R ? 4 : 1];
  if constexpr (L2R) {
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) w2l[kk] = __builtin_bit_cast(bf16x8, s2[2 * ((wv * 4 + kk) * 64 + lane) + 1]);
  }
  load_frags<MPPI_PREC_BF16>(w1r, reinterpret_cast<const bf16x8*>(net.img + net.wmf16_off), wv * N1, lane);
  auto ld4 = [&](const float* p, int row) { return *reinterpret_cast<const f32x4*>(p + row); };
  f32x4 bias1[N1], biasx;
#pragma unroll
  for (int i = 0; i < N1; ++i) bias1[i] = ld4(reinterpret_cast<const float*>(net.img + net.b_off[1]), 16 * (wv * N1 + i) + 4 * g);
  biasx = ld4(reinterpret_cast<const float*>(net.img + net.b_off[2]), 16 * wv + 4 * g);
  f32x4 bereg[X3H_BEREG ? N0 : 1];
  if constexpr (X3H_BEREG) {
#pragma unroll
    for (int i = 0; i < N0; ++i) bereg[i] = ld4(reinterpret_cast<const float*>(net.img + net.lnb_off), 16 * (wv * N0 + i) + 4 * g);
  }
  int ol = lane;  // opaque per step: LDS fragment / operand reads are not hoisted out of the horizon loop
  auto frag = [&](int plane, int f) { return *reinterpret_cast<const bf16x8*>(lds + plane + f * 1024 + ol * 16); };

  // tiles s = 0..NS-1: groups NS * blockIdx.x + s, all of solve b (launch: (Kp / 16) % NS == 0)
  const int gps = a.Kp >> 4;
  const int grp = blockIdx.x * NS;
  const int b = __builtin_amdgcn_readfirstlane(grp / gps);
  const int k = (grp - b * gps) * 16 + n;  // sample of tile 0; tile s: k + 16 s
  char* ex[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) ex[s] = lds + Y::TILES + s * Y::TBYTES;

  // own state tile (m-tile wv), initial value from x0 of solve b
  f32x4 x[NS];
  const float* x0 = a.x0 + (long)b * a.nx;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int sl = 16 * wv + 4 * g + r;
    const int src = sl < 32 ? (sl < net.qp ? sl : -1) : (sl - 32 < net.qv ? net.qp + sl - 32 : -1);
    x[0][r] = src >= 0 ? x0[src] : (B0M && sl == kCaX3hBiasSlot ? 1.0f : 0.0f);  // (the pad rows' dx is 0)
  }
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    x[s] = x[0];
    put_f16(ex[s] + Y::XB, wv, lane, x[s]);
  }
  float cx[MPPI_CTX_MAX];
#pragma unroll
  for (int i = 0; i < MPPI_CTX_MAX; ++i) cx[i] = a.ctx ? a.ctx[(long)b * MPPI_CTX_MAX + i] : a.ctx_default[i];

  // control part of the running cost: lane (wv, g) of sample n accounts for controls {4g + wv, 16 + 4g + wv}, loaded
  // PD steps ahead (fc_rollout.h); U once for the NS tiles (one solve), eps per tile (+ 64 B per tile)
  const auto rU = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.U) + (long)b * a.nu * a.H, 0,
                                                    a.nu * a.H * 4, 0x00020000);
  const auto rE = __builtin_amdgcn_make_buffer_rsrc(a.noise + (long)b * a.nu * a.H * a.Kp, 0,
                                                    a.nu * a.H * a.Kp * 4, 0x00020000);
  const float cl = a.ctrl_clamp > 0.0f ? a.ctrl_clamp : INFINITY;
  constexpr int PD = X3H_PD;
  int cuoff[2], ceoff[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int us = 16 * i + 4 * g + wv;
    cuoff[i] = us < a.nu ? us * a.H * 4 : 0x7FFFFFF0;
    ceoff[i] = us < a.nu ? (us * a.H * a.Kp + k) * 4 : 0x7FFFFFF0;
  }
  auto load_cu = [&](int t, float (&cu)[2], float (&ce)[NS][2]) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      cu[i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rU, cuoff[i], t * 4, 0));
#pragma unroll
      for (int s = 0; s < NS; ++s)
        ce[s][i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rE, ceoff[i], t * a.Kp * 4 + 64 * s, 0));
    }
  };
  float cuu[PD][2], cue[PD][NS][2];
#pragma unroll
  for (int j = 0; j < PD; ++j) {
    asm volatile("" ::: "memory");  // issue order step 0, 1, ..., PD - 1 (the loop's wait counts assume it)
    load_cu(j < a.H ? j : a.H - 1, cuu[j], cue[j]);
  }
  float cost[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) cost[s] = 0.0f;
  constexpr CostIdx ci = cost_idx(COST);
  int my_chunk = -1;  // this lane's ring chunk (tile wv, lane group g), -1: the cost reads none of its slots
#pragma unroll
  for (int e = 0; e < 16; ++e)
    if (e == 4 * wv + g) my_chunk = CC::chunk(e / 4, e % 4);
  const int ls = 4 * wv + g;
  auto ring_cost = [&](int s, int r, int t1) {
    const float* hist = reinterpret_cast<const float*>(ex[s] + Y::HIST);
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
  __syncthreads();  // the lo planes, biases and the initial state exchanges visible

  auto step = [&](const int t, auto PAR) __attribute__((always_inline)) {
    constexpr int PP = decltype(PAR)::value;
    asm volatile("" : "+v"(ol));
    {
      float cc[NS][2];
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        cc[s][0] = __builtin_amdgcn_fmed3f(cuu[PP][0] + cue[PP][s][0], -cl, cl);
        cc[s][1] = __builtin_amdgcn_fmed3f(cuu[PP][1] + cue[PP][s][1], -cl, cl);
        asm volatile("" : "+v"(cc[s][0]), "+v"(cc[s][1])::"memory");
      }
      load_cu(t + PD < a.H ? t + PD : a.H - 1, cuu[PP], cue[PP]);
#pragma unroll
      for (int s = 0; s < NS; ++s)
        cost[s] += ctrl_term_t<COST>((g == 0 && wv == 0) ? cc[s][0] : 0.0f, fmaf(cc[s][0], cc[s][0], cc[s][1] * cc[s][1]));
    }
    // ---- layer 0 (dense, centred: the LayerNorm fold), fp16 W hi (registers) + lo (LDS) against the fp16 state
    f32x4 h[NS][N0];
    {
      if constexpr (!B0M) {
        const float* b0 = reinterpret_cast<const float*>(lds + Y::B0);
#pragma unroll
        for (int i = 0; i < N0; ++i) h[0][i] = *reinterpret_cast<const f32x4*>(b0 + 16 * (wv * N0 + i) + 4 * g);
#pragma unroll
        for (int s = 1; s < NS; ++s)
#pragma unroll
          for (int i = 0; i < N0; ++i) h[s][i] = h[0][i];
      }
      bf16x8 bin[NS][2];
#pragma unroll
      for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) bin[s][ks] = PB::get_ks(ex[s] + Y::XB, ks, ol);
      if constexpr (X3H_ASM) {
        bf16x8 lo[2][N0];
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
          for (int i = 0; i < N0; ++i)
            lo[kk][i] = (X3H_DIAG || (kk == 1 && !X3H_L0LO_QV)) ? bin[0][kk] : frag(Y::F0L, (wv * N0 + i) * 2 + kk);
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
          for (int s = 0; s < NS; ++s)
#pragma unroll
            for (int i = 0; i < N0; ++i) {
              if (B0M && kk == 0)
                h[s][i] = mmh2_a0(lo[kk][i], w0h[i][kk], bin[s][kk]);
              else if (kk == 1 && !X3H_L0LO_QV)
                h[s][i] = mmh_a(w0h[i][kk], bin[s][kk], h[s][i]);  // the qvel k-step: hi only
              else
                h[s][i] = X3H_DIAG == 1 ? mmh_a(w0h[i][kk], bin[s][kk], h[s][i])
                                        : mmh2_a(lo[kk][i], w0h[i][kk], bin[s][kk], h[s][i]);
            }
        mma_fence(h);
      } else {
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
          for (int s = 0; s < NS; ++s)
#pragma unroll
            for (int i = 0; i < N0; ++i)
              h[s][i] = mmh(w0h[i][kk], bin[s][kk], mmh(frag(Y::F0L, (wv * N0 + i) * 2 + kk), bin[s][kk], h[s][i]));
      }
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        f32x2 q2[N0];
#pragma unroll
        for (int i = 0; i < N0; ++i) {
          const f32x2 lo = {h[s][i][0], h[s][i][1]}, hi = {h[s][i][2], h[s][i][3]};
          q2[i] = hi * hi + lo * lo;
        }
        q2[0] = (q2[0] + q2[1]) + (q2[2] + q2[3]);
        reinterpret_cast<float*>(ex[s] + Y::ST)[wv * 16 + n] = group_sum(q2[0].x + q2[0].y);
      }
    }
    f32x4 be[N0];  // beta' of the own rows
    if constexpr (X3H_BEREG) {
#pragma unroll
      for (int i = 0; i < N0; ++i) be[i] = bereg[i];
    }
    auto load_be = [&] {
      if constexpr (X3H_BEREG) return;
      const float* lb = reinterpret_cast<const float*>(lds + Y::LNB);
#pragma unroll
      for (int i = 0; i < N0; ++i) be[i] = *reinterpret_cast<const f32x4*>(lb + 16 * (wv * N0 + i) + 4 * g);
    };
    if constexpr (X3H_BEPRE) load_be();
    __syncthreads();
    {
      if constexpr (!X3H_BEPRE) load_be();
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        const float* st = reinterpret_cast<const float*>(ex[s] + Y::ST);
        float q = st[n];
#pragma unroll
        for (int w2 = 1; w2 < 4; ++w2) q += st[w2 * 16 + n];  // fixed order
        const float rstd = __builtin_amdgcn_rsqf(q * (1.0f / 256.0f) + 1e-5f);
        const f32x2 r2 = {rstd, rstd};
#pragma unroll
        for (int i = 0; i < N0; ++i) {
#pragma unroll
          for (int hh = 0; hh < 2; ++hh) {
            const f32x2 y = f32x2{h[s][i][2 * hh], h[s][i][2 * hh + 1]} * r2 + f32x2{be[i][2 * hh], be[i][2 * hh + 1]};
            h[s][i][2 * hh] = y.x;
            h[s][i][2 * hh + 1] = y.y;
          }
          put_relu_f16(ex[s] + Y::ACT0, wv * N0 + i, lane, h[s][i]);
        }
      }
    }
    __syncthreads();
    // ---- layer 1: one fp16 product from the register-resident fragments -> act1 (one fp16 plane)
    {
      bf16x8 bin[NS][8];
#pragma unroll
      for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int ks = 0; ks < 8; ++ks) bin[s][ks] = PB::get_ks(ex[s] + Y::ACT0, ks, ol);
      f32x4 h1[NS][N1];
#pragma unroll
      for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int i = 0; i < N1; ++i) h1[s][i] = bias1[i];
      __builtin_amdgcn_sched_barrier(0);  // every B read before the first MFMA (each MFMA waits for its own read only)
#pragma unroll
      for (int kk = 0; kk < 8; ++kk)
#pragma unroll
        for (int s = 0; s < NS; ++s)
#pragma unroll
          for (int i = 0; i < N1; ++i) h1[s][i] = mmh_a(w1r[i][kk], bin[s][kk], h1[s][i]);
      mma_fence(h1);
#pragma unroll
      for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int i = 0; i < N1; ++i) put_relu_f16(ex[s] + Y::ACT1, wv * N1 + i, lane, h1[s][i]);
    }
    __syncthreads();
    // ---- last layer (m-tile wv): fp16 W hi (registers) + lo (LDS), two accumulation chains; x += dx -> xb, cost ring
    {
      bf16x8 bin[NS][4];
#pragma unroll
      for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) bin[s][ks] = PB::get_ks(ex[s] + Y::ACT1, ks, ol);
      f32x4 dd[NS][2];
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        dd[s][0] = biasx;
        dd[s][1] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
      }
      if constexpr (X3H_ASM) {
        if constexpr (L2X1) {
#pragma unroll
          for (int kk = 0; kk < 4; ++kk)
#pragma unroll
            for (int s = 0; s < NS; ++s) dd[s][kk & 1] = mmh_a(w2h[kk], bin[s][kk], dd[s][kk & 1]);
        } else {
          if constexpr (L2R) {
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) dd[0][kk & 1] = mmh2_aa(w2l[kk], w2h[kk], bin[0][kk], dd[0][kk & 1]);
          } else {
            bf16x8 lo[4];
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) lo[kk] = X3H_DIAG ? bin[0][kk] : frag(Y::F2L, wv * 4 + kk);
#pragma unroll
            for (int kk = 0; kk < 4; ++kk)
#pragma unroll
              for (int s = 0; s < NS; ++s)
                dd[s][kk & 1] = X3H_DIAG == 1 ? mmh_a(w2h[kk], bin[s][kk], dd[s][kk & 1])
                                              : mmh2_a(lo[kk], w2h[kk], bin[s][kk], dd[s][kk & 1]);
          }
        }
        mma_fence(dd);
      } else {
#pragma unroll
        for (int kk = 0; kk < 4; ++kk)
#pragma unroll
          for (int s = 0; s < NS; ++s) {
            if constexpr (L2X1)
              dd[s][kk & 1] = mmh(w2h[kk], bin[s][kk], dd[s][kk & 1]);
            else
              dd[s][kk & 1] = mmh(w2h[kk], bin[s][kk], mmh(frag(Y::F2L, wv * 4 + kk), bin[s][kk], dd[s][kk & 1]));
          }
      }
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        x[s] += dd[s][0] + dd[s][1];
        put_f16(ex[s] + Y::XB, wv, lane, x[s]);
        if (my_chunk >= 0)
          *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(ex[s] + Y::HIST) +
                                    ((t % Y::RING) * 16 + n) * CC::HS + 4 * my_chunk) = x[s];
      }
    }
    __syncthreads();
    if ((t + 1) % Y::RING == 0 || t + 1 == a.H) {  // ring full (or horizon done): one (step, sample) per lane group
      const int ts = t - t % Y::RING + ls;
      if (ls < Y::RING && ts <= t) {
#pragma unroll
        for (int s = 0; s < NS; ++s) cost[s] += ring_cost(s, ls, ts + 1);
      }
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
  if (a.terminal_weight != 0.0f && ls == 0) {
#pragma unroll
    for (int s = 0; s < NS; ++s) cost[s] += a.terminal_weight * ring_cost(s, (a.H - 1) % Y::RING, a.H);
  }
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    cost[s] = group_sum(cost[s]);
    if (g == 0) reinterpret_cast<float*>(ex[s] + Y::CP)[wv * 16 + n] = cost[s];
  }
  __syncthreads();
  kclock_record(a, kc);
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int ks = k + 16 * s;
    if (wv == 0 && g == 0 && ks < a.K) {
      const float* cp = reinterpret_cast<const float*>(ex[s] + Y::CP);
      float c = cp[n];
#pragma unroll
      for (int w2 = 1; w2 < 4; ++w2) c += cp[w2 * 16 + n];
      a.costs[(long)b * a.Kp + ks] = isfinite(c) ? c : INFINITY;
    }
  }
  if (a.xout && k == 0) {  // env step: final state of sample 0 (tile 0, lane n = 0 of the solve's first group)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int sl = 16 * wv + 4 * g + r;
      const int src = sl < 32 ? (sl < net.qp ? sl : -1) : (sl - 32 < net.qv ? net.qp + sl - 32 : -1);
      if (src >= 0) a.xout[(long)b * a.nx + src] = x[0][r];
    }
  }
}

// one group per block, two blocks per CU (the 8-solve shard: 512 groups)
template <int COST, bool L2X1>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void fc_rollout_kernel_x3h(SolveArgs a,
                                                                                                      FcArgs net) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  fc_x3h_body<COST, L2X1, 1>(a, net, lds);
}
// NS tiles per wave, one block per CU at one wave per SIMD (the 16-solve shard: 1024 groups in one round at NS = 4)
template <int COST, bool L2X1, int NS>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void fc_rollout_kernel_x3hw(SolveArgs a,
                                                                                                       FcArgs net) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  fc_x3h_body<COST, L2X1, NS>(a, net, lds);
}

// MPPI_X3H (read per launch): unset = this kernel wherever fc_rollout_kernel_x3d would run the fp16 form; 0 = never
// (x3d keeps it); 1 = the same (explicit)
bool fc_x3h_wanted(const SolveArgs& a, const FcArgs& fa) {
  if (!MPPI_X3_F16_L0 || fa.w_off[1] < 0 || fa.ln_n != 256 || a.Kp % 16 != 0 || fa.wmf16_0_off < 0) return false;
  if (X3H_B0MMA && fa.wmf16_0b_off < 0) return false;
  if (!x3_f16_on(a.H, fa.x3_f16, fa.wmf16_off)) return false;
  const char* e = std::getenv("MPPI_X3H");
  return !(e && e[0] == '0');
}

// tiles per wave: 1 (one group per block, two blocks per CU), or MPPI_X3H_NS=2/4 (read per launch) -- one block per CU
// at one wave per SIMD, NS static chains per wave: measured slower than the dynamic interleave of two blocks per CU at
// both shard sizes (same box: 8 solves 104.6 -> 126.5 us with NS = 2; 16 solves 205-206 us in two rounds of NS = 1 ->
// 218 us in one round of NS = 4, 255 us with NS = 2; profiles/r06_ab_x3h.log), kept as A/B arms
static int x3h_ns(const SolveArgs& a) {
  const char* e = std::getenv("MPPI_X3H_NS");
  int ns = e ? std::atoi(e) : 1;
  if (ns != 1 && ns != 2 && ns != 4) ns = 1;
  while (ns > 1 && (a.Kp >> 4) % ns != 0) ns >>= 1;  // a block's tiles belong to one solve
  return ns;
}

hipError_t launch_fc_x3h(const SolveArgs& a, const FcArgs& fa, hipStream_t stream) {
  const int groups = a.B * (a.Kp >> 4);
  if (a.Kp % 16 != 0 || groups < 1 || fa.wmf16_0_off < 0 || fa.wmf16_x_off < 0 || fa.wmf16_off < 0 ||
      (X3H_B0MMA && fa.wmf16_0b_off < 0))
    return hipErrorInvalidValue;
  const bool l2x1 = x3_f16_l2x1(fa.x3_f16);
  const int ns = x3h_ns(a);
  static const char* const names[2][3] = {
      {"fc_rollout_kernel_x3h<f16>", "fc_rollout_kernel_x3hw<f16,ns=2>", "fc_rollout_kernel_x3hw<f16,ns=4>"},
      {"fc_rollout_kernel_x3h<f16,l2=1>", "fc_rollout_kernel_x3hw<f16,l2=1,ns=2>", "fc_rollout_kernel_x3hw<f16,l2=1,ns=4>"}};
  note_kernel(names[l2x1][ns == 1 ? 0 : (ns == 2 ? 1 : 2)]);
  auto go = [&](auto kern, int bytes) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(kern, dim3(groups / ns), dim3(256), bytes, stream, a, fa);
    return hipGetLastError();
  };
  auto by_ns = [&](auto cost, auto l2) {
    constexpr int C = decltype(cost)::value;
    constexpr bool L2 = decltype(l2)::value;
    switch (ns) {
      case 2: return go(fc_rollout_kernel_x3hw<C, L2, 2>, X3hLay<C, 2>::BYTES);
      case 4: return go(fc_rollout_kernel_x3hw<C, L2, 4>, X3hLay<C, 4>::BYTES);
      default: return go(fc_rollout_kernel_x3h<C, L2>, X3hLay<C, 1>::BYTES);
    }
  };
  auto by_form = [&](auto cost) {
    return l2x1 ? by_ns(cost, std::true_type{}) : by_ns(cost, std::false_type{});
  };
  if (a.cost_kind == MPPI_COST_HUMANOID_V1) return by_form(std::integral_constant<int, MPPI_COST_HUMANOID_V1>{});
  return by_form(std::integral_constant<int, MPPI_COST_HUMANOID_V3>{});
}

}  // namespace mppi
