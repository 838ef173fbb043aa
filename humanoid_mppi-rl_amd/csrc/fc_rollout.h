// The fc-stack rollout kernel template (CA / MLP dynamics) and its launch templates, shared by kernels_fc.hip
// (MLP instantiations, the dispatcher) and kernels_fc_ca.hip (the CA instantiation): separate translation units
// so each takes its own codegen flags (build.py PER_FILE_FLAGS).
#pragma once

// Learned-dynamics MPPI rollout: x_{t+1} = x_t + net([x_t, u_t]) for every (solve, sample), the H loop
// inside the kernel, cost accumulated in registers.  Replaces the per-horizon-step torch launch chain of
// src/cartpole_mppi_estimator.py:84-119 / src/quadruped_mppi_estimator.py:67-78 (net = learning/model.py)
// and the K x H mj_step calls of src/Humanoid_mppi_v3.jl:131-150.
//
// Mapping (DESIGN.md "fc-stack rollout"):
//   * a GROUP = 16 samples of one solve, processed by S = 4 waves; lane l: sample n = l & 15, lane group
//     g = l >> 4.  Wave w of a group computes m-tiles [w*MT/S, (w+1)*MT/S) of every layer (M split), so
//     the per-step MFMA and VALU work of a sample group is spread over 4 SIMDs.  bf16: one group per block,
//     two blocks per CU (2 waves per SIMD) with independent barriers, so one group's barrier/LDS waits overlap
//     the other's issue; fp32: two groups per block.
//   * activations live in the MFMA C/D layout of v_mfma_f32_16x16x32_bf16 (m-tile mt, register r =
//     feature 16*mt + 4*g + r of sample n).  Each wave writes its output tiles to a per-group LDS exchange
//     buffer already in B-operand order (bf16 k-step ks = tiles {2ks, 2ks+1}, element j <-> feature
//     32ks+16(j>>2)+4g+(j&3)); after one barrier every wave reads the full input of the next layer with one
//     ds_read_b128 per lane per k-step.  The host packs the A operand (weights) in that permuted k order.
//   * bf16: every layer's A fragments for this wave's rows stay in VGPRs for the whole horizon (REG_MASK; CA:
//     32 + 64 + 16 VGPRs), loaded once per launch; per-wave biases and the folded LayerNorm's beta' live in
//     registers.  fp32 (parity mode): v_mfma_f32_16x16x4_f32, each D register is one 4-deep k-step, the fp32
//     image is read from L2.
//   * control/noise loads are raw buffer loads with per-lane offsets fixed for the horizon and a scalar
//     per-step offset.  The step is a dependent chain bound by its latency (4 barriers).
//   * CA's LayerNorm is folded into the weights on the host (centred rows, gamma in layer 1): only sum h^2 crosses
//     the waves, one barrier; y = relu(h rstd + beta').
//   * the running cost's state part is evaluated in batches from a 16-step LDS ring (one (step, sample) per lane);
//     its control part every step, two control slots per lane; the per-lane parts are summed once after the loop.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "costs.h"
#include "fc_common.h"
#include "mppi_internal.h"

namespace mppi {

// Diagnostic build only (-DMPPI_STAMPS): per-segment s_memtime sums of the horizon loop, accumulated over all
// waves into g_stamps (read by mppi_debug_stamps). The shipped kernel contains none of this.
#ifdef MPPI_STAMPS
constexpr int kNumStamps = 8;
static __device__ unsigned long long g_stamps[kNumStamps];  // one per translation unit (summed on read)
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

// ------------------------------------------------------------------------------------------------ kernel

// CA control loads (nets without a control input): prefetch distance in steps (= the step loop's unroll, <= 3).  Same
// box, 8-solve shard of config #4 (one-step base 78.2 us): PD 1 78.9-79.7, 2 75.8, 3 74.1 (profiles/r04_ab_prefetch.log).
// Split bf16 with two tiles per wave: 1 (a second buffer pair measured 1623 us per headline launch against 1605).
#ifndef MPPI_CTRL_PD
#define MPPI_CTRL_PD 3
#endif
template <int PREC, int NS>
constexpr int kCtrlPrefetch = PREC == MPPI_PREC_BF16X3 && NS == 2 ? 1 : MPPI_CTRL_PD;

// The kernel body, shared by the launch shapes below.  REGS: every layer's A fragments of this wave live in
// registers for the whole horizon (bf16 always; fp32 in the one-wave-per-SIMD kernel), else the fp32 image is
// streamed from L2 every step (the round-1 fp32 path, kept for A/B: MPPI_F32_STREAM=1).  NS: sample tiles per wave.
// NS = 1 is one 16-sample group per 4 waves; NS = 2 (fc_rollout_kernel_wide) gives every wave two consecutive 16-sample
// groups of one solve, each with its own exchange region, sharing the barriers: two independent MFMA / VALU chains
// per wave in every phase, in place of the two co-resident blocks per CU of the NS = 1 kernel.
template <int ARCH, int PREC, int COST, bool REGS, int NS, int L1T = 3>
__device__ __forceinline__ void fc_rollout_body(const SolveArgs& a, const FcArgs& net, char* lds) {
  using A = Arch<ARCH>;
  using PR = P<PREC>;
  using L = Lay<ARCH, PREC, COST>;
  using Bop = typename PR::Bop;
  using Wt = typename PR::Wt;
  constexpr int S = kSplit;
  constexpr int N0 = A::MT0 / S, N1 = A::MT1 / S, N2 = A::MT2 / S, NX = 4 / S;
  constexpr int NL = A::NL;
  const KClock kc = kclock_begin(a);

  const int img_lds = PREC == MPPI_PREC_BF16 ? net.lds_bytes : 0;
  if constexpr (PREC == MPPI_PREC_BF16) {
    const int4* src = reinterpret_cast<const int4*>(net.img);
    int4* dst = reinterpret_cast<int4*>(lds);
    for (int i = threadIdx.x; i < (net.lds_bytes >> 4); i += blockDim.x) dst[i] = src[i];
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) *a.status = 0u;  // per-solve status word (read after the reduce)
  // static issue priority for half of the blocks: the two blocks sharing a CU otherwise tie on every arbitration
  // (MI355X_MICROARCH.md, two waves per SIMD, item 4); same-box A/B on config #4: -1.5..2 % step time
  if (NS == 1 && (blockIdx.x & 1)) __builtin_amdgcn_s_setprio(1);
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4;
  const int n = lane & 15;
  const int wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave in block (uniform)
  const int wv = wib % S;                                             // wave in group
  const int grp_in_blk = wib / S;
  const int grp = (blockIdx.x * net.groups_per_block + grp_in_blk) * NS;  // group of tile 0; tile s: grp + s
  const int groups_per_solve = a.Kp >> 4;
  const int total_groups = a.B * groups_per_solve;
  // a group past the end still runs the loop (barriers are block-wide) on a clamped copy and writes nothing.  NS = 2:
  // launch_t requires groups_per_solve % 2 == 0, so both tiles are live and belong to solve b.
  const bool live = grp < total_groups;
  const int gc = live ? grp : total_groups - 1;
  const int b = gc / groups_per_solve;
  const int k = (gc - b * groups_per_solve) * 16 + n;  // sample of tile 0; tile s: k + 16 s
  char* ex[NS];                                         // each tile's exchange region
#pragma unroll
  for (int s = 0; s < NS; ++s) ex[s] = lds + img_lds + (grp_in_blk * NS + s) * L::BYTES;

  const char* img;
  if constexpr (PREC == MPPI_PREC_BF16)
    img = lds;
  else
    img = net.img;
  auto Wp = [&](int l) { return reinterpret_cast<const Wt*>(img + net.w_off[l]); };
  // bf16: the layers of A::REG_MASK (all of them) keep this wave's A fragments in VGPRs for the whole horizon
  // (global image, read once): no weight traffic at all inside the horizon loop.  A layer outside the mask would
  // be staged in LDS (the image prefix [0, lds_bytes)) and read per step.
  constexpr bool RG = REGS;
  constexpr bool R0 = RG && (A::REG_MASK & 1), R1 = RG && (A::REG_MASK & 2);
  constexpr bool R2 = RG && NL == 4 && (A::REG_MASK & 4), RX = RG && ((A::REG_MASK >> (NL - 1)) & 1);
  constexpr int KSB0 = PR::KS(A::IN_T) / A::BLOCKS0, KS1 = PR::KS(A::MT0), KS2 = PR::KS(A::MT1);
  constexpr int KSX = PR::KS(NL == 4 ? A::MT2 : A::MT1);
  Wt w0r[R0 ? N0 : 1][R0 ? KSB0 : 1], w1r[R1 ? N1 : 1][R1 ? KS1 : 1], w2r[R2 ? N2 : 1][R2 ? KS2 : 1],
      wxr[RX ? NX : 1][RX ? KSX : 1];
  auto Wg = [&](int l) { return reinterpret_cast<const Wt*>(net.img + net.w_off[l]); };
  if constexpr (R0) load_frags<PREC>(w0r, Wg(0), wv * N0, lane);
  if constexpr (R1) load_frags<PREC>(w1r, Wg(1), wv * N1, lane);
  if constexpr (R2) load_frags<PREC>(w2r, Wg(2), wv * N2, lane);
  if constexpr (RX) load_frags<PREC>(wxr, Wg(NL - 1), wv * NX, lane);
  auto bias_img = [&](int l) { return reinterpret_cast<const float*>(net.img + net.b_off[l]); };
  auto ld4 = [&](const float* p, int row) { return *reinterpret_cast<const f32x4*>(p + row); };
  // register-resident fragments: the split-bf16 CA reads them from AGPRs in its own MFMA statements (fc_common.h mma_a;
  // each layer's accumulators then pass mma_fence before their epilogue).  Same box, config #4 CA: 8 solves 203.3 ->
  // 188.8 us, 16 solves 405.6 -> 377.5 us; the humanoid MLP (4 layers) 194.8 -> 202.1 us at 8 solves, so not there
  // (profiles/r05_ab_msplit_agpr.log)
  constexpr bool AF = PREC == MPPI_PREC_BF16X3 && ARCH == kArchCA;
  constexpr bool L1T2 = AF && L1T == 2;  // layer 1 with two products on act0's hi plane (fc_common.h x3_l1_terms)
  auto mmr = [&](const Wt& w, const Bop& bo, const f32x4& c) {
    if constexpr (AF)
      return PR::mma_a(w, bo, c);
    else
      return PR::mma(w, bo, c);
  };

  // per-wave constants in registers: biases (and LayerNorm gamma/beta) of the own tiles
  f32x4 bias0[N0], bias1[N1], bias2[N2 > 0 ? N2 : 1], biasx[NX], lnb[N0];
#pragma unroll
  for (int i = 0; i < N0; ++i) {
    const int row = 16 * (wv * N0 + i) + 4 * g;
    bias0[i] = ld4(bias_img(0), row);
    if constexpr (A::LN0) {
      lnb[i] = ld4(reinterpret_cast<const float*>(net.img + net.lnb_off), row);  // beta' (LN folded, host)
    }
  }
#pragma unroll
  for (int i = 0; i < N1; ++i) bias1[i] = ld4(bias_img(1), 16 * (wv * N1 + i) + 4 * g);
  if constexpr (NL == 4) {
#pragma unroll
    for (int i = 0; i < N2; ++i) bias2[i] = ld4(bias_img(2), 16 * (wv * N2 + i) + 4 * g);
  }
#pragma unroll
  for (int i = 0; i < NX; ++i) biasx[i] = ld4(bias_img(NL - 1), 16 * (wv * NX + i) + 4 * g);

  // own state tiles (fp32), initial value from x0 (every tile: the same x0 of solve b); published to the exchanges
  f32x4 x[NS][NX];
  const float* x0 = a.x0 + (long)b * a.nx;
#pragma unroll
  for (int i = 0; i < NX; ++i) {
    const int mt = wv * NX + i;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int sl = 16 * mt + 4 * g + r;
      const int src = sl < 32 ? (sl < net.qp ? sl : -1) : (sl - 32 < net.qv ? net.qp + sl - 32 : -1);
      x[0][i][r] = src >= 0 ? x0[src] : 0.0f;
    }
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      x[s][i] = x[0][i];
      PR::put_tile(ex[s] + L::XB, mt, lane, x[s][i]);
    }
  }


  const int bs = __builtin_amdgcn_readfirstlane(b);  // block-uniform (a block's groups share one solve)
  float cx[MPPI_CTX_MAX];  // per-solve cost context (scalar loads)
#pragma unroll
  for (int i = 0; i < MPPI_CTX_MAX; ++i) cx[i] = a.ctx ? a.ctx[(long)bs * MPPI_CTX_MAX + i] : a.ctx_default[i];
  constexpr bool U_IN = A::IN_T == 6;  // the net takes the controls as input (MLP); CA does not

  // Control loads (nets with a control input only): raw buffer loads through block-uniform descriptors (U rows and
  // noise block of solve b), a per-lane voffset fixed for the whole horizon and a scalar soffset per step (+ 64 bytes
  // = 16 samples per further tile): no per-step address VALU.  Pad slots (control index >= nu) point past the
  // descriptor range, where buffer loads return 0.  Loads are unconditional: a conditional load makes hipcc branch
  // around it and wait vmcnt(0) per element, serialising the prefetch.
  const auto rU = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.U) + (long)bs * a.nu * a.H, 0,
                                                    a.nu * a.H * 4, 0x00020000);
  const auto rE = __builtin_amdgcn_make_buffer_rsrc(a.noise + (long)bs * a.nu * a.H * a.Kp, 0,
                                                    a.nu * a.H * a.Kp * 4, 0x00020000);
  // control slots of this lane group: {4g..4g+3, 16+4g..16+4g+3} (u tiles 0,1 of the D layout)
  int uoff[U_IN ? 8 : 1], eoff[U_IN ? 8 : 1];
  if constexpr (U_IN) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int us = (j < 4) ? 4 * g + j : 16 + 4 * g + (j - 4);
      uoff[j] = us < a.nu ? us * a.H * 4 : 0x7FFFFFF0;
      eoff[j] = us < a.nu ? (us * a.H * a.Kp + k) * 4 : 0x7FFFFFF0;
    }
  }
  auto load_u = [&](int t, int s, f32x4 (&u)[2]) {
    const int su = t * 4, se = t * a.Kp * 4 + 64 * s;
#pragma unroll
    for (int j = 0; j < 8; ++j)
      u[j >> 2][j & 3] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rU, uoff[j], su, 0)) +
                         __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rE, eoff[j], se, 0));
  };
  f32x4 un[NS][2];
  if constexpr (U_IN) {
#pragma unroll
    for (int s = 0; s < NS; ++s) load_u(0, s, un[s]);
  }

  // Running cost, batched over the ring (CostChunks).  This lane evaluates the STATE part of the cost of local step
  // ls = 4 wv + g of every ring for sample n.
  using CC = CostChunks<ARCH, COST>;
  constexpr CostIdx ci = cost_idx(COST);
  float* hist[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) hist[s] = reinterpret_cast<float*>(ex[s] + L::HIST);
  int my_chunk = -1;  // this lane's ring chunk (tile wv, lane group g), -1: the cost reads none of its slots
#pragma unroll
  for (int e = 0; e < 16; ++e)
    if (e == 4 * wv + g) my_chunk = CC::chunk(e / 4, e % 4);
  const int ls = 4 * wv + g;
  // Control part of the running cost, every step, spread over the group's 256 lanes: lane (wave wv, lane group g)
  // of sample n accounts for controls {4g + wv, 16 + 4g + wv} (all 32 control slots over the 4 waves).  ctrl_term_t
  // is linear in (u0^2, sum_j u_j^2), so these per-lane terms add up to the reference's per-(step, sample) term.  The
  // MLP already holds those two u values (its layer-0 operand).  CA loads U and eps for them PD steps ahead into PD
  // register buffers (the step loop is unrolled by PD, so buffer P = t % PD is a compile-time register set and no
  // moves sit between a load and its use): with one step of lead the loads' memory latency was exposed at every step
  // end.  U staged in LDS (only eps in registers) measured slower: 77.1 us at PD = 2 against 75.8 (two more LDS reads
  // in every step's in-order LDS queue).  A flush-time load of all nu noise values per
  // (step, sample) had exposed the latency every 16 steps (round 2).
  const float cl = a.ctrl_clamp > 0.0f ? a.ctrl_clamp : INFINITY;  // clamp as one v_med3 (+-inf: none)
  constexpr int PD = U_IN ? 1 : kCtrlPrefetch<PREC, NS>;
  int cuoff[2], ceoff[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int us = 16 * i + 4 * g + wv;
    cuoff[i] = us < a.nu ? us * a.H * 4 : 0x7FFFFFF0;
    ceoff[i] = us < a.nu ? (us * a.H * a.Kp + k) * 4 : 0x7FFFFFF0;
  }
  auto load_cu = [&](int t, int s, float (&cu)[2], float (&ce)[2]) {
    const int su = t * 4, se = t * a.Kp * 4 + 64 * s;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      cu[i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rU, cuoff[i], su, 0));
      ce[i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rE, ceoff[i], se, 0));
    }
  };
  // PD = 1 carries the sums U + eps (the add, and its wait, at the step end: measured faster there than raw values
  // summed at the next step's top); PD >= 2 carries the raw values of PD steps
  float cun[NS][2], cuu[PD][NS][2], cue[PD][NS][2];
  auto load_sum = [&](int t, int s) {
    float cu[2], ce[2];
    load_cu(t, s, cu, ce);
    cun[s][0] = cu[0] + ce[0];
    cun[s][1] = cu[1] + ce[1];
  };
  if constexpr (!U_IN && PD == 1) {
#pragma unroll
    for (int s = 0; s < NS; ++s) load_sum(0, s);
  } else if constexpr (!U_IN) {
#pragma unroll
    for (int j = 0; j < PD; ++j) {
      asm volatile("" ::: "memory");  // issue order step 0, 1, ..., PD - 1 (the loop's wait counts assume it)
#pragma unroll
      for (int s = 0; s < NS; ++s) load_cu(j < a.H ? j : a.H - 1, s, cuu[j][s], cue[j][s]);
    }
  }
  float cost[NS];  // this lane's share of each tile's sample-n running + terminal cost
#pragma unroll
  for (int s = 0; s < NS; ++s) cost[s] = 0.0f;
  auto ctrl_acc = [&](int s, float u_lo, float u_hi) {  // controls 4g + wv and 16 + 4g + wv, clamped
    cost[s] += ctrl_term_t<COST>((g == 0 && wv == 0) ? u_lo : 0.0f, fmaf(u_lo, u_lo, u_hi * u_hi));
  };
  // the state part of the cost of (ring slot r, sample n) of tile s from the ring row
  auto ring_cost = [&](int s, int r, int t1) {
    f32x4 ch[CC::NCH];
#pragma unroll
    for (int c = 0; c < CC::NCH; ++c) ch[c] = *reinterpret_cast<const f32x4*>(hist[s] + (r * 16 + n) * CC::HS + 4 * c);
    float v[kCostMaxIdx];
#pragma unroll
    for (int i = 0; i < ci.n; ++i) {
      const int sl = CC::slot(ci.idx[i]);
      v[i] = ch[CC::chunk(sl / 16, (sl % 16) / 4)][sl % 4];
    }
    return cost_eval_t<COST>(v, 0.0f, 0.0f, cx, t1);
  };
  __syncthreads();  // weight image + initial state exchange visible

#ifdef MPPI_STAMPS
  unsigned long long st_[kNumStamps] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long tprev_ = __builtin_amdgcn_s_memtime();
#endif
  // one step of the horizon; PAR (t % PD as a type) selects the control prefetch buffer
  auto step = [&](const int t, auto PAR) __attribute__((always_inline)) {
    constexpr int P = decltype(PAR)::value;
    STAMP(0);
    int ol = lane;  // streamed weights: an opaque copy, fragment addresses re-derived every step (no LICM of loads)
    if constexpr (!REGS) asm volatile("" : "+v"(ol));
    f32x4 u[NS][2];
    const int tn = t + 1 < a.H ? t + 1 : t;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      if constexpr (U_IN) {
        u[s][0] = un[s][0];
        u[s][1] = un[s][1];
        load_u(tn, s, un[s]);  // prefetch the next step's controls
#pragma unroll
        for (int j = 0; j < 8; ++j) u[s][j >> 2][j & 3] = __builtin_amdgcn_fmed3f(u[s][j >> 2][j & 3], -cl, cl);
        ctrl_acc(s, u[s][0][wv], u[s][1][wv]);  // wv: wave-uniform
      } else {
        float c0, c1;
        if constexpr (PD == 1) {
          c0 = __builtin_amdgcn_fmed3f(cun[s][0], -cl, cl);
          c1 = __builtin_amdgcn_fmed3f(cun[s][1], -cl, cl);
#ifndef MPPI_DIAG_NOCTRL
          load_sum(tn, s);  // prefetch the next step's two controls
#endif
        } else {
          // buffer P's values are consumed here, before the loads that refill it: the refill lands in the same
          // registers (otherwise hipcc keeps both live and copies at the loop latch, waiting there for the new loads)
          c0 = __builtin_amdgcn_fmed3f(cuu[P][s][0] + cue[P][s][0], -cl, cl);
          c1 = __builtin_amdgcn_fmed3f(cuu[P][s][1] + cue[P][s][1], -cl, cl);
          asm volatile("" : "+v"(c0), "+v"(c1)::"memory");
#ifndef MPPI_DIAG_NOCTRL
          load_cu(t + PD < a.H ? t + PD : a.H - 1, s, cuu[P][s], cue[P][s]);  // prefetch step t + PD's controls
#endif
        }
        ctrl_acc(s, c0, c1);
      }
    }

    // ---- layer 0: own rows of W0 [x ; u] (+ LayerNorm, ReLU) -> act0
    {
      constexpr int KS = PR::KS(A::IN_T);
      constexpr int KSX = PR::KS(4);
      constexpr int KSB = KS / A::BLOCKS0;  // k-steps of this wave's (diagonal) block
      Bop bin[NS][KSB];
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        if constexpr (A::BLOCKS0 == 1) {
#pragma unroll
          for (int ks = 0; ks < KSX; ++ks) bin[s][ks] = PR::get_ks(ex[s] + L::XB, ks, ol);
          if constexpr (A::IN_T == 6) PR::put_u(bin[s] + KSX, u[s]);
        } else {
          static_assert(A::IN_T == 4, "block-diagonal layer 0 reads state slots only");
          const int blk = (wv * N0) / (A::MT0 / A::BLOCKS0);  // runtime block: index the LDS address, not registers
#pragma unroll
          for (int kk = 0; kk < KSB; ++kk) bin[s][kk] = PR::get_ks(ex[s] + L::XB, blk * KSB + kk, ol);
        }
      }
      f32x4 h[NS][N0];
#pragma unroll
      for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int i = 0; i < N0; ++i) h[s][i] = bias0[i];
      if constexpr (R0) {
#pragma unroll
        for (int kk = 0; kk < KSB; ++kk)
#pragma unroll
          for (int s = 0; s < NS; ++s)
#pragma unroll
            for (int i = 0; i < N0; ++i) h[s][i] = mmr(w0r[i][kk], bin[s][kk], h[s][i]);
        if constexpr (AF) mma_fence(h);
      } else {
#pragma unroll
        for (int s = 0; s < NS; ++s) mfma_rows<PREC, KSB, N0>(h[s], bin[s], Wp(0), wv * N0, ol);
      }
      if constexpr (A::LN0) {
        // LayerNorm folded into the weights on the host (mppi_nets.cpp): the rows are centred (mean 0 for every
        // input) and gamma sits in layer 1, so y = relu(h rstd + beta'), rstd = rsqrt(mean(h^2) + eps).  Only
        // sum h^2 crosses the waves: per-wave partial sums in packed fp32, one LDS float per (wave, sample).
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          f32x2 q2[N0];  // one partial per tile: a depth-2 chain per tile, then a tree (not 2 N0 dependent FMAs)
#pragma unroll
          for (int i = 0; i < N0; ++i) {
            const f32x2 lo = {h[s][i][0], h[s][i][1]}, hi = {h[s][i][2], h[s][i][3]};
            q2[i] = hi * hi + lo * lo;
          }
#pragma unroll
          for (int w2 = 1; w2 < N0; w2 *= 2)
#pragma unroll
            for (int i = 0; i + w2 < N0; i += 2 * w2) q2[i] = q2[i] + q2[i + w2];
          const float q_w = group_sum(q2[0].x + q2[0].y);
          float* st = reinterpret_cast<float*>(ex[s] + L::ST);
          st[wv * 16 + n] = q_w;  // the 4 lane groups store the same value (no exec masking)
        }
        STAMP(1);
#ifndef MPPI_DIAG_NOLNBAR  // timing-only diagnostic builds (results wrong): no LayerNorm statistic exchange
        __syncthreads();
#endif
        STAMP(2);
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          const float* st = reinterpret_cast<const float*>(ex[s] + L::ST);
          float q = st[n];
#ifndef MPPI_DIAG_NOLNBAR
#pragma unroll
          for (int w2 = 1; w2 < S; ++w2) q += st[w2 * 16 + n];  // fixed order
#else
          q *= 4.0f;
#endif
          const float rstd = __builtin_amdgcn_rsqf(q * (1.0f / (16.0f * A::MT0)) + 1e-5f);  // arg >= 1e-5: no denormal
          const f32x2 r2 = {rstd, rstd};
#pragma unroll
          for (int i = 0; i < N0; ++i)
#pragma unroll
            for (int hh = 0; hh < 2; ++hh) {
              const f32x2 y =
                  f32x2{h[s][i][2 * hh], h[s][i][2 * hh + 1]} * r2 + f32x2{lnb[i][2 * hh], lnb[i][2 * hh + 1]};
              h[s][i][2 * hh] = y.x;
              h[s][i][2 * hh + 1] = y.y;
            }
        }
      }
#pragma unroll
      for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int i = 0; i < N0; ++i) {
          if constexpr (L1T2)
            PR::put_tile_relu_hi(ex[s] + L::ACT0, wv * N0 + i, lane, h[s][i]);
          else
            PR::put_tile_relu(ex[s] + L::ACT0, wv * N0 + i, lane, h[s][i]);
        }
    }
#ifndef MPPI_DIAG_NOBAR2
    __syncthreads();
#endif
    STAMP(3);

    // ---- layer 1 -> act1
    {
      constexpr int KS = PR::KS(A::MT0);
      Bop bin[NS][KS];
#pragma unroll
      for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          if constexpr (L1T2)
            bin[s][ks].hi = PR::get_ks_hi(ex[s] + L::ACT0, ks, ol);
          else
            bin[s][ks] = PR::get_ks(ex[s] + L::ACT0, ks, ol);
        }
      f32x4 h[NS][N1];
#pragma unroll
      for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int i = 0; i < N1; ++i) h[s][i] = bias1[i];
      if constexpr (R1) {
        // every k-step's B operand read issued before the first MFMA (each MFMA then waits only for its own read):
        // one exposed LDS latency, not KS/2 (the default schedule read them two at a time, each pair waited on)
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int kk = 0; kk < KS; ++kk)
#pragma unroll
          for (int s = 0; s < NS; ++s)
#pragma unroll
            for (int i = 0; i < N1; ++i) {
              if constexpr (L1T2)
                h[s][i] = PR::mma_a2(w1r[i][kk], bin[s][kk].hi, h[s][i]);
              else
                h[s][i] = mmr(w1r[i][kk], bin[s][kk], h[s][i]);
            }
        if constexpr (AF) mma_fence(h);
      } else {
#pragma unroll
        for (int s = 0; s < NS; ++s) mfma_rows<PREC, KS, N1>(h[s], bin[s], Wp(1), wv * N1, ol);
      }
#pragma unroll
      for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int i = 0; i < N1; ++i) PR::put_tile_relu(ex[s] + L::ACT1, wv * N1 + i, lane, h[s][i]);
    }
#ifndef MPPI_DIAG_NOBAR3
    __syncthreads();
#endif

    // ---- (MLP) layer 2 -> act2
    if constexpr (NL == 4) {
      constexpr int KS = PR::KS(A::MT1);
      Bop bin[NS][KS];
#pragma unroll
      for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) bin[s][ks] = PR::get_ks(ex[s] + L::ACT1, ks, ol);
      f32x4 h[NS][N2];
#pragma unroll
      for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int i = 0; i < N2; ++i) h[s][i] = bias2[i];
      if constexpr (R2) {
#pragma unroll
        for (int kk = 0; kk < KS; ++kk)
#pragma unroll
          for (int s = 0; s < NS; ++s)
#pragma unroll
            for (int i = 0; i < N2; ++i) h[s][i] = mmr(w2r[i][kk], bin[s][kk], h[s][i]);
        if constexpr (AF) mma_fence(h);
      } else {
#pragma unroll
        for (int s = 0; s < NS; ++s) mfma_rows<PREC, KS, N2>(h[s], bin[s], Wp(2), wv * N2, ol);
      }
#pragma unroll
      for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int i = 0; i < N2; ++i) PR::put_tile_relu(ex[s] + L::ACT2, wv * N2 + i, lane, h[s][i]);
      __syncthreads();
    }
    STAMP(4);

    // ---- last layer: own state tiles, x += dx -> xb (B operands of the next step) and the cost ring
    {
      constexpr int MTL = NL == 4 ? A::MT2 : A::MT1;
      constexpr int KS = PR::KS(MTL);
      Bop bin[NS][KS];
#pragma unroll
      for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) bin[s][ks] = PR::get_ks(ex[s] + (NL == 4 ? L::ACT2 : L::ACT1), ks, ol);
      f32x4 dx[NS][NX];
#pragma unroll
      for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int i = 0; i < NX; ++i) dx[s][i] = biasx[i];
      if constexpr (RX && KS % 2 == 0) {
        // two accumulation chains (even / odd k-steps) of KS/2 dependent MFMAs instead of one of KS
        f32x4 d1[NS][NX];
#pragma unroll
        for (int s = 0; s < NS; ++s)
#pragma unroll
          for (int i = 0; i < NX; ++i) d1[s][i] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
        __builtin_amdgcn_sched_barrier(0);  // all KS operand reads before the first MFMA (as layer 1)
#pragma unroll
        for (int kk = 0; kk < KS; kk += 2)
#pragma unroll
          for (int s = 0; s < NS; ++s)
#pragma unroll
            for (int i = 0; i < NX; ++i) {
              dx[s][i] = mmr(wxr[i][kk], bin[s][kk], dx[s][i]);
              d1[s][i] = mmr(wxr[i][kk + 1], bin[s][kk + 1], d1[s][i]);
            }
        if constexpr (AF) {
          mma_fence(dx);
          mma_fence<false>(d1);  // (its MFMAs precede dx's pad)
        }
#pragma unroll
        for (int s = 0; s < NS; ++s)
#pragma unroll
          for (int i = 0; i < NX; ++i) dx[s][i] += d1[s][i];
      } else if constexpr (RX) {
#pragma unroll
        for (int s = 0; s < NS; ++s) {
#pragma unroll
          for (int kk = 0; kk < KS; ++kk)
#pragma unroll
            for (int i = 0; i < NX; ++i) dx[s][i] = mmr(wxr[i][kk], bin[s][kk], dx[s][i]);
        }
        if constexpr (AF) mma_fence(dx);
      } else {
#pragma unroll
        for (int s = 0; s < NS; ++s) mfma_rows<PREC, KS, NX>(dx[s], bin[s], Wp(NL - 1), wv * NX, ol);
      }
      static_assert(NX == 1, "one state tile per wave");
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        x[s][0] += dx[s][0];
        PR::put_tile(ex[s] + L::XB, wv, lane, x[s][0]);
        if (my_chunk >= 0)
          *reinterpret_cast<f32x4*>(hist[s] + ((t % kRing) * 16 + n) * CC::HS + 4 * my_chunk) = x[s][0];
      }
    }
#ifndef MPPI_DIAG_NOBAR4
    __syncthreads();
#endif
    STAMP(5);
    // ---- ring full (or horizon done): every lane evaluates the running cost of one (step, sample) per tile
#ifdef MPPI_DIAG_NOCOST
    if (t + 1 == a.H) {
#else
    if ((t + 1) % kRing == 0 || t + 1 == a.H) {
#endif
      const int ts = t - t % kRing + ls;
      if (ts <= t) {
#pragma unroll
        for (int s = 0; s < NS; ++s) cost[s] += ring_cost(s, ls, ts + 1);
      }
    }
    STAMP(6);
  };
  // whole chunks of PD steps, unconditional (a conditional step inside the loop made hipcc's wait counts at the loop
  // head conservative: vmcnt(0)), then the < PD tail steps
  int t0 = 0;
  for (; t0 + PD <= a.H; t0 += PD) {
    step(t0, std::integral_constant<int, 0>{});
    if constexpr (PD > 1) step(t0 + 1, std::integral_constant<int, 1 % PD>{});
    if constexpr (PD > 2) step(t0 + 2, std::integral_constant<int, 2 % PD>{});
  }
  if constexpr (PD > 1) if (t0 < a.H) step(t0, std::integral_constant<int, 0>{});
  if constexpr (PD > 2) if (t0 + 1 < a.H) step(t0 + 1, std::integral_constant<int, 1 % PD>{});
  // terminal cost on x_H (ring slot of step H-1), once per sample
  if (a.terminal_weight != 0.0f && ls == 0) {
#pragma unroll
    for (int s = 0; s < NS; ++s) cost[s] += a.terminal_weight * ring_cost(s, (a.H - 1) % kRing, a.H);
  }
#pragma unroll
  for (int s = 0; s < NS; ++s) cost[s] = group_sum(cost[s]);
#ifdef MPPI_STAMPS
  if (lane == 0)
    for (int i = 0; i < kNumStamps; ++i) atomicAdd(&g_stamps[i], st_[i]);
#endif
  // sum the S partial costs in a fixed order
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    float* cp = reinterpret_cast<float*>(ex[s] + L::CP);
    if (g == 0) cp[wv * 16 + n] = cost[s];
  }
  __syncthreads();
  kclock_record(a, kc);
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int ks = k + 16 * s;
    if (wv == 0 && g == 0 && live && ks < a.K) {
      const float* cp = reinterpret_cast<const float*>(ex[s] + L::CP);
      float c = cp[n];
#pragma unroll
      for (int w2 = 1; w2 < S; ++w2) c += cp[w2 * 16 + n];
      a.costs[(long)b * a.Kp + ks] = isfinite(c) ? c : INFINITY;
    }
  }
  if (a.xout && live && k == 0) {  // env step: final state of sample 0 (tile 0, lanes n = 0 of the solve's first group)
#pragma unroll
    for (int i = 0; i < NX; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int sl = 16 * (wv * NX + i) + 4 * g + r;
        const int src = sl < 32 ? (sl < net.qp ? sl : -1) : (sl - 32 < net.qv ? net.qp + sl - 32 : -1);
        if (src >= 0) a.xout[(long)b * a.nx + src] = x[0][i][r];
      }
  }
}

// waves_per_eu(1,2): at most 2 waves per SIMD (<= 2 blocks of 4 waves per CU); telling hipcc the real occupancy
// lets it keep every layer's A fragments in VGPRs instead of minimising registers.  bf16 (fragments in registers)
// and the streamed fp32 path.
template <int ARCH, int PREC, int COST>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(1, 2))) void fc_rollout_kernel(SolveArgs a,
                                                                                                   FcArgs net) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  fc_rollout_body<ARCH, PREC, COST, PREC == MPPI_PREC_BF16, 1>(a, net, lds);
}

// bf16, two sample tiles per wave (NS = 2) at one wave per SIMD: one 4-wave block of 32 samples per CU, every
// phase holding two independent chains, and the whole 512-entry VGPR/AGPR file for the doubled activations.
template <int ARCH, int COST>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void fc_rollout_kernel_wide(SolveArgs a,
                                                                                                       FcArgs net) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  fc_rollout_body<ARCH, MPPI_PREC_BF16, COST, true, 2>(a, net, lds);
}

// Exact fp32 (MPPI_PREC_FP32): v_mfma_f32_16x16x4_f32 is 1/16 of the bf16 rate (32 cycles per MFMA per SIMD), so the
// step is MFMA-issue-bound once the fragments stop streaming from L2.  Every layer's fp32 A fragments of a wave stay
// in registers (folded CA: 64 + 128 + 32 = 224 per lane; MLP 208) at ONE wave per SIMD, where the unified 512-entry
// VGPR/AGPR file holds them (MFMA A operands may be AGPRs); one group of 4 waves per block and per CU.
template <int ARCH, int COST>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void fc_rollout_kernel_f32(SolveArgs a,
                                                                                                      FcArgs net) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  fc_rollout_body<ARCH, MPPI_PREC_FP32, COST, true, 1>(a, net, lds);
}

// Split bf16 (MPPI_PREC_BF16X3, fp32-accurate): the same body, every product on three bf16 MFMAs (fc_common.h P<>), every
// layer's hi / lo fragments of a wave in registers (CA 28 fragments x 8 = 224 VGPRs, MLP 208) at one wave per SIMD, as
// the exact-fp32 kernel: 3 x 16 cycles of matrix pipe per 16x16x32 product instead of 8 x 32 for the f32 MFMAs.
template <int ARCH, int COST, int L1T>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void fc_rollout_kernel_x3(SolveArgs a,
                                                                                                     FcArgs net) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  fc_rollout_body<ARCH, MPPI_PREC_BF16X3, COST, true, 1, L1T>(a, net, lds);
}

// ... with two 16-sample tiles per wave (NS = 2): one 4-wave block of 32 samples of one solve per CU, each fragment
// feeding both tiles' MFMAs, two independent chains in every phase to cover the MFMA and LDS latencies that one wave per
// SIMD leaves exposed
template <int ARCH, int COST, int L1T>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void fc_rollout_kernel_x3w(SolveArgs a,
                                                                                                      FcArgs net) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  fc_rollout_body<ARCH, MPPI_PREC_BF16X3, COST, true, 2, L1T>(a, net, lds);
}
int fc_x3_tiles();  // MPPI_X3_TILES=1/2: split-bf16 sample tiles per wave (read per launch; default 2); kernels_fc.hip

bool fc_f32_stream();  // MPPI_F32_STREAM=1: the streamed fp32 kernel (A/B); kernels_fc.hip
#ifdef MPPI_AB_ARMS  // the A/B-only library (csrc/ab/, MPPI_AB_ARMS=1 build.py); not in the shipped libmppi_hip.so
int fc_wide();         // MPPI_FC_WIDE=0/1: bf16 with two sample tiles per wave (fc_rollout_kernel_wide); kernels_fc.hip
// the wide kernel's launch (its own translation unit and codegen flags, build.py PER_FILE_FLAGS); ab/kernels_fc_wide.hip
hipError_t launch_fc_wide(int arch, int cost, const SolveArgs& a, FcArgs fa, int img_lds, hipStream_t stream);
#endif

template <int ARCH, int PREC, int COST>
static hipError_t launch_t(const SolveArgs& a, FcArgs fa, int img_lds, hipStream_t stream) {
  using L = Lay<ARCH, PREC, COST>;
  const int total_groups = a.B * (a.Kp >> 4);
  if constexpr (PREC == MPPI_PREC_BF16X3) {  // 4 waves per block, one wave per SIMD; 1 or 2 sample tiles per wave
    fa.groups_per_block = 1;
    const bool wide = fc_x3_tiles() == 2 && (a.Kp >> 4) % 2 == 0;
    const bool two = ARCH == kArchCA && x3_l1_terms(a.H, fa.x3_l1) == 2;  // (the MLP keeps three products: fc_common.h)
    auto kern = wide ? (two ? fc_rollout_kernel_x3w<ARCH, COST, 2> : fc_rollout_kernel_x3w<ARCH, COST, 3>)
                     : (two ? fc_rollout_kernel_x3<ARCH, COST, 2> : fc_rollout_kernel_x3<ARCH, COST, 3>);
    const int lds = (wide ? 2 : 1) * L::BYTES;
    note_kernel(wide ? (two ? "fc_rollout_kernel_x3w<l1=2>" : "fc_rollout_kernel_x3w<l1=3>")
                     : (two ? "fc_rollout_kernel_x3<l1=2>" : "fc_rollout_kernel_x3<l1=3>"));
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(kern, dim3(wide ? total_groups / 2 : total_groups), dim3(64 * kSplit), lds, stream, a, fa);
    return hipGetLastError();
  }
  const bool f32_regs = PREC == MPPI_PREC_FP32 && !fc_f32_stream();
  // bf16 wide: two consecutive groups of one solve per wave, one 4-wave block per CU (kernels_fc_wide.hip); only when
  // the halved grid still covers every CU (config #3's 128 groups keep one group per block)
#ifdef MPPI_AB_ARMS
  if (PREC == MPPI_PREC_BF16 && fc_wide() && (a.Kp >> 4) % 2 == 0 && total_groups >= 2 * 256)
    return launch_fc_wide(ARCH, COST, a, fa, img_lds, stream);
#endif
  // bf16 and fp32-in-registers: one group per block (bf16: two blocks per CU, each with its own barriers; fp32: one
  // wave per SIMD); the streamed fp32 path: two groups per block when that still spreads the groups over all CUs
  const int gpb = (PREC == MPPI_PREC_FP32 && !f32_regs && total_groups >= 2 * 256 &&
                   img_lds + 2 * L::BYTES <= 160 * 1024) ? 2 : 1;
  fa.groups_per_block = gpb;
  const int grid = (total_groups + gpb - 1) / gpb;
  const size_t lds = (size_t)img_lds + (size_t)gpb * L::BYTES;
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  auto kern = f32_regs ? fc_rollout_kernel_f32<ARCH, COST>
                      : fc_rollout_kernel<ARCH, PREC == MPPI_PREC_BF16X3 ? MPPI_PREC_BF16 : PREC, COST>;
  note_kernel(f32_regs ? "fc_rollout_kernel_f32" : (PREC == MPPI_PREC_FP32 ? "fc_rollout_kernel<fp32>" : "fc_rollout_kernel"));
  // > 64 KiB of dynamic LDS must be opted into per kernel (gfx950 has 160 KiB per CU).
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * kSplit * gpb), lds, stream, a, fa);
  return hipGetLastError();
}

template <int ARCH, int COST>
static hipError_t launch_prec(const SolveArgs& a, const FcArgs& fa, int precision, hipStream_t s) {
  if (precision == MPPI_PREC_BF16) return launch_t<ARCH, MPPI_PREC_BF16, COST>(a, fa, fa.lds_bytes, s);
  if (precision == MPPI_PREC_BF16X3) return launch_t<ARCH, MPPI_PREC_BF16X3, COST>(a, fa, 0, s);
  return launch_t<ARCH, MPPI_PREC_FP32, COST>(a, fa, 0, s);
}

template <int ARCH>
static hipError_t launch_cost(const SolveArgs& a, const FcArgs& fa, int precision, hipStream_t s) {
  switch (a.cost_kind) {
    case MPPI_COST_HUMANOID_V3: return launch_prec<ARCH, MPPI_COST_HUMANOID_V3>(a, fa, precision, s);
    case MPPI_COST_HUMANOID_V1: return launch_prec<ARCH, MPPI_COST_HUMANOID_V1>(a, fa, precision, s);
    case MPPI_COST_QUAD_JL: return launch_prec<ARCH, MPPI_COST_QUAD_JL>(a, fa, precision, s);
    case MPPI_COST_QUAD_EST: return launch_prec<ARCH, MPPI_COST_QUAD_EST>(a, fa, precision, s);
    case MPPI_COST_CARTPOLE_EST: return launch_prec<ARCH, MPPI_COST_CARTPOLE_EST>(a, fa, precision, s);
    case MPPI_COST_CARTPOLE: return launch_prec<ARCH, MPPI_COST_CARTPOLE>(a, fa, precision, s);
    default: return hipErrorInvalidValue;
  }
}

#ifdef MPPI_AB_ARMS  // ab/kernels_fc_pipe.hip: the layer-pipelined CA rollout (an A/B arm: MPPI_FC_PIPE=1 forces it)
bool fc_pipe_wanted(const SolveArgs& a);
hipError_t launch_fc_pipe(const SolveArgs& a, FcArgs fa, hipStream_t stream);
#endif

// kernels_fc_wave.hip: the per-wave CA rollout (weights in LDS, every layer of NS sample tiles in one wave; batches
// with >= 2 tile pairs per wave slot; MPPI_FC_WAVE=0/1/2 forces); fc_wave_ns: 0 = not this kernel, else NS
int fc_wave_ns(const SolveArgs& a, const FcArgs& fa);
hipError_t launch_fc_wave(const SolveArgs& a, const FcArgs& fa, int ns, hipStream_t stream);
// ... and its MLP (hidden 128 x 2) counterpart (MPPI_FC_WAVE=0/1/2 forces it too)
int fc_wave_mlp_ns(const SolveArgs& a, const FcArgs& fa);
hipError_t launch_fc_wave_mlp(const SolveArgs& a, const FcArgs& fa, int ns, hipStream_t stream);
// ... and the split-bf16 per-wave CA rollout (fc_wave32_x3_kernel; batches with >= 4 wave-tiles of 32 per CU;
// MPPI_X3_WAVE=0 keeps the M-split split-bf16 kernels)
bool fc_wave_x3_wanted(const SolveArgs& a, const FcArgs& fa);
hipError_t launch_fc_wave_x3(const SolveArgs& a, const FcArgs& fa, hipStream_t stream);
// kernels_fc_x3m.hip: the split per-wave MLP rollout (MPPI_X3M=0/1 forces it off / on; default by batch size)
bool fc_wave_mlp_x3_wanted(const SolveArgs& a, const FcArgs& fa);
hipError_t launch_fc_wave_mlp_x3(const SolveArgs& a, const FcArgs& fa, hipStream_t stream);
// kernels_fc_x3mp.hip: the same at 32 samples per wave on 32x32x16 MFMAs (MPPI_X3M32=0/1; default by batch size)
bool fc_wave32_mlp_x3_wanted(const SolveArgs& a, const FcArgs& fa);
hipError_t launch_fc_wave32_mlp_x3(const SolveArgs& a, const FcArgs& fa, hipStream_t stream);
hipError_t launch_fc_wave_x3p(const SolveArgs& a, const FcArgs& fa, hipStream_t stream);  // two waves per SIMD
// kernels_fc_x3d.hip: the split M-split CA rollout with two groups per block at two waves per SIMD (the few-tiles
// shards; MPPI_X3D=0 keeps fc_rollout_kernel_x3w)
bool fc_x3d_wanted(const SolveArgs& a, const FcArgs& fa);
hipError_t launch_fc_x3d(const SolveArgs& a, const FcArgs& fa, hipStream_t stream);
// kernels_fc_x3h.hip: its fp16 form at one group per block, two blocks per CU (MPPI_X3H=0 keeps x3d)
bool fc_x3h_wanted(const SolveArgs& a, const FcArgs& fa);
hipError_t launch_fc_x3h(const SolveArgs& a, const FcArgs& fa, hipStream_t stream);

// kernels_fc_ca.hip
hipError_t launch_fc_ca(const SolveArgs& a, const FcArgs& fa, int precision, hipStream_t stream);
#ifdef MPPI_STAMPS
int fc_ca_stamps(unsigned long long* out, int reset);
#endif

}  // namespace mppi
