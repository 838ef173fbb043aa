// Layer-pipelined rollout of the folded humanoid CrossAttention surrogate (bf16; BASELINE config #4 with many solves
// per GPU).  Same arithmetic as fc_rollout_kernel<kArchCA> (fc_rollout.h: folded weights, bf16 activations, fp32
// accumulation and fp32 state), a different split of the work:
//
//   * a block = 4 waves = 3 pipeline stages over 3 sample tiles (16 samples each) in flight:
//       A  (one wave):  layer 0 (all 256 rows) + the folded LayerNorm (sum h^2 over the whole row in one wave: no
//                       cross-wave statistics exchange), ReLU -> act0
//       B1, B2:         layer 1, output tiles 0..3 / 4..7 -> act1; the control part of the running cost
//       C  (one wave):  the last layer (all 4 state tiles), x += dx (fp32), x (bf16) -> the tile's layer-0 operand,
//                       the state part of the running cost (4-step LDS ring)
//   * tick k: A works on tile k mod 3, B on tile (k-1) mod 3, C on tile (k-2) mod 3; every stage reads what another
//     stage wrote in tick k-1, so ONE barrier per tick (fc_rollout_kernel: 4 per 16-sample step) and a tile
//     advances one horizon step every 3 ticks;
//   * each wave keeps only its own stage's A fragments in registers (A: 32, B: 32, C: 16), loaded once;
//   * layer 0's bias rides in the MFMA (the image's hi / lo pair in the pad state slots 28, 29, which hold 1.0 here);
//   * two blocks per CU with the roles rotated by block parity, so a SIMD pairs one block's A with the other's B.
// Forced with MPPI_FC_PIPE=1 (an A/B arm since the per-wave kernel, kernels_fc_wave.hip, beats it on the batches where
// it used to be chosen).
#include "fc_rollout.h"

#include <cstdlib>

namespace mppi {

constexpr int kPipeRing = 4;  // C's cost ring: 4 steps x 16 samples = one (step, sample) per lane of the wave

template <int COST>
struct PipeLay {
  using CC = CostChunks<kArchCA, COST>;
  static constexpr int XB = 0;                     // [3 tiles][2 k-steps][64 lanes][16 B]: x as layer-0 B operand
  static constexpr int ACT0 = XB + 3 * 2048;       // [2 parity][8 k-steps][1 KB]
  static constexpr int ACT1 = ACT0 + 2 * 8192;     // [2 parity][4 k-steps][1 KB]
  static constexpr int VEC = ACT1 + 2 * 4096;      // beta'[256], bx[64] (f32)
  static constexpr int HIST = VEC + (256 + 64) * 4;  // [3 tiles][kPipeRing][16][HS] f32
  static constexpr int XS = HIST + 3 * kPipeRing * 16 * CC::HS * 4;  // [3 tiles][4 m-tiles][64 lanes] f32x4: x (C)
  static constexpr int CQ = XS + 3 * 4 * 64 * 16;  // [2 B waves][3 tiles][64 lanes] f32: control-cost partials
  static constexpr int BYTES = CQ + 2 * 3 * 64 * 4;
  static_assert(BYTES <= 80 * 1024, "two blocks per CU");
};

template <int COST>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void fc_pipe_kernel(SolveArgs a,
                                                                                              FcArgs net) {
  using A = Arch<kArchCA>;
  using PR = P<MPPI_PREC_BF16>;
  using Bop = PR::Bop;
  using Wt = PR::Wt;
  using Y = PipeLay<COST>;
  using CC = typename Y::CC;
  static_assert(A::MT0 == 16 && A::MT1 == 8 && A::IN_T == 4 && A::NL == 3, "folded humanoid CA shape");
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const KClock kc = kclock_begin(a);
  if (blockIdx.x == 0 && threadIdx.x == 0) *a.status = 0u;
  const int lane = threadIdx.x & 63, g = lane >> 4, n = lane & 15;
  const int wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int role = (wib + 2 * (blockIdx.x & 1)) & 3;  // 0: A, 1: B1, 2: B2, 3: C
  const int H = a.H;
  const int gps = a.Kp >> 4, total = a.B * gps;
  constexpr int NTICK = 3;  // ticks per round; rounds r = 0..H: 3H + 3 ticks (the last ones partly idle)

  // the block's 3 tiles (tile t = global 16-sample group 3 blockIdx + t; past the end: a clamped copy, no writes)
  int tb[3], tk[3];
  bool live[3];
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    const int T = 3 * blockIdx.x + t;
    live[t] = T < total;
    const int Tc = live[t] ? T : total - 1;
    tb[t] = Tc / gps;
    tk[t] = (Tc - tb[t] * gps) * 16;  // first sample of the tile
  }
  float* vec = reinterpret_cast<float*>(lds + Y::VEC);
  for (int i = threadIdx.x; i < 256; i += 256) {  // beta', bx
    vec[i] = reinterpret_cast<const float*>(net.img + net.lnb_off)[i];
    if (i < 64) vec[256 + i] = reinterpret_cast<const float*>(net.img + net.b_off[2])[i];
  }
  auto state_src = [&](int sl) { return sl < 32 ? (sl < net.qp ? sl : -1) : (sl - 32 < net.qv ? net.qp + sl - 32 : -1); };
  // the layer-0 operand's value of state slot sl: the state, 1.0 in the two slots that carry b0 (kCaBiasSlotHi/Lo:
  // the image's bf16 hi / lo pair, so the MFMA computes W0 x + b0), 0 in the other pads
  auto slot_val = [&](const float* x0, int sl) {
    const int src = state_src(sl);
    return src >= 0 ? x0[src] : ((sl == kCaBiasSlotHi || sl == kCaBiasSlotLo) ? 1.0f : 0.0f);
  };
  if (wib == 0) {
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      const float* x0 = a.x0 + (long)tb[t] * a.nx;
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        f32x4 v;
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = slot_val(x0, 16 * mt + 4 * g + r);
        PR::put_tile(lds + Y::XB + t * 2048, mt, lane, v);
      }
    }
  }
  auto Wg = [&](int l) { return reinterpret_cast<const Wt*>(net.img + net.w_off[l]); };

  if (role == 0) {
    // ================================================================== A: layer 0 (all 256 rows) + LayerNorm -> act0
    Wt fr[16][2];
    load_frags<MPPI_PREC_BF16>(fr, Wg(0), 0, lane);
    __syncthreads();
    for (int r = 0; r <= H; ++r) {
#pragma unroll
      for (int ph = 0; ph < NTICK; ++ph) {
        if (r < H) {  // tile ph, step r
          const char* xb = lds + Y::XB + ph * 2048;
          const Bop b0 = PR::get_ks(xb, 0, lane), b1 = PR::get_ks(xb, 1, lane);
          f32x4 be[16];  // beta': the first 8 tiles read under the MFMAs, the rest 8 tiles ahead of their use
#pragma unroll
          for (int i = 0; i < 8; ++i) be[i] = *reinterpret_cast<const f32x4*>(vec + 16 * i + 4 * g);
          f32x4 h[16];
#pragma unroll
          for (int i = 0; i < 16; ++i) h[i] = PR::mma(fr[i][0], b0, f32x4{0.0f, 0.0f, 0.0f, 0.0f});  // b0: slots 28/29
#pragma unroll
          for (int i = 0; i < 16; ++i) h[i] = PR::mma(fr[i][1], b1, h[i]);
          // folded LayerNorm (rows centred on the host): var = mean(h^2) over the 256 features of sample n
          f32x2 q2[4] = {f32x2{0.0f, 0.0f}, f32x2{0.0f, 0.0f}, f32x2{0.0f, 0.0f}, f32x2{0.0f, 0.0f}};
#pragma unroll
          for (int i = 0; i < 16; ++i) {  // four accumulation chains, then a tree
            const f32x2 lo = {h[i][0], h[i][1]}, hi = {h[i][2], h[i][3]};
            q2[i & 3] = hi * hi + (lo * lo + q2[i & 3]);
          }
          const f32x2 qs = (q2[0] + q2[1]) + (q2[2] + q2[3]);
          const float q = group_sum(qs.x + qs.y);
          const float rstd = __builtin_amdgcn_rsqf(q * (1.0f / 256.0f) + 1e-5f);
          const f32x2 r2 = {rstd, rstd};
          char* out = lds + Y::ACT0 + ((r + ph) & 1) * 8192;  // tick parity (3r + ph) & 1
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            if (i + 8 < 16) be[i + 8] = *reinterpret_cast<const f32x4*>(vec + 16 * (i + 8) + 4 * g);
            const f32x2 ylo = f32x2{h[i][0], h[i][1]} * r2 + f32x2{be[i][0], be[i][1]};
            const f32x2 yhi = f32x2{h[i][2], h[i][3]} * r2 + f32x2{be[i][2], be[i][3]};
            PR::put_tile_relu(out, i, lane, f32x4{ylo.x, ylo.y, yhi.x, yhi.y});
          }
        }
        __syncthreads();
      }
    }
    __syncthreads();  // (B's control-cost partials -> C)
  } else if (role <= 2) {
    // ================================================================== B: layer 1 (half of the rows) -> act1, and
    // the control part of the running cost of the same tile and step: B1 control slots 4g..4g+3, B2 16+4g..16+4g+3
    const int hb = role - 1, m0 = 4 * hb;
    Wt fr[4][8];
    load_frags<MPPI_PREC_BF16>(fr, Wg(1), m0, lane);
    f32x4 bias1[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
      bias1[i] = *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(net.img + net.b_off[1]) +
                                                 16 * (m0 + i) + 4 * g);
    const float cl = a.ctrl_clamp > 0.0f ? a.ctrl_clamp : INFINITY;
    int uoff[4], eoff[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int us = 16 * hb + 4 * g + j;
      uoff[j] = us < a.nu ? us * a.H * 4 : 0x7FFFFFF0;  // pad slots past the descriptor range read 0
      eoff[j] = us < a.nu ? (us * a.H * a.Kp + n) * 4 : 0x7FFFFFF0;
    }
    auto load_u = [&](int t, int step, float (&u)[4]) {  // U + eps of (tile t, step): raw buffer loads
      const auto rU = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.U) + (long)tb[t] * a.nu * a.H, 0,
                                                        a.nu * a.H * 4, 0x00020000);
      const auto rE = __builtin_amdgcn_make_buffer_rsrc(a.noise + (long)tb[t] * a.nu * a.H * a.Kp, 0,
                                                        a.nu * a.H * a.Kp * 4, 0x00020000);
      const int su = step * 4, se = (step * a.Kp + tk[t]) * 4;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        u[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rU, uoff[j], su, 0)) +
               __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rE, eoff[j], se, 0));
    };
    float upf[3][4];  // the tile's controls of its next step, prefetched one round ahead
#pragma unroll
    for (int t = 0; t < 3; ++t) load_u(t, 0, upf[t]);
    float cost[3] = {0.0f, 0.0f, 0.0f};
    __syncthreads();
    for (int r = 0; r <= H; ++r) {
#pragma unroll
      for (int ph = 0; ph < NTICK; ++ph) {
        constexpr int kTile[3] = {2, 0, 1};  // tile (k - 1) mod 3 at phase ph
        const int t = kTile[ph];
        const int s = ph == 0 ? r - 1 : r;
        if (s >= 0 && s < H) {
          {
            float usq = 0.0f;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const float u = __builtin_amdgcn_fmed3f(upf[t][j], -cl, cl);
              usq = fmaf(u, u, usq);
            }
            const float u0c = __builtin_amdgcn_fmed3f(upf[t][0], -cl, cl);
            cost[t] += ctrl_term_t<COST>((hb == 0 && g == 0) ? u0c : 0.0f, usq);  // control 0: B1, lane group 0
            load_u(t, s + 1 < H ? s + 1 : s, upf[t]);
          }
          const char* in = lds + Y::ACT0 + ((r + ph + 1) & 1) * 8192;  // parity of tick k - 1
          Bop bin[8];
#pragma unroll
          for (int ks = 0; ks < 8; ++ks) bin[ks] = PR::get_ks(in, ks, lane);
          f32x4 h[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) h[i] = bias1[i];
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int kk = 0; kk < 8; ++kk)
#pragma unroll
            for (int i = 0; i < 4; ++i) h[i] = PR::mma(fr[i][kk], bin[kk], h[i]);
          char* out = lds + Y::ACT1 + ((r + ph) & 1) * 4096;
#pragma unroll
          for (int i = 0; i < 4; ++i) PR::put_tile_relu(out, m0 + i, lane, h[i]);
        }
        __syncthreads();
      }
    }
    float* cq = reinterpret_cast<float*>(lds + Y::CQ) + hb * 3 * 64 + lane;
#pragma unroll
    for (int t = 0; t < 3; ++t) cq[t * 64] = cost[t];
    __syncthreads();
  } else {
    // ================================================================== C: last layer, state, state part of the cost
    Wt fr[4][4];
    load_frags<MPPI_PREC_BF16>(fr, Wg(2), 0, lane);
    // the fp32 state of the 3 tiles in the accumulator layout, this lane's 16 values per tile, in LDS
    f32x4* xs = reinterpret_cast<f32x4*>(lds + Y::XS) + lane;
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      const float* x0 = a.x0 + (long)tb[t] * a.nx;
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        f32x4 v;
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) v[rr] = slot_val(x0, 16 * mt + 4 * g + rr);  // 1.0 in the b0 slots: dx = 0
        xs[(t * 4 + mt) * 64] = v;
      }
    }
    float cx[3][MPPI_CTX_MAX];  // each tile's solve's cost context (block-uniform: scalar registers)
#pragma unroll
    for (int t = 0; t < 3; ++t)
#pragma unroll
      for (int i = 0; i < MPPI_CTX_MAX; ++i)
        cx[t][i] = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(
                                                 int, a.ctx ? a.ctx[(long)tb[t] * MPPI_CTX_MAX + i] : a.ctx_default[i])));
    // ring chunks this lane stores: state tile mt, lane group g (CostChunks: only the slots the cost reads)
    int chunk[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      chunk[mt] = -1;
#pragma unroll
      for (int e = 0; e < 16; ++e)
        if (e == 4 * mt + g) chunk[mt] = CC::chunk(e / 4, e % 4);
    }
    float cost[3] = {0.0f, 0.0f, 0.0f};
    auto ring_cost = [&](int t, int slot, int t1) {
      const float* hist = reinterpret_cast<const float*>(lds + Y::HIST) + (t * kPipeRing + slot) * 16 * CC::HS;
      f32x4 ch[CC::NCH];
#pragma unroll
      for (int c = 0; c < CC::NCH; ++c) ch[c] = *reinterpret_cast<const f32x4*>(hist + n * CC::HS + 4 * c);
      constexpr CostIdx ci = cost_idx(COST);
      float v[kCostMaxIdx];
#pragma unroll
      for (int i = 0; i < ci.n; ++i) {
        const int sl = CC::slot(ci.idx[i]);
        v[i] = ch[CC::chunk(sl / 16, (sl % 16) / 4)][sl % 4];
      }
      return cost_eval_t<COST>(v, 0.0f, 0.0f, cx[t], t1);
    };
    __syncthreads();
    for (int r = 0; r <= H; ++r) {
#pragma unroll
      for (int ph = 0; ph < NTICK; ++ph) {
        constexpr int kTile[3] = {1, 2, 0};  // tile (k - 2) mod 3 at phase ph
        const int t = kTile[ph];
        const int s = ph == 2 ? r : r - 1;
        if (s >= 0 && s < H) {
          const char* in = lds + Y::ACT1 + ((r + ph + 1) & 1) * 4096;
          Bop bin[4];
#pragma unroll
          for (int ks = 0; ks < 4; ++ks) bin[ks] = PR::get_ks(in, ks, lane);
          f32x4 xn[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) xn[i] = *reinterpret_cast<const f32x4*>(vec + 256 + 16 * i + 4 * g);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int kk = 0; kk < 4; ++kk)
#pragma unroll
            for (int i = 0; i < 4; ++i) xn[i] = PR::mma(fr[i][kk], bin[kk], xn[i]);
          float* hist = reinterpret_cast<float*>(lds + Y::HIST) + (t * kPipeRing + s % kPipeRing) * 16 * CC::HS;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            xn[i] += xs[(t * 4 + i) * 64];
            xs[(t * 4 + i) * 64] = xn[i];
            PR::put_tile(lds + Y::XB + t * 2048, i, lane, xn[i]);
            if (chunk[i] >= 0) *reinterpret_cast<f32x4*>(hist + n * CC::HS + 4 * chunk[i]) = xn[i];
          }
          // ring full (or horizon done): lane group g evaluates the state cost of step s - s % 4 + g of sample n
          if ((s + 1) % kPipeRing == 0 || s + 1 == H) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the ring rows this wave just wrote
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const int ts = s - s % kPipeRing + g;
            if (ts <= s) cost[t] += ring_cost(t, g, ts + 1);
          }
        }
        __syncthreads();
      }
    }
    __syncthreads();  // B's control-cost partials
    const float* cq = reinterpret_cast<const float*>(lds + Y::CQ) + lane;
    // terminal cost on x_H (ring slot of step H - 1), then the per-sample sums over the 4 lane groups
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      if (a.terminal_weight != 0.0f && g == 0) cost[t] += a.terminal_weight * ring_cost(t, (H - 1) % kPipeRing, H);
      cost[t] += cq[t * 64] + cq[(3 + t) * 64];
      cost[t] = group_sum(cost[t]);
      const int k = tk[t] + n;
      if (g == 0 && live[t] && k < a.K) a.costs[(long)tb[t] * a.Kp + k] = isfinite(cost[t]) ? cost[t] : INFINITY;
      if (a.xout && live[t] && tk[t] == 0 && n == 0) {  // env step: final state of sample 0 of the solve
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int rr = 0; rr < 4; ++rr) {
            const int src = state_src(16 * i + 4 * g + rr);
            if (src >= 0) a.xout[(long)tb[t] * a.nx + src] = xs[(t * 4 + i) * 64][rr];
          }
      }
    }
  }
  __syncthreads();
  kclock_record(a, kc);
}

// MPPI_FC_PIPE=1 forces this kernel (read per launch, so a test can switch it).  It used to be chosen by itself for
// batches that fill whole rounds of 2 blocks x 3 tiles per CU (48 solves of config #4: 423.6 vs 446.5 us for the M-split
// kernel); the per-wave kernel (kernels_fc_wave.hip) is faster on every such batch (48 solves: 330 us; 24: 190 vs 212
// us; scripts/gpu_sweep_wave.sh), so it is now an A/B arm only.
static int fc_pipe_mode() {
  const char* e = std::getenv("MPPI_FC_PIPE");
  return e ? std::atoi(e) : -1;
}

bool fc_pipe_wanted(const SolveArgs& a) {
  (void)a;
  return fc_pipe_mode() == 1;
}

hipError_t launch_fc_pipe(const SolveArgs& a, FcArgs fa, hipStream_t stream) {
  const int tiles = a.B * (a.Kp >> 4);
  const int grid = (tiles + 2) / 3;
  auto go = [&](auto kern, int bytes) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(256), bytes, stream, a, fa);
    return hipGetLastError();
  };
  if (a.cost_kind == MPPI_COST_HUMANOID_V1) return go(fc_pipe_kernel<MPPI_COST_HUMANOID_V1>, PipeLay<MPPI_COST_HUMANOID_V1>::BYTES);
  return go(fc_pipe_kernel<MPPI_COST_HUMANOID_V3>, PipeLay<MPPI_COST_HUMANOID_V3>::BYTES);
}

}  // namespace mppi
