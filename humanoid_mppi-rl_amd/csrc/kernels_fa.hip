// FeatureAttentionStatePredictor rollout (learning/model.py:48-153): x_{t+1} = x_t + net([x_t, u_t]) with every
// state/control scalar a token, for every (solve, sample), the H loop inside the kernel.  Replaces the per-step
// torch launch chain of src/cartpole_mppi_estimator.py:84-119 (FA hidden 64) and
// src/quadruped_mppi_estimator.py:67-78 (FA hidden 512).
//
// Mapping (DESIGN.md "FA rollout"):
//   * a workgroup owns G = floor(16 NT / L) whole samples of one solve (NT = 1, 2 or 4 token n-tiles, fa_nt):
//     token rows r = s*L + i (L = nx + nu tokens, rows >= G*L are padding) for the whole horizon.  The residual
//     stream lives in registers as MFMA accumulators: wave w owns feature m-tiles [w*MPW, (w+1)*MPW) x the NT
//     token n-tiles (D layout: lane holds features 16mt + 4g + r of token 16nt + (lane & 15)).
//   * every Linear is  out[feature][token] = W * act^T  with W the A operand (pre-packed 16x32 fragments streamed
//     from L2/MALL through A-fragment pipelines, shared by all workgroups) and act the B operand read from an LDS
//     [token][feature] buffer.  LayerNorm outputs, Q/K/V, the attention output and FFN hidden chunks pass through
//     LDS; the out-proj and the second FFN GEMM accumulate straight into the residual registers (attention is
//     processed a chunk of whole heads at a time, the FFN a chunk of hidden rows at a time: K-split sums).
//   * attention over the L tokens of a sample: D >= 128 (bf16) on MFMA (S^T = K Q^T, softmax, P V through LDS);
//     small nets on VALU, one task per (head, sample, query, 4 output features) with an online softmax.
//   * LayerNorm statistics: per-wave (mean, M2) over the wave's features, combined across waves (Chan et al.).
//   * the scalar feature encoding LayerNorm(w v + b) uses closed-form moments (host-computed in double).
//   * D = 64: the image's fp32 vectors (encoding, pos, LayerNorm, biases, output row) are staged in LDS once.
//   * a row scalar array XU[r] holds each token's input value (state or perturbed control); the output layer
//     updates the state rows in place; one thread per sample evaluates the running cost.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "costs.h"
#include "mppi_internal.h"

namespace mppi {

// Diagnostic build only (-DMPPI_STAMPS): per-phase s_memtime sums of the horizon loop, accumulated over all waves
// into g_fa_stamps (read by mppi_debug_fa_stamps). The shipped kernel contains none of this.
#ifdef MPPI_STAMPS
constexpr int kNumFaStamps = 8;
__device__ unsigned long long g_fa_stamps[kNumFaStamps];
#define FA_STAMP(i)                                                            \
  do {                                                                         \
    __builtin_amdgcn_sched_barrier(0);                                         \
    unsigned long long t_;                                                     \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory"); \
    __builtin_amdgcn_sched_barrier(0);                                         \
    st_[i] += t_ - tprev_;                                                     \
    tprev_ = t_;                                                               \
  } while (0)
#else
#define FA_STAMP(i) \
  do {              \
  } while (0)
#endif

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;

struct FaArgs {
  const char* img;
  int img_bytes;
  int D, L, G, nx, nu, nlayers;
  int we, be, ge, bte, pos, wout;
  int ln1g[kFaMaxLayers], ln1b[kFaMaxLayers], bqkv[kFaMaxLayers], bo[kFaMaxLayers];
  int ln2g[kFaMaxLayers], ln2b[kFaMaxLayers], b1[kFaMaxLayers], b2[kFaMaxLayers];
  int wqkv[kFaMaxLayers], wo[kFaMaxLayers], w1[kFaMaxLayers], w2[kFaMaxLayers];
  float enc_mw, enc_mb, enc_vw, enc_cwb, enc_vb, b_out;
  int vec_lds;  // bytes of the image's fp32-vector prefix staged in LDS (0: read from L2)
  int s_wqkv[kFaMaxLayers], s_w1[kFaMaxLayers], s_w2[kFaMaxLayers];  // fa_small_kernel image
  int s_c1, s_c2;  // fa_small_kernel: centred, gamma-scaled encoding weight / bias vectors
  int s_bqkv[kFaMaxLayers], s_b1[kFaMaxLayers];  // fa_small_kernel: biases of the LayerNorm-folded GEMMs
};

// ------------------------------------------------------------------------------------------- precision traits
// One k-block = 32 input features.  bf16: one v_mfma_f32_16x16x32_bf16, lane group g holds features
// 32kb + 8g + [0,8).  fp32: eight v_mfma_f32_16x16x4f32, lane group g holds features 32kb + 16h + 4g + [0,4)
// (h = 0, 1; MFMA m of half h consumes element m).  A fragments are packed in the same order (mppi_nets.cpp).
template <int PREC>
struct FP;
template <>
struct FP<MPPI_PREC_BF16> {
  static constexpr int E = 2;        // bytes per activation element in LDS
  static constexpr int FRAG = 1024;  // bytes per packed 16x32 A fragment
  using Frag = bf16x8;
  __device__ static Frag ldA(const char* frag, int lane) { return *reinterpret_cast<const bf16x8*>(frag + lane * 16); }
  __device__ static Frag ldB(const char* row, int kb, int g) {
    return *reinterpret_cast<const bf16x8*>(row + (32 * kb + 8 * g) * 2);
  }
  __device__ static f32x4 mma(const Frag& a, const Frag& b, const f32x4& c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
  __device__ static void st4(char* p, const f32x4& v) {
    bf16x4 h = {(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
    *reinterpret_cast<bf16x4*>(p) = h;
  }
  __device__ static f32x4 ld4(const char* p) {
    const bf16x4 h = *reinterpret_cast<const bf16x4*>(p);
    return f32x4{(float)h[0], (float)h[1], (float)h[2], (float)h[3]};
  }
};
template <>
struct FP<MPPI_PREC_FP32> {
  static constexpr int E = 4;
  static constexpr int FRAG = 2048;
  struct Frag {
    f32x4 lo, hi;
  };
  __device__ static Frag ldA(const char* frag, int lane) {
    const f32x4* p = reinterpret_cast<const f32x4*>(frag + lane * 32);
    return Frag{p[0], p[1]};
  }
  __device__ static Frag ldB(const char* row, int kb, int g) {
    return Frag{*reinterpret_cast<const f32x4*>(row + (32 * kb + 4 * g) * 4),
                *reinterpret_cast<const f32x4*>(row + (32 * kb + 16 + 4 * g) * 4)};
  }
  __device__ static f32x4 mma(const Frag& a, const Frag& b, f32x4 c) {
#pragma unroll
    for (int m = 0; m < 4; ++m) c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.lo[m], b.lo[m], c, 0, 0, 0);
#pragma unroll
    for (int m = 0; m < 4; ++m) c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.hi[m], b.hi[m], c, 0, 0, 0);
    return c;
  }
  __device__ static void st4(char* p, const f32x4& v) { *reinterpret_cast<f32x4*>(p) = v; }
  __device__ static f32x4 ld4(const char* p) { return *reinterpret_cast<const f32x4*>(p); }
};

// sum over the 4 lane groups (lanes n, n+16, n+32, n+48), result in every lane
__device__ __forceinline__ float fa_group_sum(float v) {
  auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  const float s = __uint_as_float(p[0]) + __uint_as_float(p[1]);
  auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(s), __float_as_uint(s), false, false);
  return __uint_as_float(q[0]) + __uint_as_float(q[1]);
}

// One attention MFMA step over 32 (or, for 16-wide heads, 16) of the contraction index: A rows at `a` and B rows
// at `b` are [row][k] bf16 with the k slice contiguous; lane (m | n = lane & 15, g = lane >> 4) reads its row's
// 8 (or 4) k values.  bf16 only (the fp32 parity mode keeps the VALU attention).
template <int KW>
__device__ __forceinline__ f32x4 att_mma(const char* a, const char* b, int g, f32x4 c) {
  if constexpr (KW == 32) {
    const bf16x8 av = *reinterpret_cast<const bf16x8*>(a + 16 * g), bv = *reinterpret_cast<const bf16x8*>(b + 16 * g);
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, c, 0, 0, 0);
  } else {
    typedef __attribute__((ext_vector_type(4))) short s16x4;
    const s16x4 av = *reinterpret_cast<const s16x4*>(a + 8 * g), bv = *reinterpret_cast<const s16x4*>(b + 8 * g);
    return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(av, bv, c, 0, 0, 0);
  }
}

// max / sum over the 4 lane groups (lanes n, n+16, n+32, n+48), result in every lane
__device__ __forceinline__ float fa_group_max(float v) {
  auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  const float s = fmaxf(__uint_as_float(p[0]), __uint_as_float(p[1]));
  auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(s), __float_as_uint(s), false, false);
  return fmaxf(__uint_as_float(q[0]), __uint_as_float(q[1]));
}

// running cost of one sample from its state row (compile-time gather per kind: no scratch)
template <int KIND>
__device__ __forceinline__ float fa_cost_t(const float* x, float u0, float usq, const float* cx) {
  constexpr CostIdx ci = cost_idx(KIND);
  float v[kCostMaxIdx];
#pragma unroll
  for (int i = 0; i < ci.n; ++i) v[i] = x[ci.idx[i]];
  return cost_eval_t<KIND>(v, u0, usq, cx);
}
__device__ __forceinline__ float fa_cost(int kind, const float* x, float u0, float usq, const float* cx) {
  switch (kind) {
    case MPPI_COST_CARTPOLE: return fa_cost_t<MPPI_COST_CARTPOLE>(x, u0, usq, cx);
    case MPPI_COST_CARTPOLE_EST: return fa_cost_t<MPPI_COST_CARTPOLE_EST>(x, u0, usq, cx);
    case MPPI_COST_HUMANOID_V3: return fa_cost_t<MPPI_COST_HUMANOID_V3>(x, u0, usq, cx);
    case MPPI_COST_QUAD_JL: return fa_cost_t<MPPI_COST_QUAD_JL>(x, u0, usq, cx);
    default: return fa_cost_t<MPPI_COST_QUAD_EST>(x, u0, usq, cx);
  }
}

// A-fragment pipeline: the first PF k-blocks of a GEMM, loaded ahead (possibly across a barrier / VALU phase:
// in-flight global loads are not drained by the workgroup barrier here, which waits on lgkmcnt only).
template <int PREC, int MT, int PF>
struct APipe {
  typename FP<PREC>::Frag a[PF][MT];
};

template <int PREC, int MT, int KB, int PF>
__device__ __forceinline__ void pipe_prime(APipe<PREC, MT, PF>& p, const char* __restrict__ W, int mt0, int lane) {
  using F = FP<PREC>;
#pragma unroll
  for (int s = 0; s < (PF < KB ? PF : KB); ++s)
#pragma unroll
    for (int i = 0; i < MT; ++i) p.a[s][i] = F::ldA(W + ((mt0 + i) * KB + s) * F::FRAG, lane);
}

// acc[i][nt] += W(m-tile mt0 + i) * X^T over KB k-blocks from a primed pipe, refilling it PF k-blocks ahead;
// next() runs as soon as this GEMM's last A load is issued (it primes the following GEMM's pipe).
template <int PREC, int MT, int KB, int PF, int NT, class Next>
__device__ __forceinline__ void fa_gemm_p(f32x4 (&acc)[MT][NT], APipe<PREC, MT, PF>& p, const char* __restrict__ W,
                                          int mt0, const char* X, int xs, int lane, Next&& next) {
  using F = FP<PREC>;
  const int g = lane >> 4, n = lane & 15;
  if constexpr (KB <= PF) next();
#pragma unroll
  for (int kb = 0; kb < KB; ++kb) {
    typename F::Frag b[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) b[nt] = F::ldB(X + (16 * nt + n) * xs, kb, g);
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) acc[i][nt] = F::mma(p.a[kb % PF][i], b[nt], acc[i][nt]);
    if (kb + PF < KB) {
#pragma unroll
      for (int i = 0; i < MT; ++i) p.a[kb % PF][i] = F::ldA(W + ((mt0 + i) * KB + kb + PF) * F::FRAG, lane);
      if (kb + PF == KB - 1) next();
    }
  }
}

template <int D, int PREC, int NT>
struct FaLay {
  static constexpr int R = 16 * NT;  // token rows per workgroup
  static constexpr int NW = fa_nw(D);
  static constexpr int CW = fa_cw(D);  // attention chunk width (whole heads)
  static constexpr int FC = fa_fc(D);  // FFN hidden chunk
  static constexpr int E = FP<PREC>::E;
  static constexpr int XN_S = D * E + 16;  // row strides (+16 B: consecutive rows start 4 banks apart)
  static constexpr int CW_S = CW * E + 16;
  static constexpr int HID_S = FC * E + 16;
  static constexpr int XN = 0;
  // Q | K | V | O | P; HID aliases it.  fp32 (VALU attention): V [R][CW], P fp32 [HC][R][L].  bf16 (MFMA
  // attention): V transposed [CW][R] (rows VT_S), P bf16 [HC][R][R] (rows P_S).
  static constexpr bool MA = PREC == MPPI_PREC_BF16 && D >= 128;  // small nets (cartpole L=5): VALU is faster
  static constexpr int VT_S = R * 2 + 16, P_S = R * 2 + 16;
  static constexpr int VB = MA ? (CW * VT_S > R * CW_S ? CW * VT_S : R * CW_S) : R * CW_S;
  static constexpr int ATT = XN + R * XN_S;
  static constexpr int Q = ATT, K = Q + R * CW_S, V = K + R * CW_S, O = V + VB;
  static constexpr int P = O + R * CW_S;
  static constexpr int HC = CW / (D / kFaHeads);
  __host__ __device__ static constexpr int att_bytes(int L) {
    return 3 * R * CW_S + VB + (MA ? HC * R * P_S : HC * R * L * 4);
  }
  __host__ __device__ static constexpr int small(int L) {
    return ATT + (att_bytes(L) > R * HID_S ? att_bytes(L) : R * HID_S);
  }
  // small region: ST [NW][64] float2 | OUTP [NW][64] float | XU [64] float
  __host__ __device__ static constexpr int bytes(int L) { return small(L) + NW * R * 12 + R * 4; }
};

template <int D, int PREC, int NT>
__global__ __launch_bounds__(64 * fa_nw(D)) void fa_rollout_kernel(SolveArgs a, FaArgs f) {
  using F = FP<PREC>;
  using Y = FaLay<D, PREC, NT>;
  constexpr int R = Y::R;  // token rows of this workgroup (NT n-tiles)
  constexpr int NW = Y::NW, NTH = 64 * NW;  // threads
  constexpr int HD = D / kFaHeads, CW = Y::CW, HC = Y::HC, NCH = kFaHeads / HC;
  constexpr int FC = Y::FC, NFC = 4 * D / FC;
  constexpr int MPW = D / 16 / NW;           // residual m-tiles per wave
  constexpr int QMT = 3 * CW / 16 / NW;      // Q|K|V m-tiles per wave per chunk
  constexpr int FMT = FC / 16 / NW;          // FFN hidden m-tiles per wave per chunk
  constexpr int E = Y::E;
  // A-fragment pipeline depths (k-blocks in flight) of the Q|K|V / FFN1 GEMMs and of the MPW-tile GEMMs
  // (out-proj, FFN2) that accumulate into the residual.  D = 512 streams 12.6 MB of fragments per sample-step from
  // L2: the deep pipelines (3 / 4 k-blocks) cover the L2 latency although they spill ~150 VGPRs of per-chunk
  // constants outside the inner loops (same-box sweep over PF 2..8 x PFR 1..5: 119 ms at 2/1, 86 ms at 3/4).
  constexpr int PF = D >= 512 ? 3 : 2, PFR = D >= 512 ? 4 : (MPW >= 4 ? 1 : 2);
  static_assert(MPW >= 1 && QMT >= 1 && FMT >= 1 && (3 * CW / 16) % NW == 0, "FA blocking");
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const KClock kc = kclock_begin(a);

  // w: provably wave-uniform (readfirstlane): scalar m-tile offsets, no per-lane copies
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, n = lane & 15,
            w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int L = f.L, G = f.G, nx = f.nx, nu = f.nu;
  const int gps = (a.K + G - 1) / G;  // workgroups per solve
  const int b = blockIdx.x / gps;
  const int k0 = (blockIdx.x - b * gps) * G;
  if (blockIdx.x == 0 && tid == 0) *a.status = 0u;

  char* XN = lds + Y::XN;
  char* Qb = lds + Y::Q;
  char* Kb = lds + Y::K;
  char* Vb = lds + Y::V;
  char* Ob = lds + Y::O;
  float* Pb = reinterpret_cast<float*>(lds + Y::P);
  char* HID = lds + Y::ATT;
  float2* ST = reinterpret_cast<float2*>(lds + Y::small(L));
  float* OUTP = reinterpret_cast<float*>(lds + Y::small(L) + NW * R * 8);
  float* XU = OUTP + NW * R;

  // zero all LDS once: padding rows stay finite
  for (int i = tid; i < Y::bytes(L) / 16; i += NTH) reinterpret_cast<int4*>(lds)[i] = make_int4(0, 0, 0, 0);
  // small nets: the image's fp32 vectors (encoding, pos, LayerNorm gamma/beta, biases, output row; the image
  // prefix before the first packed matrix) staged in LDS once, so no per-step vector load waits on L2
  char* VEC = lds + Y::bytes(L);
  for (int i = tid; i < f.vec_lds / 16; i += NTH) reinterpret_cast<int4*>(VEC)[i] = reinterpret_cast<const int4*>(f.img)[i];
  __syncthreads();

  const char* img = f.img;
  // the image as one buffer resource: fp32 vector loads (LayerNorm gamma/beta, biases, pos) take the vector's byte
  // offset as the scalar soffset and only the lane's 4-float index as voffset, so no per-lane 64-bit address is
  // hoisted out of the horizon loop (D = 512 spilled them to scratch: 119 -> 56 spilled VGPRs, 85.5 -> 83.6 ms)
  const __amdgpu_buffer_rsrc_t wrs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(img), 0, f.img_bytes, 0x00020000);
  auto ld4g = [&](int off, int idx) {  // off: wave-uniform, so the LDS / L2 choice is a scalar branch
    if (D <= 64 && off < f.vec_lds) return *reinterpret_cast<const f32x4*>(VEC + off + idx * 4);
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(wrs, idx * 4, off, 0));
  };

  // per-lane token rows of the 4 n-tiles: token index (for pos) and whether the row is a real token
  int tok[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int r = 16 * nt + n;
    tok[nt] = r < G * L ? r % L : 0;
  }

  // initial state rows
  const float* x0 = a.x0 + (long)b * nx;
  for (int r = tid; r < G * L; r += NTH) {
    const int i = r % L;
    if (i < nx) XU[r] = x0[i];
  }
  // control prefetch: thread tid < G*nu owns (sample s, control j)
  const bool uown = tid < G * nu;
  const int us = uown ? tid / nu : 0, uj = uown ? tid - (tid / nu) * nu : 0;
  const int uk = min(k0 + us, a.Kp - 1);
  const float* Ub = a.U + ((long)b * nu + uj) * a.H;
  const float* eb = a.noise + (((long)b * nu + uj) * a.H) * a.Kp + uk;
  float unext = uown ? Ub[0] + eb[0] : 0.0f;

  // cost thread tid < G owns sample tid
  const bool cown = tid < G;
  const int ck = k0 + tid;
  float cx[MPPI_CTX_MAX];
#pragma unroll
  for (int i = 0; i < MPPI_CTX_MAX; ++i) cx[i] = a.ctx ? a.ctx[(long)b * MPPI_CTX_MAX + i] : a.ctx_default[i];
  float cost = 0.0f, cu0 = 0.0f, cusq = 0.0f;
  auto eval_cost = [&](float u0, float usq) { return fa_cost(a.cost_kind, XU + tid * L, u0, usq, cx); };

  f32x4 res[MPW][NT];  // residual stream, D layout

  // LayerNorm over the D features of every token row -> XN (E-typed), gamma/beta at vector offsets
  auto layer_norm = [&](int goff, int boff) {
    // gamma/beta of the own tiles are loaded up front, so their latency hides behind the statistics and the
    // barrier (stamps, cartpole FA: LayerNorm was 31 % of the step with the loads after the barrier; D = 512:
    // -0.9 % step time in spite of its spills)
    constexpr bool PRE = true;
    f32x4 gpre[PRE ? MPW : 1], bpre[PRE ? MPW : 1];
    if constexpr (PRE) {
#pragma unroll
      for (int i = 0; i < MPW; ++i) {
        const int fcol = 16 * (w * MPW + i) + 4 * g;
        gpre[i] = ld4g(goff, fcol);
        bpre[i] = ld4g(boff, fcol);
      }
    }
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      float s = 0.0f;
#pragma unroll
      for (int i = 0; i < MPW; ++i) s += (res[i][nt][0] + res[i][nt][1]) + (res[i][nt][2] + res[i][nt][3]);
      const float mw = fa_group_sum(s) * (1.0f / (16.0f * MPW));
      float q = 0.0f;
#pragma unroll
      for (int i = 0; i < MPW; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float d = res[i][nt][r] - mw;
          q = fmaf(d, d, q);
        }
      q = fa_group_sum(q);
      if (g == 0) ST[w * R + 16 * nt + n] = make_float2(mw, q);
    }
    __syncthreads();
    float mean[NT], rstd[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int row = 16 * nt + n;
      float m = 0.0f, M2 = 0.0f;
#pragma unroll
      for (int w2 = 0; w2 < NW; ++w2) m += ST[w2 * R + row].x;
      m *= 1.0f / NW;
#pragma unroll
      for (int w2 = 0; w2 < NW; ++w2) {
        const float2 p = ST[w2 * R + row];
        const float d = p.x - m;
        M2 += p.y + (16.0f * MPW) * d * d;
      }
      mean[nt] = m;
      rstd[nt] = 1.0f / sqrtf(M2 * (1.0f / D) + 1e-5f);
    }
#pragma unroll
    for (int i = 0; i < MPW; ++i) {
      const int fcol = 16 * (w * MPW + i) + 4 * g;
      f32x4 ga, be;
      if constexpr (PRE) {
        ga = gpre[i];
        be = bpre[i];
      } else {
        ga = ld4g(goff, fcol);
        be = ld4g(boff, fcol);
      }
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        f32x4 y;
#pragma unroll
        for (int r = 0; r < 4; ++r) y[r] = fmaf((res[i][nt][r] - mean[nt]) * rstd[nt], ga[r], be[r]);
        F::st4(XN + (16 * nt + n) * Y::XN_S + fcol * E, y);
      }
    }
    __syncthreads();
  };

  // packed matrices of layer l, chunk c (mppi_nets.cpp::build_fa_net order)
  auto Wqkv = [&](int l, int c) { return img + f.wqkv[l] + (long)c * (3 * CW / 16) * (D / 32) * F::FRAG; };
  auto Wo = [&](int l, int c) { return img + f.wo[l] + (long)c * (D / 16) * (CW / 32) * F::FRAG; };
  auto W1 = [&](int l, int c) { return img + f.w1[l] + (long)c * (FC / 16) * (D / 32) * F::FRAG; };
  auto W2 = [&](int l, int c) { return img + f.w2[l] + (long)c * (D / 16) * (FC / 32) * F::FRAG; };
  // one A-fragment pipeline per GEMM kind, each primed while the previous GEMM finishes.  (One 8- or 16-slot
  // fragment ring shared by every GEMM of the step was tried for D = 512: 94-103 ms vs 84 ms per config-#3 launch.)
  APipe<PREC, QMT, PF> pq;
  APipe<PREC, MPW, PFR> po;
  APipe<PREC, FMT, PF> pf1;
  APipe<PREC, MPW, PFR> pf2;
  pipe_prime<PREC, QMT, D / 32, PF>(pq, Wqkv(0, 0), w * QMT, lane);

#ifdef MPPI_STAMPS
  unsigned long long st_[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long tprev_ = __builtin_amdgcn_s_memtime();
#endif
  for (int t = 0; t < a.H; ++t) {
    // ---- controls of step t (perturbed, clamped) into their token rows; prefetch step t+1
    if (uown) {
      float u = unext;
      if (a.ctrl_clamp > 0.0f) u = fminf(a.ctrl_clamp, fmaxf(-a.ctrl_clamp, u));
      XU[us * L + nx + uj] = u;
      const int tn = t + 1 < a.H ? t + 1 : t;
      unext = Ub[tn] + eb[(long)tn * a.Kp];
    }
    __syncthreads();
    if (cown) {
      float s2 = 0.0f;
      for (int j = 0; j < nu; ++j) {
        const float u = XU[tid * L + nx + j];
        s2 = fmaf(u, u, s2);
      }
      cusq = s2;
      cu0 = XU[tid * L + nx];
    }

    // ---- feature encoding: ReLU(LN(w v + b)) + pos  (closed-form LN moments)
    {
      float ev[NT], em[NT], er[NT];
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const float v = XU[16 * nt + n];
        const float var = fmaxf(fmaf(v, fmaf(v, f.enc_vw, 2.0f * f.enc_cwb), f.enc_vb), 0.0f);
        ev[nt] = v;
        em[nt] = fmaf(v, f.enc_mw, f.enc_mb);
        er[nt] = 1.0f / sqrtf(var + 1e-5f);
      }
#pragma unroll
      for (int i = 0; i < MPW; ++i) {
        const int fcol = 16 * (w * MPW + i) + 4 * g;
        const f32x4 we = ld4g(f.we, fcol), be = ld4g(f.be, fcol), ge = ld4g(f.ge, fcol), bt = ld4g(f.bte, fcol);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          const f32x4 pe = ld4g(f.pos, tok[nt] * D + fcol);
#pragma unroll
          for (int r = 0; r < 4; ++r)
            res[i][nt][r] = fmaxf(fmaf((fmaf(we[r], ev[nt], be[r]) - em[nt]) * er[nt], ge[r], bt[r]), 0.0f) + pe[r];
        }
      }
    }

    FA_STAMP(0);
    for (int l = 0; l < f.nlayers; ++l) {
      // ---- pre-LN multi-head self-attention over the L tokens of each sample
      layer_norm(f.ln1g[l], f.ln1b[l]);
      FA_STAMP(1);
      for (int c = 0; c < NCH; ++c) {
        {  // Q|K|V of chunk c (Q pre-scaled by 1/sqrt(HD) on the host)
          f32x4 acc[QMT][NT];
#pragma unroll
          for (int i = 0; i < QMT; ++i) {
            const f32x4 bq = ld4g(f.bqkv[l], c * 3 * CW + 16 * (w * QMT + i) + 4 * g);
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) acc[i][nt] = bq;
          }
          fa_gemm_p<PREC, QMT, D / 32, PF, NT>(acc, pq, Wqkv(l, c), w * QMT, XN, Y::XN_S, lane,
                                           [&] { pipe_prime<PREC, MPW, CW / 32, PFR>(po, Wo(l, c), w * MPW, lane); });
#pragma unroll
          for (int i = 0; i < QMT; ++i) {
            const int mt = w * QMT + i;
            const int which = mt / (CW / 16), col = 16 * (mt - which * (CW / 16)) + 4 * g;
            if (Y::MA && which == 2) {  // bf16: V transposed, Vt[feature][token]
#pragma unroll
              for (int nt = 0; nt < NT; ++nt)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                  *reinterpret_cast<__bf16*>(Vb + (col + r) * Y::VT_S + (16 * nt + n) * 2) = (__bf16)acc[i][nt][r];
              continue;
            }
            char* dst = which == 0 ? Qb : (which == 1 ? Kb : Vb);
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) F::st4(dst + (16 * nt + n) * Y::CW_S + col * E, acc[i][nt]);
          }
        }
        FA_STAMP(2);
        __syncthreads();
        if constexpr (Y::MA) {
          // ---- bf16: attention on MFMA, per head h of the chunk (block-diagonal over the workgroup's samples).
          // S^T = K Q^T: unit (h, i-tile) -> all j-tiles of S^T[j][i]; the softmax over j for column i is an
          // in-lane max/sum over (j-tile, r) plus a 4-lane-group reduction; P[h][i][j] (bf16, normalised) rows.
          constexpr int NTI = R / 16, KW = HD >= 32 ? 32 : 16, KJ = R >= 32 ? 32 : 16;  // contraction over d / j
          static_assert(HD % KW == 0 && R % KJ == 0, "attention MFMA blocking");
          char* Pbh = reinterpret_cast<char*>(Pb);
          for (int u = w; u < HC * NTI; u += NW) {
            const int h = u / NTI, it = u - h * NTI;
            f32x4 st[NTI];
#pragma unroll
            for (int mj = 0; mj < NTI; ++mj) {
              st[mj] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
              for (int kb = 0; kb < HD / KW; ++kb)
                st[mj] = att_mma<KW>(Kb + (16 * mj + n) * Y::CW_S + (h * HD + KW * kb) * 2,
                                     Qb + (16 * it + n) * Y::CW_S + (h * HD + KW * kb) * 2, g, st[mj]);
            }
            // column i = 16 it + n; rows j = 16 mj + 4 g + r; same-sample pairs only
            const int i = 16 * it + n;
            const int si = i < G * L ? i / L : -1;
            float m = -INFINITY;
#pragma unroll
            for (int mj = 0; mj < NTI; ++mj)
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const int j = 16 * mj + 4 * g + r;
                if (!(j < G * L && j / L == si)) st[mj][r] = -INFINITY;
                m = fmaxf(m, st[mj][r]);
              }
            m = fa_group_max(m);
            float sum = 0.0f;
#pragma unroll
            for (int mj = 0; mj < NTI; ++mj)
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const float e = si >= 0 ? __expf(st[mj][r] - m) : 0.0f;
                st[mj][r] = e;
                sum += e;
              }
            sum = fa_group_sum(sum);
            const float inv = sum > 0.0f ? 1.0f / sum : 0.0f;
#pragma unroll
            for (int mj = 0; mj < NTI; ++mj) F::st4(Pbh + (h * R + i) * Y::P_S + (16 * mj + 4 * g) * 2, st[mj] * inv);
          }
          __syncthreads();
          // O^T = V^T P^T: unit (h, d-tile, i-tile); D layout O^T[d][i] -> O[i][d] rows, 4 features per store
          for (int u = w; u < HC * (HD / 16) * NTI; u += NW) {
            const int it = u % NTI, hd = u / NTI, h = hd / (HD / 16), dt = hd - h * (HD / 16);
            f32x4 o = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
            for (int kb = 0; kb < R / KJ; ++kb)
              o = att_mma<KJ>(Vb + (h * HD + 16 * dt + n) * Y::VT_S + KJ * kb * 2,
                              Pbh + (h * R + 16 * it + n) * Y::P_S + KJ * kb * 2, g, o);
            F::st4(Ob + (16 * it + n) * Y::CW_S + (h * HD + 16 * dt + 4 * g) * 2, o);
          }
          __syncthreads();
        } else {
          // VALU attention in one phase (scores and probabilities never pass through LDS): thread = (head h,
          // sample s, query token i, 4-feature quarter q4 of the head): the row's L scores with an online softmax
          // (running max and sum, rescaled as they grow), accumulated straight into O for its 4 features; the HD/4
          // threads of a row each recompute its scores.  (Three phases with two more barriers before.)
          constexpr int QQ = HD / 4;
          for (int task = tid; task < HC * G * L * QQ; task += NTH) {
            const int q4 = task % QQ, t2 = task / QQ, i = t2 % L, t3 = t2 / L, s = t3 % G, h = t3 / G;
            const char* qp = Qb + (s * L + i) * Y::CW_S + h * HD * E;
            f32x4 qv[QQ];
#pragma unroll
            for (int d = 0; d < QQ; ++d) qv[d] = F::ld4(qp + 4 * d * E);
            float m = -INFINITY, lsum = 0.0f;
            f32x4 o = {0.0f, 0.0f, 0.0f, 0.0f};
            for (int j = 0; j < L; ++j) {
              const char* kp = Kb + (s * L + j) * Y::CW_S + h * HD * E;
              float sc = 0.0f;
#pragma unroll
              for (int d = 0; d < QQ; ++d) {
                const f32x4 kv = F::ld4(kp + 4 * d * E);
                sc = fmaf(qv[d][0], kv[0], fmaf(qv[d][1], kv[1], fmaf(qv[d][2], kv[2], fmaf(qv[d][3], kv[3], sc))));
              }
              const float mn = fmaxf(m, sc), corr = __expf(m - mn), pj = __expf(sc - mn);
              const f32x4 vv = F::ld4(Vb + (s * L + j) * Y::CW_S + (h * HD + 4 * q4) * E);
              lsum = fmaf(lsum, corr, pj);
#pragma unroll
              for (int r = 0; r < 4; ++r) o[r] = fmaf(pj, vv[r], o[r] * corr);
              m = mn;
            }
            F::st4(Ob + (s * L + i) * Y::CW_S + (h * HD + 4 * q4) * E, o * (1.0f / lsum));
          }
          __syncthreads();
        }
        FA_STAMP(3);
        // out-proj, K-split over chunks: res += Wo[:, chunk c] O^T; then prime the next chunk's Q|K|V or FFN1
        fa_gemm_p<PREC, MPW, CW / 32, PFR, NT>(res, po, Wo(l, c), w * MPW, Ob, Y::CW_S, lane, [&] {
          if (c + 1 < NCH)
            pipe_prime<PREC, QMT, D / 32, PF>(pq, Wqkv(l, c + 1), w * QMT, lane);
          else
            pipe_prime<PREC, FMT, D / 32, PF>(pf1, W1(l, 0), w * FMT, lane);
        });
        FA_STAMP(4);
      }
#pragma unroll
      for (int i = 0; i < MPW; ++i) {
        const f32x4 bo = ld4g(f.bo[l], 16 * (w * MPW + i) + 4 * g);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) res[i][nt] += bo;
      }
      // ---- pre-LN FFN: res += W2 ReLU(W1 LN(res) + b1) + b2, hidden in chunks of FC rows
      layer_norm(f.ln2g[l], f.ln2b[l]);
      FA_STAMP(1);
      for (int fc = 0; fc < NFC; ++fc) {
        {
          f32x4 hacc[FMT][NT];
#pragma unroll
          for (int i = 0; i < FMT; ++i) {
            const f32x4 b1 = ld4g(f.b1[l], fc * FC + 16 * (w * FMT + i) + 4 * g);
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) hacc[i][nt] = b1;
          }
          fa_gemm_p<PREC, FMT, D / 32, PF, NT>(hacc, pf1, W1(l, fc), w * FMT, XN, Y::XN_S, lane,
                                           [&] { pipe_prime<PREC, MPW, FC / 32, PFR>(pf2, W2(l, fc), w * MPW, lane); });
#pragma unroll
          for (int i = 0; i < FMT; ++i)
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) {
              f32x4 hv = hacc[i][nt];
#pragma unroll
              for (int r = 0; r < 4; ++r) hv[r] = fmaxf(hv[r], 0.0f);
              F::st4(HID + (16 * nt + n) * Y::HID_S + (16 * (w * FMT + i) + 4 * g) * E, hv);
            }
        }
        FA_STAMP(5);
        __syncthreads();
        // then prime the next FFN chunk, the next layer's first Q|K|V, or (last layer) the next step's
        fa_gemm_p<PREC, MPW, FC / 32, PFR, NT>(res, pf2, W2(l, fc), w * MPW, HID, Y::HID_S, lane, [&] {
          if (fc + 1 < NFC)
            pipe_prime<PREC, FMT, D / 32, PF>(pf1, W1(l, fc + 1), w * FMT, lane);
          else
            pipe_prime<PREC, QMT, D / 32, PF>(pq, Wqkv(l + 1 < f.nlayers ? l + 1 : 0, 0), w * QMT, lane);
        });
        __syncthreads();
        FA_STAMP(6);
      }
#pragma unroll
      for (int i = 0; i < MPW; ++i) {
        const f32x4 b2 = ld4g(f.b2[l], 16 * (w * MPW + i) + 4 * g);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) res[i][nt] += b2;
      }
    }

    // ---- output layer (D -> 1 per token); state rows x += y
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      float s = 0.0f;
#pragma unroll
      for (int i = 0; i < MPW; ++i) {
        const f32x4 wo = ld4g(f.wout, 16 * (w * MPW + i) + 4 * g);
#pragma unroll
        for (int r = 0; r < 4; ++r) s = fmaf(wo[r], res[i][nt][r], s);
      }
      s = fa_group_sum(s);
      if (g == 0) OUTP[w * R + 16 * nt + n] = s;
    }
    __syncthreads();
    for (int r = tid; r < G * L; r += NTH) {
      if (r % L < nx) {
        float y = f.b_out;
#pragma unroll
        for (int w2 = 0; w2 < NW; ++w2) y += OUTP[w2 * R + r];
        XU[r] += y;
      }
    }
    __syncthreads();
    if (cown) cost += eval_cost(cu0, cusq);
    FA_STAMP(7);
  }
#ifdef MPPI_STAMPS
  if (lane == 0)
    for (int i = 0; i < kNumFaStamps; ++i) atomicAdd(&g_fa_stamps[i], st_[i]);
#endif
  kclock_record(a, kc);  // after the horizon's last barrier
  if (cown) {
    if (a.terminal_weight != 0.0f) cost += a.terminal_weight * eval_cost(0.0f, 0.0f);
    if (ck < a.K) a.costs[(long)b * a.Kp + ck] = isfinite(cost) ? cost : INFINITY;
  }
  if (a.xout && k0 == 0 && tid < nx) a.xout[(long)b * nx + tid] = XU[tid];  // env step: sample 0's final state
}

// ------------------------------------------------------------------------------------------------ small nets
// fa_small_kernel: the FeatureAttention net with hidden 64, 4 heads of 16 and L <= 16 tokens (the cartpole
// estimator's net, src/cartpole_mppi_estimator.py:28-33), bf16.  A workgroup of 4 waves owns NT tiles of 16 token
// rows (floor(16 / L) whole samples per tile) for the whole horizon.  Every wave holds the WHOLE residual stream of
// its tiles in registers (64 features x 16 tokens = 16 VGPRs per tile), so:
//   * LayerNorms are wave-local (in-lane sums + a 4-lane-group reduction), and their outputs feed the GEMMs straight
//     from registers: the accumulator tiles 2kb, 2kb+1 packed to bf16 are k-block kb of the B operand, with the
//     weights packed in that k order (mppi_nets.cpp::small_k);
//   * wave h computes head h: Q_h, K_h (W as the A operand) and V_h (operands swapped, so the tile comes out token-
//     major), then S^T = K_h Q_h^T and O_h^T = V_h^T P^T as two v_mfma_f32_16x16x16_bf16 whose operands are those
//     accumulator tiles as they are (softmax over the 4 lane groups, block-diagonal sample mask);
//   * each wave stores its head's O tile (bf16) to LDS; after one barrier every wave computes the whole out-proj
//     from the gathered rows (identical arithmetic, so identical residuals in every wave);
//   * the second FFN GEMM is split over the waves by K (the wave's own 64-row slice of the FFN hidden layer, computed
//     by the first FFN GEMM from its registers), and the four partial residual updates are summed in a fixed order
//     after one barrier: 2 barriers per layer.
// Weights stream from L2 (the image is ~200 KB), each wave loading only its own fragments, a phase ahead.
typedef __attribute__((ext_vector_type(4))) short s16x4;

__device__ __forceinline__ bf16x8 fs_pack8(const f32x4& lo, const f32x4& hi) {
  return bf16x8{(__bf16)lo[0], (__bf16)lo[1], (__bf16)lo[2], (__bf16)lo[3],
                (__bf16)hi[0], (__bf16)hi[1], (__bf16)hi[2], (__bf16)hi[3]};
}
__device__ __forceinline__ s16x4 fs_pack4(const f32x4& v) {
  return __builtin_bit_cast(s16x4, bf16x4{(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]});
}
__device__ __forceinline__ f32x4 fs_mma32(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 fs_mma16(const s16x4& a, const s16x4& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0);
}

// LDS bytes of fa_small_kernel beyond the staged vectors: the out-proj fragments of every layer (8 KB each, shared by
// the 4 waves, staged once), the FFN2 partial-update exchange [4 waves][NT][4][64] f32x4, the attention output rows
// O [NT][16][64 + 8] bf16, then the token-value rows XU [NT][16]
constexpr int kFsORow = (64 + 8) * 2;
constexpr int kFsWoBytes = 8 * 1024;  // per layer: 4 m-tiles x 2 k-blocks x 1 KB
__host__ __device__ constexpr int fa_small_xp_bytes(int NT) { return 4 * NT * 4 * 64 * 16; }
__host__ __device__ constexpr int fa_small_o_bytes(int NT) { return NT * 16 * kFsORow; }
__host__ __device__ constexpr int fa_small_lds(int NT, int nl) {
  return nl * kFsWoBytes + fa_small_xp_bytes(NT) + fa_small_o_bytes(NT) + NT * 16 * 4;
}

template <int NT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3, 3))) void fa_small_kernel(SolveArgs a, FaArgs f) {
  constexpr int D = 64;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const KClock kc = kclock_begin(a);
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, n = lane & 15;
  const int h = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave = attention head
  const int L = f.L, nx = f.nx, nu = f.nu;
  const int Gt = 16 / L, G = NT * Gt;  // samples per tile, per workgroup
  const int gps = (a.K + G - 1) / G;   // workgroups per solve
  const int b = blockIdx.x / gps;
  const int k0 = (blockIdx.x - b * gps) * G;
  if (blockIdx.x == 0 && tid == 0) *a.status = 0u;

  char* VEC = lds;  // the image's fp32 vectors [0, vec_lds)
  char* WO = lds + f.vec_lds;  // out-proj fragments, layer l at l * kFsWoBytes
  f32x4* XP = reinterpret_cast<f32x4*>(WO + f.nlayers * kFsWoBytes);
  char* OB = lds + f.vec_lds + fa_small_xp_bytes(NT);
  float* XU = reinterpret_cast<float*>(OB + fa_small_o_bytes(NT));
  for (int i = tid; i < f.vec_lds / 16; i += 256) reinterpret_cast<int4*>(VEC)[i] = reinterpret_cast<const int4*>(f.img)[i];
  for (int l = 0; l < f.nlayers; ++l)
    for (int i = tid; i < kFsWoBytes / 16; i += 256)
      reinterpret_cast<int4*>(WO + l * kFsWoBytes)[i] = reinterpret_cast<const int4*>(f.img + f.wo[l])[i];
  __syncthreads();
  auto vec4 = [&](int off, int idx) { return *reinterpret_cast<const f32x4*>(VEC + off + idx * 4); };
  auto vec1 = [&](int off, int idx) { return *reinterpret_cast<const float*>(VEC + off + idx * 4); };
  auto xp = [&](int w, int nt, int mt) -> f32x4& { return XP[((w * NT + nt) * 4 + mt) * 64 + lane]; };

  // this lane's token row n of every tile: token index, and the sample's control slot (-1: state or pad row)
  const bool rvalid = n < Gt * L;
  const int tok = rvalid ? n % L : 0;
  const int cj = (rvalid && tok >= nx) ? tok - nx : -1;
  // attention mask: key 4g + r attends query n iff both are real rows of the same sample
  bool kval[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int j = 4 * g + r;
    kval[r] = rvalid && j < Gt * L && j / L == n / L;
  }
  // token values: state rows carry x, control rows the step's perturbed control (loaded a step ahead)
  float xu[NT], un[NT];
  const float* x0 = a.x0 + (long)b * nx;
  // control loads are unconditional (a conditional load makes hipcc wait for it at once): rows without a control
  // read slot 0 and discard it
  const float* ub = a.U + ((long)b * nu + (cj >= 0 ? cj : 0)) * a.H;
  const float* eb[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    xu[nt] = (rvalid && tok < nx) ? x0[tok] : 0.0f;
    const int kk = min(k0 + nt * Gt + n / L, a.Kp - 1);
    eb[nt] = a.noise + ((long)b * nu + (cj >= 0 ? cj : 0)) * a.H * a.Kp + kk;
  }
  auto load_ctrl = [&](int t) {
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) un[nt] = ub[t] + eb[nt][(long)t * a.Kp];
  };
  load_ctrl(0);

  float cx[MPPI_CTX_MAX];
#pragma unroll
  for (int i = 0; i < MPPI_CTX_MAX; ++i) cx[i] = a.ctx ? a.ctx[(long)b * MPPI_CTX_MAX + i] : a.ctx_default[i];
  const bool cown = h == 0 && tid < G;  // wave 0, lane s: the running cost of sample s
  const int cbase = (tid / Gt) * 16 + (tid % Gt) * L;
  float cost = 0.0f;

  f32x4 res[NT][4];  // residual stream of every tile, D layout: feature 16 mt + 4 g + r of token n
  // LayerNorm over the 64 features of token n (population variance, eps 1e-5) without its affine map (folded into
  // the next GEMM on the host) -> bf16 B operand in register k order
  auto layer_norm = [&](const f32x4 (&x)[4], bf16x8 (&xn)[2]) {
    float s = 0.0f;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) s += (x[mt][0] + x[mt][1]) + (x[mt][2] + x[mt][3]);
    const float mean = fa_group_sum(s) * (1.0f / D);
    float q = 0.0f;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float d = x[mt][r] - mean;
        q = fmaf(d, d, q);
      }
    const float rstd = __builtin_amdgcn_rsqf(fa_group_sum(q) * (1.0f / D) + 1e-5f);  // argument >= 1e-5
    f32x4 y[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) y[mt][r] = (x[mt][r] - mean) * rstd;
    xn[0] = fs_pack8(y[0], y[1]);
    xn[1] = fs_pack8(y[2], y[3]);
  };

  // this wave's fragments of layer l (each wave loads only its own): Q_h K_h V_h (2 k-blocks each), the out-proj
  // columns of head h (4 m-tiles), the FFN1 rows of hidden slice h (4 m-tiles x 2 k-blocks), the FFN2 k-blocks of
  // slice h (4 m-tiles x 2)
  // through one buffer resource: the fragment offset is the scalar soffset, the lane's 16 B the fixed voffset (no
  // per-lane 64-bit addresses)
  const __amdgpu_buffer_rsrc_t wrs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(f.img), 0, f.img_bytes, 0x00020000);
  auto frag = [&](int off) {
    return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(wrs, lane * 16, off, 0));
  };
  bf16x8 fq[2], fk[2], fv[2], f1[4][2], f2[4][2];
  auto load_attn = [&](int l) {
    const int o = f.s_wqkv[l] + h * 6 * 1024;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      fq[kb] = frag(o + kb * 1024);
      fk[kb] = frag(o + (2 + kb) * 1024);
      fv[kb] = frag(o + (4 + kb) * 1024);
    }
  };
  auto load_ffn1 = [&](int l) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) f1[i][kb] = frag(f.s_w1[l] + ((4 * h + i) * 2 + kb) * 1024);
  };
  auto load_ffn2 = [&](int l) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) f2[i][kb] = frag(f.s_w2[l] + (i * 8 + 2 * h + kb) * 1024);
  };
  load_attn(0);

#ifdef MPPI_STAMPS
  unsigned long long st_[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long tprev_ = __builtin_amdgcn_s_memtime();
#endif
  for (int t = 0; t < a.H; ++t) {
    FA_STAMP(6);
    // ---- controls of step t into their token rows (clamped); prefetch step t+1
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
      if (cj >= 0) xu[nt] = a.ctrl_clamp > 0.0f ? fminf(a.ctrl_clamp, fmaxf(-a.ctrl_clamp, un[nt])) : un[nt];
    load_ctrl(t + 1 < a.H ? t + 1 : t);
    // ---- feature encoding: ReLU(LN(w v + b)) + pos, every feature in every wave.  LN(w v + b) = rstd(v) (v c1 + c2)
    // with the centred, gamma-scaled c1 = (w - mean w) gamma, c2 = (b - mean b) gamma (host) and the closed-form
    // variance of w v + b over the features
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const float v = xu[nt];
      const float var = fmaxf(fmaf(v, fmaf(v, f.enc_vw, 2.0f * f.enc_cwb), f.enc_vb), 0.0f);
      const float er = __builtin_amdgcn_rsqf(var + 1e-5f);
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const int fcol = 16 * mt + 4 * g;
        const f32x4 c1 = vec4(f.s_c1, fcol), c2 = vec4(f.s_c2, fcol), bt = vec4(f.bte, fcol);
        const f32x4 pe = vec4(f.pos, tok * D + fcol);
#pragma unroll
        for (int r = 0; r < 4; ++r) res[nt][mt][r] = fmaxf(fmaf(fmaf(v, c1[r], c2[r]), er, bt[r]), 0.0f) + pe[r];
      }
    }

    FA_STAMP(0);
    for (int l = 0; l < f.nlayers; ++l) {
      // ---- pre-LN attention, head h of every tile
      f32x4 part[NT][4];
      {
        const f32x4 bq = vec4(f.s_bqkv[l], 16 * h + 4 * g), bk = vec4(f.s_bqkv[l], D + 16 * h + 4 * g);
        const float bvv = vec1(f.s_bqkv[l], 2 * D + 16 * h + n);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          bf16x8 xn[2];
          layer_norm(res[nt], xn);
          f32x4 q = bq, kk = bk, v = {bvv, bvv, bvv, bvv};
#pragma unroll
          for (int kb = 0; kb < 2; ++kb) {
            q = fs_mma32(fq[kb], xn[kb], q);    // Q_h^T [dim][token]
            kk = fs_mma32(fk[kb], xn[kb], kk);  // K_h^T [dim][token]
            v = fs_mma32(xn[kb], fv[kb], v);    // V_h [token][dim]
          }
          // S^T[key][query] = K_h Q_h^T (Q pre-scaled by 1/sqrt(16) on the host), softmax over the keys of query n
          f32x4 sc = fs_mma16(fs_pack4(kk), fs_pack4(q), f32x4{0.0f, 0.0f, 0.0f, 0.0f});
          float m = -INFINITY;
#pragma unroll
          for (int r = 0; r < 4; ++r) m = fmaxf(m, kval[r] ? sc[r] : -INFINITY);
          m = fa_group_max(m);
          float sum = 0.0f;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            sc[r] = kval[r] ? __expf(sc[r] - m) : 0.0f;
            sum += sc[r];
          }
          sum = fa_group_sum(sum);
          const float inv = sum > 0.0f ? 1.0f / sum : 0.0f;
          // O_h^T[dim][query] = V_h^T P^T (P normalised, bf16), then head h's out-proj columns: a K-split partial
          const f32x4 o = fs_mma16(fs_pack4(v), fs_pack4(sc * inv), f32x4{0.0f, 0.0f, 0.0f, 0.0f});
          // O[query n][16 h + 4 g + r]: this head's 4 features of row n (one 8-byte store)
          *reinterpret_cast<s16x4*>(OB + (nt * 16 + n) * kFsORow + (16 * h + 4 * g) * 2) = fs_pack4(o);
        }
      }
      FA_STAMP(1);
      __syncthreads();
      // out-proj from the gathered heads, every m-tile in every wave (identical arithmetic: identical residuals)
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const f32x4 bo = vec4(f.bo[l], 16 * mt + 4 * g);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          f32x4 acc = bo;
#pragma unroll
          for (int kb = 0; kb < 2; ++kb)  // the whole out-proj (natural k order: its input O comes from LDS rows)
            acc = fs_mma32(*reinterpret_cast<const bf16x8*>(WO + l * kFsWoBytes + (mt * 2 + kb) * 1024 + lane * 16),
                           *reinterpret_cast<const bf16x8*>(OB + (nt * 16 + n) * kFsORow + (32 * kb + 8 * g) * 2), acc);
          res[nt][mt] += acc;
        }
      }
      load_ffn1(l);
      load_ffn2(l);
      FA_STAMP(2);
      // ---- pre-LN FFN: hidden slice h (64 rows) from registers, its K-split share of the second GEMM
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        bf16x8 xn[2];
        layer_norm(res[nt], xn);
        f32x4 hid[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          hid[i] = vec4(f.s_b1[l], 64 * h + 16 * i + 4 * g);
#pragma unroll
          for (int kb = 0; kb < 2; ++kb) hid[i] = fs_mma32(f1[i][kb], xn[kb], hid[i]);
#pragma unroll
          for (int r = 0; r < 4; ++r) hid[i][r] = fmaxf(hid[i][r], 0.0f);
        }
        const bf16x8 hb0 = fs_pack8(hid[0], hid[1]), hb1 = fs_pack8(hid[2], hid[3]);
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
          part[nt][mt] = fs_mma32(f2[mt][1], hb1, fs_mma32(f2[mt][0], hb0, f32x4{0.0f, 0.0f, 0.0f, 0.0f}));
      }
      load_attn(l + 1 < f.nlayers ? l + 1 : 0);  // the next layer's (or the next step's first) fragments
      FA_STAMP(3);
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) xp(h, nt, mt) = part[nt][mt];
      __syncthreads();
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const f32x4 b2 = vec4(f.b2[l], 16 * mt + 4 * g);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          res[nt][mt] += ((xp(0, nt, mt) + xp(1, nt, mt)) + (xp(2, nt, mt) + xp(3, nt, mt))) + b2;
      }
      FA_STAMP(4);
    }

    // ---- output layer (64 -> 1 per token), state rows x += y; wave 0 evaluates the running costs
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      float y = 0.0f;
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const f32x4 wo = vec4(f.wout, 16 * mt + 4 * g);
#pragma unroll
        for (int r = 0; r < 4; ++r) y = fmaf(wo[r], res[nt][mt][r], y);
      }
      y = fa_group_sum(y) + f.b_out;
      if (rvalid && tok < nx) xu[nt] += y;
    }
    if (h == 0) {  // wave-local: XU rows written and read by wave 0 only (in-order LDS)
      if (g == 0)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) XU[nt * 16 + n] = xu[nt];
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
      __builtin_amdgcn_wave_barrier();
      if (cown) {
        const float* xr = XU + cbase;
        float usq = 0.0f;
        for (int j = 0; j < nu; ++j) usq = fmaf(xr[nx + j], xr[nx + j], usq);
        cost += fa_cost(a.cost_kind, xr, nu > 0 ? xr[nx] : 0.0f, usq, cx);
      }
      __builtin_amdgcn_wave_barrier();
    }
    FA_STAMP(5);
  }
#ifdef MPPI_STAMPS
  if (lane == 0)
    for (int i = 0; i < kNumFaStamps; ++i) atomicAdd(&g_fa_stamps[i], st_[i]);
#endif
  kclock_record(a, kc, tid == 0);
  if (cown) {
    if (a.terminal_weight != 0.0f) cost += a.terminal_weight * fa_cost(a.cost_kind, XU + cbase, 0.0f, 0.0f, cx);
    const int ck = k0 + tid;
    if (ck < a.K) a.costs[(long)b * a.Kp + ck] = isfinite(cost) ? cost : INFINITY;
  }
  if (a.xout && k0 == 0 && h == 0 && g == 0 && rvalid && tok < nx && n < L)  // env step: sample 0's final state
    a.xout[(long)b * nx + tok] = xu[0];
}

template <int NT>
static hipError_t launch_fa_small_t(const SolveArgs& a, const FaArgs& fa, hipStream_t stream) {
  const int G = NT * (16 / fa.L);
  if (G < 1) return hipErrorInvalidValue;
  const size_t lds = (size_t)fa.vec_lds + fa_small_lds(NT, fa.nlayers);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  auto kern = fa_small_kernel<NT>;
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)lds);
  if (e != hipSuccess) return e;
  const int gps = (a.K + G - 1) / G;
  hipLaunchKernelGGL(kern, dim3(gps * a.B), dim3(256), lds, stream, a, fa);
  return hipGetLastError();
}

template <int D, int PREC, int NT>
static hipError_t launch_fa_t(const SolveArgs& a, FaArgs fa, hipStream_t stream) {
  using Y = FaLay<D, PREC, NT>;
  fa.G = Y::R / fa.L;
  if (fa.G < 1) return hipErrorInvalidValue;
  size_t lds = (size_t)Y::bytes(fa.L);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  // D = 64: stage the fp32 vectors in LDS when they are small (the cartpole net: 9 KB); fa.vec_lds holds the
  // candidate prefix size on entry
  constexpr int kFaVecLds = 16 * 1024;
  if (D > 64 || fa.vec_lds > kFaVecLds || lds + fa.vec_lds > 160 * 1024) fa.vec_lds = 0;
  lds += fa.vec_lds;
  auto kern = fa_rollout_kernel<D, PREC, NT>;
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  const int gps = (a.K + fa.G - 1) / fa.G;
  hipLaunchKernelGGL(kern, dim3(gps * a.B), dim3(64 * Y::NW), lds, stream, a, fa);
  return hipGetLastError();
}

// Token rows per workgroup (16 NT) for hidden width D <= 128: the fewest n-tiles that hold one sample (more
// workgroups, so a K = 2048 cartpole solve fills the 256 CUs; small-D weights are L1/L2-resident, so the lower
// A-fragment reuse costs little); MPPI_FA_NT=1|2|4 overrides (read once).  D = 512 always uses 64 rows.
static int fa_nt(int L) {
  static const int env = [] {
    const char* e = getenv("MPPI_FA_NT");
    return e ? atoi(e) : 0;
  }();
  const int nmin = L <= 16 ? 1 : (L <= 32 ? 2 : 4);
  return (env == 1 || env == 2 || env == 4) && env >= nmin ? env : nmin;
}

static bool fa_small_on() {
  static const bool on = [] {
    const char* e = getenv("MPPI_FA_SMALL");
    return !(e && atoi(e) == 0);
  }();
  return on;
}

template <int D, int PREC>
static hipError_t launch_fa_nt(const SolveArgs& a, const FaArgs& fa, hipStream_t stream) {
  switch (fa_nt(fa.L)) {
    case 1: return launch_fa_t<D, PREC, 1>(a, fa, stream);
    case 2: return launch_fa_t<D, PREC, 2>(a, fa, stream);
    default: return launch_fa_t<D, PREC, 4>(a, fa, stream);
  }
}

// LDS bytes the FA kernel needs for (D, precision, L) at its largest row count; 0 when not built.
int fa_lds_bytes(int D, int precision, int L) {
  if (precision == MPPI_PREC_FP32) return D == 64 ? FaLay<64, MPPI_PREC_FP32, 4>::bytes(L) : 0;
  switch (D) {
    case 64: return FaLay<64, MPPI_PREC_BF16, 4>::bytes(L);
    case 128: return FaLay<128, MPPI_PREC_BF16, 4>::bytes(L);
    case 512: return FaLay<512, MPPI_PREC_BF16, 4>::bytes(L);
    default: return 0;
  }
}

hipError_t launch_fa_rollout(const SolveArgs& a, const FaNet& n, hipStream_t stream) {
  FaArgs fa;
  fa.img = reinterpret_cast<const char*>(n.d_img);
  fa.img_bytes = n.img_bytes;
  fa.D = n.D;
  fa.L = n.L;
  fa.nx = a.nx;
  fa.nu = a.nu;
  fa.nlayers = n.nlayers;
  fa.we = n.we;
  fa.be = n.be;
  fa.ge = n.ge;
  fa.bte = n.bte;
  fa.pos = n.pos;
  fa.wout = n.wout;
  for (int l = 0; l < kFaMaxLayers; ++l) {
    fa.ln1g[l] = n.ln1g[l];
    fa.ln1b[l] = n.ln1b[l];
    fa.bqkv[l] = n.bqkv[l];
    fa.bo[l] = n.bo[l];
    fa.ln2g[l] = n.ln2g[l];
    fa.ln2b[l] = n.ln2b[l];
    fa.b1[l] = n.b1[l];
    fa.b2[l] = n.b2[l];
    fa.wqkv[l] = n.wqkv[l];
    fa.wo[l] = n.wo[l];
    fa.w1[l] = n.w1[l];
    fa.w2[l] = n.w2[l];
    fa.s_wqkv[l] = n.s_wqkv[l];
    fa.s_w1[l] = n.s_w1[l];
    fa.s_w2[l] = n.s_w2[l];
    fa.s_bqkv[l] = n.s_bqkv[l];
    fa.s_b1[l] = n.s_b1[l];
  }
  fa.s_c1 = n.s_c1;
  fa.s_c2 = n.s_c2;
  fa.enc_mw = n.enc_mw;
  fa.enc_mb = n.enc_mb;
  fa.enc_vw = n.enc_vw;
  fa.enc_cwb = n.enc_cwb;
  fa.enc_vb = n.enc_vb;
  fa.b_out = n.b_out;
  fa.vec_lds = n.wqkv[0];  // the fp32 vectors precede the first packed matrix (mppi_nets.cpp::build_fa_net)
  if (n.L < 1 || n.L > kFaRows || a.nx + a.nu != n.L) return hipErrorInvalidValue;
  if (n.precision == MPPI_PREC_FP32) {
    if (n.D == 64) return launch_fa_nt<64, MPPI_PREC_FP32>(a, fa, stream);
    return hipErrorInvalidValue;
  }
  // small nets (bf16, hidden 64, L <= 16): the register-resident-residual kernel (MPPI_FA_SMALL=0: the general one)
  // (one 16-row tile per workgroup: two were slower, 1.23 vs 0.86 ms per cartpole estimator solve, same box)
  if (n.small && fa_small_on()) return launch_fa_small_t<1>(a, fa, stream);
  switch (n.D) {
    case 64: return launch_fa_nt<64, MPPI_PREC_BF16>(a, fa, stream);
    case 128: return launch_fa_nt<128, MPPI_PREC_BF16>(a, fa, stream);
    case 512: return launch_fa_t<512, MPPI_PREC_BF16, 4>(a, fa, stream);
    default: return hipErrorInvalidValue;
  }
}

#ifdef MPPI_STAMPS
extern "C" int mppi_debug_fa_stamps(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_fa_stamps), sizeof(unsigned long long) * kNumFaStamps) != hipSuccess)
    return -2;
  if (reset) {
    unsigned long long z[kNumFaStamps] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_fa_stamps), z, sizeof(z)) != hipSuccess) return -2;
  }
  return 0;
}
#endif

}  // namespace mppi
