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

#include "fa_common.h"
#include "frag_traits.h"

namespace mppi {

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

// A-fragment pipeline: the first PF k-blocks of a GEMM, loaded ahead (possibly across a barrier / VALU phase:
// in-flight global loads are not drained by the workgroup barrier here, which waits on lgkmcnt only).  Storage for
// MTA m-tiles; a GEMM of MT <= MTA tiles uses the first MT.
template <int PREC, int MTA, int PF>
struct APipe {
  typename FP<PREC>::Frag a[PF][MTA];
};

template <int PREC, int MT, int KB, int PF, int MTA>
__device__ __forceinline__ void pipe_prime(APipe<PREC, MTA, PF>& p, const char* __restrict__ W, int mt0, int lane) {
  static_assert(MT <= MTA, "pipe storage");
  using F = FP<PREC>;
#pragma unroll
  for (int s = 0; s < (PF < KB ? PF : KB); ++s)
#pragma unroll
    for (int i = 0; i < MT; ++i) p.a[s][i] = F::ldA(W + ((mt0 + i) * KB + s) * F::FRAG, lane);
}

// acc[i][nt] += W(m-tile mt0 + i) * X^T over KB k-blocks from a primed pipe, refilling it PF k-blocks ahead;
// next() runs as soon as this GEMM's last A load is issued (it primes the following GEMM's pipe).
template <int PREC, int MT, int KB, int PF, int NT, int MTA, class Next>
__device__ __forceinline__ void fa_gemm_p(f32x4 (&acc)[MT][NT], APipe<PREC, MTA, PF>& p, const char* __restrict__ W,
                                          int mt0, const char* X, int xs, int lane, Next&& next) {
  static_assert(MT <= MTA, "pipe storage");
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

// out-proj / FFN2 A-fragment pipeline depth at hidden 512 (build-time knob for same-box A/B: -DMPPI_FA_PFR=n)
#ifndef MPPI_FA_PFR
#define MPPI_FA_PFR 4
#endif
constexpr int kFaPfr512 = MPPI_FA_PFR;

template <int D, int PREC, int NT, int NH>
struct FaLay {
  static constexpr int R = 16 * NT;  // token rows per workgroup
  static constexpr int NW = fa_nw(D, NT, NH);
  static constexpr int CW = fa_cw(D, NH, NT);  // attention chunk width (whole heads)
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
  static constexpr int HC = CW / (D / NH);
  __host__ __device__ static constexpr int att_bytes(int L) {  // (the VALU attention keeps P in registers)
    return 3 * R * CW_S + VB + (MA ? HC * R * P_S : 0);
  }
  __host__ __device__ static constexpr int small(int L) {
    return ATT + (att_bytes(L) > R * HID_S ? att_bytes(L) : R * HID_S);
  }
  // small region: ST [NW][64] float2 | OUTP [NW][64] float | XU [64] float
  __host__ __device__ static constexpr int bytes(int L) { return small(L) + NW * R * 12 + R * 4; }
};

template <int D, int PREC, int NT, int NH>
__global__ __launch_bounds__(64 * fa_nw(D, NT, NH)) void fa_rollout_kernel(SolveArgs a, FaArgs f) {
  using F = FP<PREC>;
  using Y = FaLay<D, PREC, NT, NH>;
  constexpr int R = Y::R;  // token rows of this workgroup (NT n-tiles)
  constexpr int NW = Y::NW, NTH = 64 * NW;  // threads
  constexpr int HD = D / NH, CW = Y::CW, HC = Y::HC, NCH = NH / HC;
  constexpr int FC = Y::FC, NFC = 4 * D / FC;
  constexpr int MPW = D / 16 / NW;           // residual m-tiles per wave
  constexpr int QMT = 3 * CW / 16 / NW;      // Q|K|V m-tiles per wave per chunk
  constexpr int FMT = FC / 16 / NW;          // FFN hidden m-tiles per wave per chunk
  constexpr int E = Y::E;
  // A-fragment pipeline depths (k-blocks in flight) of the Q|K|V / FFN1 GEMMs and of the MPW-tile GEMMs
  // (out-proj, FFN2) that accumulate into the residual.  D = 512 streams 12.6 MB of fragments per sample-step from
  // L2: the deep pipelines (3 / 4 k-blocks) cover the L2 latency although they spill ~150 VGPRs of per-chunk
  // constants outside the inner loops (same-box sweep over PF 2..8 x PFR 1..5: 119 ms at 2/1, 86 ms at 3/4).
  constexpr int PF = D >= 512 ? 3 : 2, PFR = D >= 512 ? kFaPfr512 : (MPW >= 4 ? 1 : 2);
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
  auto eval_cost = [&](float u0, float usq, int t1) { return fa_cost(a.cost_kind, XU + tid * L, u0, usq, cx, t1); };

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
  // Two pipes, alternating: A feeds Q|K|V and FFN1, B the out-proj and FFN2; every GEMM primes the other one
  // (Q|K|V -> out-proj -> Q|K|V of the next chunk or FFN1 -> FFN2 -> FFN1 of the next chunk or Q|K|V of the next
  // layer), so a GEMM never refills the pipe it is reading.  Four separate pipes (one per GEMM kind) held 188 VGPRs
  // of fragments at hidden 512 and spilled to scratch (WRITE_SIZE ~24 GB per config-#3 launch).
  constexpr int MTA = QMT > FMT ? QMT : FMT;
  APipe<PREC, MTA, PF> pA;
  APipe<PREC, MPW, PFR> pB;
  auto& pq = pA;
  auto& pf1 = pA;
  auto& po = pB;
  auto& pf2 = pB;
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
          constexpr int NTI = R / 16, KW = HD >= 32 ? 32 : 16, KJ = R % 32 == 0 ? 32 : 16;  // contraction over d / j
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
              F::st4_relu(HID + (16 * nt + n) * Y::HID_S + (16 * (w * FMT + i) + 4 * g) * E, hacc[i][nt]);
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
    if (cown) cost += eval_cost(cu0, cusq, t + 1);
    FA_STAMP(7);
  }
#ifdef MPPI_STAMPS
  if (lane == 0)
    for (int i = 0; i < kNumFaStamps; ++i) atomicAdd(&g_fa_stamps[i], st_[i]);
#endif
  kclock_record(a, kc);  // after the horizon's last barrier
  if (cown) {
    if (a.terminal_weight != 0.0f) cost += a.terminal_weight * eval_cost(0.0f, 0.0f, a.H);
    if (ck < a.K) a.costs[(long)b * a.Kp + ck] = isfinite(cost) ? cost : INFINITY;
  }
  if (a.xout && k0 == 0 && tid < nx) a.xout[(long)b * nx + tid] = XU[tid];  // env step: sample 0's final state
}


template <int D, int PREC, int NT, int NH>
static hipError_t launch_fa_t(const SolveArgs& a, FaArgs fa, hipStream_t stream) {
  using Y = FaLay<D, PREC, NT, NH>;
  fa.G = Y::R / fa.L;
  if (fa.G < 1) return hipErrorInvalidValue;
  size_t lds = (size_t)Y::bytes(fa.L);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  // D = 64: stage the fp32 vectors in LDS when they are small (the cartpole net: 9 KB); fa.vec_lds holds the
  // candidate prefix size on entry
  constexpr int kFaVecLds = 16 * 1024;
  if (D > 64 || fa.vec_lds > kFaVecLds || lds + fa.vec_lds > 160 * 1024) fa.vec_lds = 0;
  lds += fa.vec_lds;
  auto kern = fa_rollout_kernel<D, PREC, NT, NH>;
  note_kernel("fa_rollout_kernel");
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  const int gps = (a.K + fa.G - 1) / fa.G;
  hipLaunchKernelGGL(kern, dim3(gps * a.B), dim3(64 * Y::NW), lds, stream, a, fa);
  return hipGetLastError();
}

// Token rows per workgroup (16 NT) for hidden width D <= 128: the fewest n-tiles that hold one sample (more
// workgroups, so a K = 2048 cartpole solve fills the 256 CUs; small-D weights are L1/L2-resident, so the lower
// A-fragment reuse costs little); MPPI_FA_NT=1|2|4 overrides (read once).  D = 512 always uses 64 rows.  More than
// 64 tokens take 5 n-tiles (80 rows).
static int fa_nt(int L) {
  static const int env = [] {
    const char* e = getenv("MPPI_FA_NT");
    return e ? atoi(e) : 0;
  }();
  const int nmin = fa_nt_min(L);
  return nmin <= 4 && (env == 1 || env == 2 || env == 4) && env >= nmin ? env : nmin;
}

// MPPI_FA_LAYERED=1: hidden 512 through the layer-by-layer path (kernels_fa_layered.hip), read per launch.  Off by
// default: config #3 measured 93.8 ms per solve against 82 ms for this file's fused kernel
static bool fa_layered_on() {
  const char* e = getenv("MPPI_FA_LAYERED");
  return e && atoi(e) == 1;
}

static bool fa_small_on() {
  static const bool on = [] {
    const char* e = getenv("MPPI_FA_SMALL");
    return !(e && atoi(e) == 0);
  }();
  return on;
}

template <int D, int PREC, int NH>
static hipError_t launch_fa_nt(const SolveArgs& a, const FaArgs& fa, hipStream_t stream) {
  switch (fa_nt(fa.L)) {
    case 1: return launch_fa_t<D, PREC, 1, NH>(a, fa, stream);
    case 2: return launch_fa_t<D, PREC, 2, NH>(a, fa, stream);
    case 4: return launch_fa_t<D, PREC, 4, NH>(a, fa, stream);
    default: return launch_fa_t<D, PREC, 5, NH>(a, fa, stream);
  }
}

template <int D, int PREC>
static hipError_t launch_fa_nh(const SolveArgs& a, const FaArgs& fa, int nh, hipStream_t stream) {
  return nh == 8 ? launch_fa_nt<D, PREC, 8>(a, fa, stream) : launch_fa_nt<D, PREC, 4>(a, fa, stream);
}

template <int D, int PREC>
static int fa_lay_bytes(int nh, int L) {
  const int nt = fa_nt_min(L);
  if (nt > 4) return nh == 8 ? FaLay<D, PREC, 5, 8>::bytes(L) : FaLay<D, PREC, 5, 4>::bytes(L);
  return nh == 8 ? FaLay<D, PREC, 4, 8>::bytes(L) : FaLay<D, PREC, 4, 4>::bytes(L);
}

// LDS bytes the FA kernel needs for (D, precision, heads, L) at its largest row count; 0 when not built (hidden 512
// takes at most 64 tokens: 80 rows of its activations do not fit the LDS).
int fa_lds_bytes(int D, int precision, int nh, int L) {
  if (nh != 4 && nh != 8) return 0;
  if (precision == MPPI_PREC_FP32) return D == 64 ? fa_lay_bytes<64, MPPI_PREC_FP32>(nh, L) : 0;
  switch (D) {
    case 64: return fa_lay_bytes<64, MPPI_PREC_BF16>(nh, L);
    case 128: return fa_lay_bytes<128, MPPI_PREC_BF16>(nh, L);
    case 512: return L <= 64 ? (nh == 8 ? FaLay<512, MPPI_PREC_BF16, 4, 8>::bytes(L)
                                        : FaLay<512, MPPI_PREC_BF16, 4, 4>::bytes(L)) : 0;
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
    if (n.D == 64) return launch_fa_nh<64, MPPI_PREC_FP32>(a, fa, n.nh, stream);
    return hipErrorInvalidValue;
  }
  // small nets (bf16, hidden 64, 4 heads, L <= 16): the register-resident-residual kernel (MPPI_FA_SMALL=0: the
  // general one) (one 16-row tile per workgroup: two were slower, 1.23 vs 0.86 ms per cartpole estimator solve)
  if (n.small && fa_small_on()) return launch_fa_small(a, fa, stream);
  switch (n.D) {
    case 64: return launch_fa_nh<64, MPPI_PREC_BF16>(a, fa, n.nh, stream);
    case 128: return launch_fa_nh<128, MPPI_PREC_BF16>(a, fa, n.nh, stream);
    case 512:
      if (n.L > 64) return hipErrorInvalidValue;
      // the layer-by-layer path when selected and its workspace holds the batch
      if (n.lay && n.d_ws && (long)a.B * a.K * n.L <= n.ws_rows && fa_layered_on()) return launch_fa_layered(a, n, stream);
      return n.nh == 8 ? launch_fa_t<512, MPPI_PREC_BF16, 4, 8>(a, fa, stream)
                       : launch_fa_t<512, MPPI_PREC_BF16, 4, 4>(a, fa, stream);
    default: return hipErrorInvalidValue;
  }
}

#ifdef MPPI_STAMPS
extern "C" int mppi_debug_fa_stamps(unsigned long long* out, int reset) {  // both FA translation units' sums
  unsigned long long s[kNumFaStamps];
  if (fa_small_stamps(s, reset) != 0) return -2;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_fa_stamps), sizeof(unsigned long long) * kNumFaStamps) != hipSuccess)
    return -2;
  for (int i = 0; i < kNumFaStamps; ++i) out[i] += s[i];
  if (reset) {
    unsigned long long z[kNumFaStamps] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_fa_stamps), z, sizeof(z)) != hipSuccess) return -2;
  }
  return 0;
}
#endif

}  // namespace mppi
