// FeatureAttentionStatePredictor rollout at hidden 512, layer by layer (learning/model.py:48-153 as driven by
// src/quadruped_mppi_estimator.py:58-79): every horizon step runs each Linear of the net as ONE GEMM over all
// B*K*L token rows of the batch, so a weight tile fetched into a CU serves 128 token rows (the fused
// fa_rollout_kernel serves the 49 rows of one sample per fetch and streams the 12.6 MB image from L2 per
// sample-step).  Per step t (DESIGN.md §4 "layered FA"):
//
//   fal_encode_kernel        cost of step t-1 on x_t, u_t into the control tokens, the scalar feature encoding
//                            ReLU(LN(w v + b)) + pos -> residual H (fp32), LayerNorm1 of layer 0 -> XN (bf16)
//   per layer l:
//     fal_gemm<256, Q|K|V>   QKV = XN Wqkv^T + b                    (bf16 out; Q pre-scaled by 1/sqrt(head dim))
//     fal_attn_kernel        per (sample, head): S^T = K Q^T, softmax over the L keys, P (bf16) V -> O (bf16)
//     fal_gemm<512, RES_LN>  H += O Wo^T + bo;  XN = LayerNorm2(H)   (full 512-wide rows per workgroup)
//     fal_gemm<256, RELU>    F = ReLU(XN W1^T + b1)                 (bf16 out)
//     fal_gemm<512, RES_LN>  H += F W2^T + b2;  XN = LayerNorm1 of layer l+1(H)
//       (last layer: RES_OUT  y = (H + F W2^T + b2) . w_out + b_out;  x_{t+1} = x_t + y on the state tokens)
//   fal_finish_kernel        (after step H-1) the last running cost, the terminal cost, costs[], env-step state
//
// Rounding points are the fused kernel's (oracle/nets_ref.py::fa_forward_engine "bf16"): LayerNorm outputs, Q/K/V,
// P, O and the FFN hidden activations in bf16, the residual stream, scores, softmax, biases and LayerNorm
// statistics in fp32.  Token rows r = (solve b * K + sample k) * L + token i, contiguous per sample.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdlib>

#include "fa_common.h"

namespace mppi {

namespace {

typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((address_space(3))) void* lds_ptr_t;

constexpr int kD = 512;    // hidden width this path is built for
constexpr int kBM = 128;   // token-row padding granule (the largest GEMM row tile)
constexpr int kVtS = 136;  // bytes per V^T row in the attention kernel (64 keys + 8 B: conflict-free b64 reads)

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
// max / sum of a value and lane ^ 32's (the two halves of a 32x32 accumulator's rows), identical in both lanes:
// v_permlane32_swap of (v, v) leaves {own, other} in lanes 0-31 and {other, own} in lanes 32-63
__device__ __forceinline__ float max32(float v) {
  auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(p[0]), __uint_as_float(p[1]));
}
__device__ __forceinline__ float sum32(float v) {
  auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(p[0]) + __uint_as_float(p[1]);
}
__device__ __forceinline__ unsigned pk_bf16(float a, float b) {
  const __bf16 x = (__bf16)a, y = (__bf16)b;
  return (unsigned)__builtin_bit_cast(unsigned short, x) | ((unsigned)__builtin_bit_cast(unsigned short, y) << 16);
}
__device__ __forceinline__ void st_bf16x4(__bf16* p, f32x4 v) {
  *reinterpret_cast<uint2*>(p) = make_uint2(pk_bf16(v[0], v[1]), pk_bf16(v[2], v[3]));
}

// 16-B chunk swizzle of an LDS tile row (BK / 8 chunks per row): ds_read_b128 of 32 consecutive rows at one k chunk
// spreads over all 64 banks within each 16-lane group (rows are a multiple of 16 apart from the tile base, so the
// swizzle of a fragment row is the lane's)
template <int CH>
__device__ __forceinline__ int chunk_swz(int row) {
  return CH == 8 ? (row >> 1) & 7 : (row >> 2) & 3;
}

// one stage of a GEMM tile: NI 16-B global_load_lds per lane (sources advanced by s stages of `rs` bytes)
// (the LDS address space exists in the device pass only; the host pass just needs the kernel's signature)
template <int NI>
__device__ __forceinline__ void fal_stage(const char* const (&src)[NI], const int (&dst)[NI], char* lds, int s,
                                          int buf, int rs, int sb) {
#ifdef __HIP_DEVICE_COMPILE__
#pragma unroll
  for (int i = 0; i < NI; ++i)
    __builtin_amdgcn_global_load_lds(src[i] + (long)s * rs, (lds_ptr_t)(lds + buf * sb + dst[i]), 16, 0, 0);
#endif
}

}  // namespace

// bf16 out (+ ReLU); full-row: residual + LayerNorm (H and XN written); residual + LayerNorm of the last layer's
// out-proj (XN and the row scalar HW = H . w_out written: H is not needed again); the last FFN2 + output layer
// (y = HW + (acc + b) . w_out + b_out: H is not read)
enum FalEpi : int { kEpiBf16 = 0, kEpiReluBf16 = 1, kEpiResLn = 2, kEpiResOut = 3, kEpiResLnW = 4 };

struct FalGemm {
  const __bf16* X;     // [rows][Kd] activations (A operand rows)
  const __bf16* W;     // [N][Kd] weights (B operand: C = X W^T)
  int Kd, N;           // contraction length, output columns (bf16 outputs: their row pitch; full-row kinds: 512)
  const float* bias;   // [N]
  __bf16* Y;           // bf16 output [rows][N] (kEpiBf16 / kEpiReluBf16) or the LayerNorm output [rows][512]
  float* H;            // residual stream [rows][512] (kEpiResLn / kEpiResOut)
  const float* g;      // LayerNorm gamma / beta (kEpiResLn)
  const float* b;
  const float* wout;   // output layer row (kEpiResOut)
  float bout;
  float* XU;           // token input scalars: state tokens updated in place (kEpiResOut)
  float* HW;           // [rows] H . w_out of the last layer's residual after its out-proj (kEpiResLnW -> kEpiResOut)
  int L, nx, M;        // tokens per sample, state tokens, real token rows (rows >= M are padding)
  int tiles;           // output tiles (row tiles x column tiles)
};

// C[BM rows x BN cols] = X W^T, 8 waves as 2 (rows) x 4 (cols), wave tile BM/2 x BN/4 on v_mfma_f32_32x32x16_bf16.
// X and W tiles of BK k-columns are staged into LDS by global_load_lds (16 B per lane, source addresses swizzled so
// the linear LDS image reads conflict-free), NST stages in a ring, one barrier per stage: the wait for stage s leaves
// the NST-2 younger stages in flight (counted vmcnt), and stage s+NST-1 is issued after the barrier into the buffer
// stage s-1 was read from.  The epilogue moves the accumulators through LDS in 32-row passes so every store is a
// coalesced row.
template <int BM, int BN, int BK, int NST, int EPI>
__global__ __launch_bounds__(512) void fal_gemm_kernel(FalGemm p) {
  constexpr int TM = BM / 2, TN = BN / 4, TI = TM / 32, TJ = TN / 32;
  // glds per wave per stage NI (instructions QT = ROWS / RPI; when 8 does not divide QT the last ones are issued
  // twice, same source and destination, so every wave counts the same NI loads per stage)
  constexpr int CH = BK / 8, RPI = 64 / CH, ROWS = BM + BN, QT = ROWS / RPI, NI = (QT + 7) / 8;
  constexpr int SB = ROWS * BK * 2, KS = BK / 16, RS = BK * 2;
  static_assert(TI >= 1 && TJ >= 1 && ROWS % RPI == 0 && NST >= 2 && NST <= 4, "fal_gemm blocking");
  static_assert(EPI < kEpiResLn ? (BN == 128 || BN == 256) : BN == kD, "fal_gemm epilogue width");
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w >> 2, wn = w & 3, lr = lane & 31, h = lane >> 5;

  // persistent: gridDim.x (a multiple of 8) workgroups loop over the tiles, so a tile's output stores drain while
  // the workgroup's next tile streams in.  Blocks are dispatched round-robin over the 8 XCDs: XCD x owns a
  // contiguous range of tiles, which its workgroups sweep together, so one row tile's N / BN column tiles run at
  // once on one XCD (the X tile is fetched into one L2; the whole W stays resident in every XCD's L2)
  const int nct = p.N / BN;
  const int xcd = blockIdx.x & 7, gx = gridDim.x >> 3, q8 = p.tiles >> 3, r8 = p.tiles & 7;
  const int tbase = xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8, tcnt = q8 + (xcd < r8 ? 1 : 0);
  for (int it = blockIdx.x >> 3; it < tcnt; it += gx) {
    const int id = tbase + it;
    const int rt = id / nct, ct = id - rt * nct;
    const long row0 = (long)rt * BM;
    const int col0 = ct * BN;

    // this thread's glds sources (image row q*RPI + lane/CH of instruction q = w + 8i; rows < BM are X)
    const char* src[NI];
    int dst[NI];
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int q = w + 8 * i < QT ? w + 8 * i : QT - 1, row = q * RPI + lane / CH, cc = (lane % CH) ^ chunk_swz<CH>(row);
      src[i] = row < BM ? reinterpret_cast<const char*>(p.X + (row0 + row) * p.Kd + 8 * cc)
                        : reinterpret_cast<const char*>(p.W + (long)(col0 + row - BM) * p.Kd + 8 * cc);
      dst[i] = q * RPI * RS;
    }
    int koff[KS];
    const int sw = chunk_swz<CH>(lr);
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) koff[kk] = lr * RS + 16 * ((2 * kk + h) ^ sw);

    f32x16 acc[TI][TJ];
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j) acc[i][j] = f32x16{};

#ifndef FAL_DIAG  // diagnostic builds only: 1 = no epilogue stores (kept live), 2 = no main loop
#define FAL_DIAG 0
#endif
    const int nK = FAL_DIAG == 2 ? 0 : p.Kd / BK;
#pragma unroll
    for (int s = 0; s < NST - 1; ++s)
      if (s < nK) fal_stage<NI>(src, dst, lds, s, s, RS, SB);
    for (int s = 0; s < nK; ++s) {
      const int ahead = nK - 1 - s;  // stages issued after s (capped at NST - 2)
      if (NST >= 4 && ahead >= 2)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NI) : "memory");
      else if (NST >= 3 && ahead >= 1)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NI) : "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      if (s + NST - 1 < nK) fal_stage<NI>(src, dst, lds, s + NST - 1, (s + NST - 1) % NST, RS, SB);
      const char* st = lds + (s % NST) * SB;
#pragma unroll
      for (int kk = 0; kk < KS; ++kk) {
        bf16x8 a[TI], b[TJ];
#pragma unroll
        for (int i = 0; i < TI; ++i) a[i] = *reinterpret_cast<const bf16x8*>(st + (wm * TM + i * 32) * RS + koff[kk]);
#pragma unroll
        for (int j = 0; j < TJ; ++j)
          b[j] = *reinterpret_cast<const bf16x8*>(st + (BM + wn * TN + j * 32) * RS + koff[kk]);
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
          for (int j = 0; j < TJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
      }
    }
    __syncthreads();  // every wave is done with the stages (the last wait was vmcnt(0))

    // epilogue: BM/32 passes of 32 rows through an fp32 [32][BN] LDS image; each wave then finishes 4 whole rows
    constexpr int VW = BN / 64;  // output columns per lane (bf16 kinds) / 8 for the full-row kinds
    float* E = reinterpret_cast<float*>(lds);
    f32x4 bv[2], gv[2], bev[2], wv[2];
    typedef __attribute__((ext_vector_type(2))) float f32x2;
    f32x2 bv2 = {};
    if constexpr (VW == 2) {
      bv2 = *reinterpret_cast<const f32x2*>(p.bias + col0 + 2 * lane);
    } else {
#pragma unroll
      for (int c = 0; c < VW / 4; ++c) bv[c] = *reinterpret_cast<const f32x4*>(p.bias + col0 + 256 * c + 4 * lane);
    }
    constexpr bool LN = EPI == kEpiResLn || EPI == kEpiResLnW;  // full-row kinds that read H and normalise
    if constexpr (LN) {
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        gv[c] = *reinterpret_cast<const f32x4*>(p.g + 256 * c + 4 * lane);
        bev[c] = *reinterpret_cast<const f32x4*>(p.b + 256 * c + 4 * lane);
      }
    }
    if constexpr (EPI == kEpiResOut || EPI == kEpiResLnW) {
#pragma unroll
      for (int c = 0; c < 2; ++c) wv[c] = *reinterpret_cast<const f32x4*>(p.wout + 256 * c + 4 * lane);
    }
#pragma unroll
    for (int ps = 0; ps < BM / 32; ++ps) {
      // the residual rows this wave finishes in this pass, loaded ahead of the LDS exchange
      f32x4 hv[4][2];
      float hw[4];
      if constexpr (LN) {
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const long gr = row0 + 32 * ps + 4 * w + rr;
#pragma unroll
          for (int c = 0; c < 2; ++c) hv[rr][c] = *reinterpret_cast<const f32x4*>(p.H + gr * kD + 256 * c + 4 * lane);
        }
      }
      if constexpr (EPI == kEpiResOut) {
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) hw[rr] = p.HW[row0 + 32 * ps + 4 * w + rr];
      }
      if (wm == ps / TI) {
#pragma unroll
        for (int j = 0; j < TJ; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            E[((r & 3) + 8 * (r >> 2) + 4 * h) * BN + wn * TN + j * 32 + lr] = acc[ps % TI][j][r];
      }
      __syncthreads();
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int row = 4 * w + rr;
        const long gr = row0 + 32 * ps + row;
        const float* er = E + row * BN;
        if constexpr (EPI == kEpiBf16 || EPI == kEpiReluBf16) {
          if constexpr (VW == 2) {
            f32x2 v = *reinterpret_cast<const f32x2*>(er + 2 * lane) + bv2;
            if constexpr (EPI == kEpiReluBf16) v = f32x2{fmaxf(v[0], 0.0f), fmaxf(v[1], 0.0f)};
            if (gr < p.M) *reinterpret_cast<unsigned*>(p.Y + gr * p.N + col0 + 2 * lane) = pk_bf16(v[0], v[1]);
          } else {
            f32x4 v = *reinterpret_cast<const f32x4*>(er + 4 * lane) + bv[0];
            if constexpr (EPI == kEpiReluBf16)
#pragma unroll
              for (int c = 0; c < 4; ++c) v[c] = fmaxf(v[c], 0.0f);
            if (FAL_DIAG == 1)
              asm volatile("" ::"v"(v[0] + v[1] + v[2] + v[3]));
            else if (gr < p.M)
              st_bf16x4(p.Y + gr * p.N + col0 + 4 * lane, v);
          }
        } else {
          f32x4 v[2];
          float s = 0.0f;
#pragma unroll
          for (int c = 0; c < 2; ++c) {
            v[c] = *reinterpret_cast<const f32x4*>(er + 256 * c + 4 * lane) + bv[c];
            if constexpr (LN) v[c] += hv[rr][c];
            s += (v[c][0] + v[c][1]) + (v[c][2] + v[c][3]);
          }
          if constexpr (LN) {
            const float mean = wave_sum(s) * (1.0f / kD);
            float q = 0.0f;
#pragma unroll
            for (int c = 0; c < 2; ++c)
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                const float d = v[c][e] - mean;
                q = fmaf(d, d, q);
              }
            const float rstd = 1.0f / sqrtf(wave_sum(q) * (1.0f / kD) + 1e-5f);
            if constexpr (EPI == kEpiResLnW) {
              float y = 0.0f;
#pragma unroll
              for (int c = 0; c < 2; ++c)
#pragma unroll
                for (int e = 0; e < 4; ++e) y = fmaf(v[c][e], wv[c][e], y);
              y = wave_sum(y);
              if (lane == 0 && gr < p.M) p.HW[gr] = y;
            }
            if (gr < p.M) {
#pragma unroll
              for (int c = 0; c < 2; ++c) {
                if constexpr (EPI == kEpiResLn) *reinterpret_cast<f32x4*>(p.H + gr * kD + 256 * c + 4 * lane) = v[c];
                f32x4 y;
#pragma unroll
                for (int e = 0; e < 4; ++e) y[e] = fmaf((v[c][e] - mean) * rstd, gv[c][e], bev[c][e]);
                st_bf16x4(p.Y + gr * kD + 256 * c + 4 * lane, y);
              }
            }
          } else {  // output layer: one scalar per token; x += y on the state tokens
            float y = 0.0f;
#pragma unroll
            for (int c = 0; c < 2; ++c)
#pragma unroll
              for (int e = 0; e < 4; ++e) y = fmaf(v[c][e], wv[c][e], y);
            y = wave_sum(y) + hw[rr] + p.bout;
            if (lane == 0 && gr < p.M && (int)(gr % p.L) < p.nx) p.XU[gr] += y;
          }
        }
      }
      __syncthreads();
    }
  }  // tiles
}

// Self-attention of one sample per workgroup, one head per wave (head dim HD = 512 / heads), on 32x32x16 MFMAs
// with the L <= 64 tokens padded to 64: S^T = K Q^T (keys on the accumulator rows, queries on the lanes), the
// softmax over the keys in-lane plus one lane-half swap, then O = P V with the accumulator tiles of P^T (packed to
// bf16) as the A operand as they stand; V reaches the B operand through a per-wave V^T image in LDS, read in the
// accumulator's permuted key order.
template <int HD>
__global__ __launch_bounds__(64 * (kD / HD)) void fal_attn_kernel(const __bf16* __restrict__ QKV, __bf16* O, int L) {
  constexpr int QP = 3 * kD, C8 = HD / 8, DT = HD / 32;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, lane = tid & 63, hd = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lr = lane & 31, h = lane >> 5;
  const long r0 = (long)blockIdx.x * L;
  const __bf16* base = QKV + r0 * QP;
  char* Vt = lds + hd * HD * kVtS;
  // V^T[d][key]: lane = key, one 16-B piece of its row per iteration, 8 d rows written (keys >= L zero)
#pragma unroll 4
  for (int d8 = 0; d8 < C8; ++d8) {
    bf16x8 v = lane < L ? *reinterpret_cast<const bf16x8*>(base + (long)lane * QP + 2 * kD + hd * HD + 8 * d8)
                        : bf16x8{};
#pragma unroll
    for (int e = 0; e < 8; ++e) *reinterpret_cast<__bf16*>(Vt + (8 * d8 + e) * kVtS + 2 * lane) = v[e];
  }
  // S^T tiles [key tile][query tile]
  f32x16 st[2][2];
#pragma unroll
  for (int jt = 0; jt < 2; ++jt)
#pragma unroll
    for (int it = 0; it < 2; ++it) st[jt][it] = f32x16{};
#pragma unroll
  for (int ds = 0; ds < HD / 16; ++ds) {
    bf16x8 kf[2], qf[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const long row = (long)(32 * t + lr) * QP + hd * HD + 16 * ds + 8 * h;
      kf[t] = *reinterpret_cast<const bf16x8*>(base + row + kD);
      qf[t] = *reinterpret_cast<const bf16x8*>(base + row);
    }
#pragma unroll
    for (int jt = 0; jt < 2; ++jt)
#pragma unroll
      for (int it = 0; it < 2; ++it) st[jt][it] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf[jt], qf[it], st[jt][it], 0, 0, 0);
  }
  // softmax over keys j = 32 jt + (r & 3) + 8 (r >> 2) + 4 h for query column 32 it + lr; P^T as bf16 A fragments
  bf16x8 pa[2][2][2];  // [query tile][key tile][k-step]
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    float m = -INFINITY;
#pragma unroll
    for (int jt = 0; jt < 2; ++jt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int j = 32 * jt + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (j >= L) st[jt][it][r] = -INFINITY;
        m = fmaxf(m, st[jt][it][r]);
      }
    m = max32(m);
    float sum = 0.0f;
#pragma unroll
    for (int jt = 0; jt < 2; ++jt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float e = __expf(st[jt][it][r] - m);
        st[jt][it][r] = e;
        sum += e;
      }
    sum = sum32(sum);
    const float inv = 1.0f / sum;
#pragma unroll
    for (int jt = 0; jt < 2; ++jt)
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int e = 0; e < 8; ++e) pa[it][jt][s][e] = (__bf16)(st[jt][it][8 * s + e] * inv);
  }
  __syncthreads();  // V^T written (each wave reads its own image; the barrier orders the lanes' LDS writes)
  f32x16 o[2][DT];
#pragma unroll
  for (int it = 0; it < 2; ++it)
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) o[it][dt] = f32x16{};
#pragma unroll
  for (int jt = 0; jt < 2; ++jt)
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        const char* vr = Vt + (32 * dt + lr) * kVtS + 2 * (32 * jt + 16 * s + 4 * h);
        const bf16x4 v0 = *reinterpret_cast<const bf16x4*>(vr), v1 = *reinterpret_cast<const bf16x4*>(vr + 16);
        const bf16x8 vb = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
#pragma unroll
        for (int it = 0; it < 2; ++it) o[it][dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pa[it][jt][s], vb, o[it][dt], 0, 0, 0);
      }
  // O[query][hd * HD + d], bf16, query rows < L
  __bf16* ob = O + r0 * kD + hd * HD + lr;
#pragma unroll
  for (int it = 0; it < 2; ++it)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int i = 32 * it + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (i < L) {
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) ob[(long)i * kD + 32 * dt] = (__bf16)o[it][dt][r];
      }
    }
}

struct FalEnc {
  float* XU;      // [rows] token input scalars
  float* H;       // [rows][512]
  __bf16* XN;     // [rows][512]
  float* cost;    // [B*K] running-cost accumulators
  const char* img;
  int we, be, ge, bte, pos, ln1g, ln1b;
  float enc_mw, enc_mb, enc_vw, enc_cwb, enc_vb;
  int L;
};

namespace {

__device__ __forceinline__ float fal_cost(const SolveArgs& a, const float* x, int b, float u0, float usq, int t1) {
  float cx[MPPI_CTX_MAX];
#pragma unroll
  for (int i = 0; i < MPPI_CTX_MAX; ++i) cx[i] = a.ctx ? a.ctx[(long)b * MPPI_CTX_MAX + i] : a.ctx_default[i];
  return fa_cost(a.cost_kind, x, u0, usq, cx, t1);
}

}  // namespace

// Step t's inputs, one sample per workgroup: (t > 0) the running cost of step t-1 on x_t with u_{t-1} still in the
// control tokens, then u_t = clamp(U + eps) into them, then every token's encoding (closed-form LayerNorm moments of
// w v + b) into H and layer 0's LayerNorm1 into XN; one wave per token row, 8 features per lane.
__global__ __launch_bounds__(256) void fal_encode_kernel(SolveArgs a, FalEnc e, int t) {
  const int gk = blockIdx.x, b = gk / a.K, k = gk - b * a.K;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, nx = a.nx, nu = a.nu, L = e.L;
  const long r0 = (long)gk * L;
  float* XU = e.XU + r0;
  if (t == 0) {
    if (a.kclock && tid == 0) {  // the launch clock's start (fal_finish_kernel records the end and advances it)
      const unsigned slot = (unsigned)(*a.kclock_ctr & (kClockSlots - 1));
      atomicMin(a.kclock + 2 * slot, (unsigned long long)wall_clock64());
    }
    if (gk == 0 && tid == 0) *a.status = 0u;
    if (tid < nx) XU[tid] = a.x0[(long)b * nx + tid];
    if (tid == 0) e.cost[gk] = 0.0f;
  } else if (tid == 0) {
    float usq = 0.0f;
    for (int j = 0; j < nu; ++j) usq = fmaf(XU[nx + j], XU[nx + j], usq);
    e.cost[gk] += fal_cost(a, XU, b, XU[nx], usq, t);
  }
  __syncthreads();
  if (tid < nu) {
    float u = a.U[((long)b * nu + tid) * a.H + t] + a.noise[(((long)b * nu + tid) * a.H + t) * a.Kp + k];
    if (a.ctrl_clamp > 0.0f) u = fminf(a.ctrl_clamp, fmaxf(-a.ctrl_clamp, u));
    XU[nx + tid] = u;
  }
  __syncthreads();
  auto vec = [&](int off, int c) { return *reinterpret_cast<const f32x4*>(e.img + off + 4 * (256 * c + 4 * lane)); };
  f32x4 we[2], be[2], ge[2], bt[2], g1[2], b1[2];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    we[c] = vec(e.we, c);
    be[c] = vec(e.be, c);
    ge[c] = vec(e.ge, c);
    bt[c] = vec(e.bte, c);
    g1[c] = vec(e.ln1g, c);
    b1[c] = vec(e.ln1b, c);
  }
  for (int i = w; i < L; i += 4) {
    const float v = XU[i];
    const float var = fmaxf(fmaf(v, fmaf(v, e.enc_vw, 2.0f * e.enc_cwb), e.enc_vb), 0.0f);
    const float em = fmaf(v, e.enc_mw, e.enc_mb), er = 1.0f / sqrtf(var + 1e-5f);
    f32x4 hv[2];
    float s = 0.0f;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const f32x4 pe = vec(e.pos + i * kD * 4, c);
#pragma unroll
      for (int q = 0; q < 4; ++q)
        hv[c][q] = fmaxf(fmaf((fmaf(we[c][q], v, be[c][q]) - em) * er, ge[c][q], bt[c][q]), 0.0f) + pe[q];
      s += (hv[c][0] + hv[c][1]) + (hv[c][2] + hv[c][3]);
      *reinterpret_cast<f32x4*>(e.H + (r0 + i) * kD + 256 * c + 4 * lane) = hv[c];
    }
    const float mean = wave_sum(s) * (1.0f / kD);
    float q2 = 0.0f;
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float d = hv[c][q] - mean;
        q2 = fmaf(d, d, q2);
      }
    const float rstd = 1.0f / sqrtf(wave_sum(q2) * (1.0f / kD) + 1e-5f);
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      f32x4 y;
#pragma unroll
      for (int q = 0; q < 4; ++q) y[q] = fmaf((hv[c][q] - mean) * rstd, g1[c][q], b1[c][q]);
      st_bf16x4(e.XN + (r0 + i) * kD + 256 * c + 4 * lane, y);
    }
  }
}

// After the last step: the running cost of step H-1 on x_H, the terminal cost, costs[b][k], the env-step state.
__global__ __launch_bounds__(256) void fal_finish_kernel(SolveArgs a, FalEnc e) {
  const KClock kc = kclock_begin(a);
  const int gk = blockIdx.x * 256 + threadIdx.x, nx = a.nx, nu = a.nu;
  if (gk < a.B * a.K) {
    const int b = gk / a.K, k = gk - b * a.K;
    const float* XU = e.XU + (long)gk * e.L;
    float usq = 0.0f;
    for (int j = 0; j < nu; ++j) usq = fmaf(XU[nx + j], XU[nx + j], usq);
    float cost = e.cost[gk] + fal_cost(a, XU, b, XU[nx], usq, a.H);
    if (a.terminal_weight != 0.0f) cost += a.terminal_weight * fal_cost(a, XU, b, 0.0f, 0.0f, a.H);
    a.costs[(long)b * a.Kp + k] = isfinite(cost) ? cost : INFINITY;
    if (a.xout && k == 0)
      for (int i = 0; i < nx; ++i) a.xout[(long)b * nx + i] = XU[i];
  }
  __syncthreads();
  kclock_record(a, kc);
}

namespace {

template <int BM, int BN, int BK, int NST>
constexpr int gemm_lds() {
  constexpr int stages = NST * (BM + BN) * BK * 2, epi = 32 * BN * 4;
  return stages > epi ? stages : epi;
}

template <int BM, int BN, int BK, int NST, int EPI>
hipError_t launch_gemm(const FalGemm& g, long rows_p, hipStream_t s) {
  auto kern = fal_gemm_kernel<BM, BN, BK, NST, EPI>;
  constexpr int lds = gemm_lds<BM, BN, BK, NST>();
  // the attribute on every launch (cheap, and per device: a process may drive several GPUs)
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  if (e != hipSuccess) return e;
  // resident workgroups on the current device (CUs x workgroups per CU), a multiple of 8; cached per device
  constexpr int kMaxDev = 64;
  static std::atomic<int> slot_cache[kMaxDev];
  int dev = 0, per = 0;
  e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  int slots = dev >= 0 && dev < kMaxDev ? slot_cache[dev].load(std::memory_order_relaxed) : 0;
  if (!slots) {
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, reinterpret_cast<const void*>(kern), 512, lds);
    if (e != hipSuccess) return e;
    slots = (current_device_cus() * (per > 0 ? per : 1)) / 8 * 8;
    if (slots < 8) slots = 8;
    if (dev >= 0 && dev < kMaxDev) slot_cache[dev].store(slots, std::memory_order_relaxed);
  }
  if (g.Kd % BK != 0 || g.N % BN != 0 || rows_p % BM != 0) return hipErrorInvalidValue;
  FalGemm a = g;
  a.tiles = (int)(rows_p / BM * (g.N / BN));
  const int grid = a.tiles < slots ? (a.tiles + 7) / 8 * 8 : slots;
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(512), lds, s, a);
  return hipGetLastError();
}

// GEMM shapes (build-time knobs for same-box A/B: -DFAL_PROJ=BM,BN,BK,NST for the bf16-output GEMMs, -DFAL_RES=...
// for the full-row residual + LayerNorm GEMMs)
#ifndef FAL_PROJ
#define FAL_PROJ 128, 256, 32, 3
#endif
#ifndef FAL_RES
#define FAL_RES 128, 512, 32, 3
#endif
template <int EPI>
hipError_t launch_proj(const FalGemm& g, long rows_p, hipStream_t s) { return launch_gemm<FAL_PROJ, EPI>(g, rows_p, s); }
template <int EPI>
hipError_t launch_res(const FalGemm& g, long rows_p, hipStream_t s) { return launch_gemm<FAL_RES, EPI>(g, rows_p, s); }

template <int HD>
hipError_t launch_attn(const __bf16* qkv, __bf16* o, int L, int samples, hipStream_t s) {
  auto kern = fal_attn_kernel<HD>;
  constexpr int lds = (kD / HD) * HD * kVtS;
  const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(kern, dim3(samples), dim3(64 * (kD / HD)), lds, s, qkv, o, L);
  return hipGetLastError();
}

}  // namespace

// token rows padded to the GEMM tile, plus 64 rows so the attention's 64-token windows stay inside the buffers
long fa_layered_rows(long rows) { return (rows + kBM - 1) / kBM * kBM + 64; }

size_t fa_layered_ws_bytes(long rows) {
  const long R = fa_layered_rows(rows);
  return (size_t)R * (4 + 4 + kD * 4 + kD * 2 + 3 * kD * 2 + 4 * kD * 2) + (size_t)rows * 4 + 1024;
}

hipError_t launch_fa_layered(const SolveArgs& a, const FaNet& n, hipStream_t s) {
  const long M = (long)a.B * a.K * n.L, Mp = (M + kBM - 1) / kBM * kBM, R = fa_layered_rows(M);
  if (!n.lay || !n.d_ws || M > n.ws_rows || n.D != kD || n.L > 64 || (n.nh != 4 && n.nh != 8))
    return hipErrorInvalidValue;
  note_kernel("fa_layered");
  char* ws = reinterpret_cast<char*>(n.d_ws);
  const long RW = fa_layered_rows(n.ws_rows);  // the workspace's own carve (independent of this batch)
  float* XU = reinterpret_cast<float*>(ws);
  float* Hb = reinterpret_cast<float*>(ws + RW * 4);
  __bf16* XN = reinterpret_cast<__bf16*>(ws + RW * (4 + kD * 4));
  __bf16* QKV = reinterpret_cast<__bf16*>(ws + RW * (4 + kD * 4 + kD * 2));
  __bf16* F = reinterpret_cast<__bf16*>(ws + RW * (4 + kD * 4 + kD * 2 + 3 * kD * 2));
  float* HWb = reinterpret_cast<float*>(ws + RW * (4 + kD * 4 + kD * 2 + 3 * kD * 2 + 4 * kD * 2));
  float* cost = reinterpret_cast<float*>(ws + RW * (4 + 4 + kD * 4 + kD * 2 + 3 * kD * 2 + 4 * kD * 2));
  (void)R;
  const char* img = reinterpret_cast<const char*>(n.d_img);
  auto mat = [&](int off) { return reinterpret_cast<const __bf16*>(img + off); };
  auto vecp = [&](int off) { return reinterpret_cast<const float*>(img + off); };
  FalEnc e{XU, Hb, XN, cost, img, n.we, n.be, n.ge, n.bte, n.pos, n.ln1g[0], n.ln1b[0],
           n.enc_mw, n.enc_mb, n.enc_vw, n.enc_cwb, n.enc_vb, n.L};
  const int samples = a.B * a.K;
  hipError_t err;
  for (int t = 0; t < a.H; ++t) {
    hipLaunchKernelGGL(fal_encode_kernel, dim3(samples), dim3(256), 0, s, a, e, t);
    if ((err = hipGetLastError()) != hipSuccess) return err;
    for (int l = 0; l < n.nlayers; ++l) {
      const bool last = l + 1 == n.nlayers;
      FalGemm g{};
      g.L = n.L;
      g.nx = a.nx;
      g.M = (int)M;
      // Q | K | V
      g.X = XN;
      g.W = mat(n.lwqkv[l]);
      g.Kd = kD;
      g.N = 3 * kD;
      g.bias = vecp(n.lbqkv[l]);
      g.Y = QKV;
      if ((err = launch_proj<kEpiBf16>(g, Mp, s)) != hipSuccess) return err;
      // attention -> O (into XN: the Q|K|V GEMM has consumed it)
      err = n.nh == 4 ? launch_attn<128>(QKV, XN, n.L, samples, s) : launch_attn<64>(QKV, XN, n.L, samples, s);
      if (err != hipSuccess) return err;
      // out-proj + residual + LayerNorm2
      g.X = XN;
      g.W = mat(n.lwo[l]);
      g.N = kD;
      g.bias = vecp(n.bo[l]);
      g.Y = XN;
      g.H = Hb;
      g.g = vecp(n.ln2g[l]);
      g.b = vecp(n.ln2b[l]);
      g.wout = vecp(n.wout);
      g.HW = HWb;
      if ((err = last ? launch_res<kEpiResLnW>(g, Mp, s) : launch_res<kEpiResLn>(g, Mp, s)) != hipSuccess) return err;
      // FFN1 + ReLU
      g.X = XN;
      g.W = mat(n.lw1[l]);
      g.N = 4 * kD;
      g.bias = vecp(n.b1[l]);
      g.Y = F;
      if ((err = launch_proj<kEpiReluBf16>(g, Mp, s)) != hipSuccess) return err;
      // FFN2 + residual + (next LayerNorm1 | output layer)
      g.X = F;
      g.W = mat(n.lw2[l]);
      g.Kd = 4 * kD;
      g.N = kD;
      g.bias = vecp(n.b2[l]);
      g.Y = XN;
      g.H = Hb;
      if (!last) {
        g.g = vecp(n.ln1g[l + 1]);
        g.b = vecp(n.ln1b[l + 1]);
        err = launch_res<kEpiResLn>(g, Mp, s);
      } else {
        g.wout = vecp(n.wout);
        g.bout = n.b_out;
        g.XU = XU;
        err = launch_res<kEpiResOut>(g, Mp, s);
      }
      if (err != hipSuccess) return err;
    }
  }
  hipLaunchKernelGGL(fal_finish_kernel, dim3((samples + 255) / 256), dim3(256), 0, s, a, e);
  return hipGetLastError();
}

}  // namespace mppi
