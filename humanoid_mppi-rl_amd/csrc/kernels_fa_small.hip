// FeatureAttention rollout for small nets (hidden 64, <= 16 tokens, bf16; the cartpole estimator's net):
// fa_small_kernel.  Its own translation unit so it builds with -fno-slp-vectorize (build.py PER_FILE_FLAGS):
// packed-f32 VALU beside its MFMAs measured slower for this kernel, faster for the general kernels.
#include <cstdlib>

#include "fa_common.h"

namespace mppi {

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
// relu(lo | hi) packed to bf16: the ReLU as v_pk_max_i16 on the packed bit patterns after the conversion (a negative
// bf16 is a negative int16), 4 instead of 8 VALU per 8 values; bit-identical for every non-NaN input (fc_common.h)
__device__ __forceinline__ bf16x8 fs_pack8_relu(const f32x4& lo, const f32x4& hi) {
  typedef __attribute__((ext_vector_type(2))) float f2;
  typedef __attribute__((ext_vector_type(2))) __bf16 b2;
  typedef __attribute__((ext_vector_type(2))) short i2;
  auto pk = [](float a, float b) {
    const b2 p = __builtin_convertvector(f2{a, b}, b2);
    return __builtin_bit_cast(unsigned, __builtin_elementwise_max(__builtin_bit_cast(i2, p), i2{0, 0}));
  };
  typedef __attribute__((ext_vector_type(4))) unsigned u4;
  return __builtin_bit_cast(bf16x8, u4{pk(lo[0], lo[1]), pk(lo[2], lo[3]), pk(hi[0], hi[1]), pk(hi[2], hi[3])});
}
__device__ __forceinline__ s16x4 fs_pack4(const f32x4& v) {
  return __builtin_bit_cast(s16x4, bf16x4{(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]});
}
__device__ __forceinline__ f32x4 fs_mma32(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
// max(a, b) / ReLU as one v_med3_f32 against FLT_MAX: fmaxf on an MFMA or permlane result costs an extra
// v_max_f32 v, v, v per operand (IEEE-mode NaN quieting), and a +inf bound is folded back into fmaxf by the compiler
__device__ __forceinline__ float fs_max(float a, float b) { return __builtin_amdgcn_fmed3f(a, b, 3.402823466e38f); }
__device__ __forceinline__ float fs_group_max(float v) {
  auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  const float s = fs_max(__uint_as_float(p[0]), __uint_as_float(p[1]));
  auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(s), __float_as_uint(s), false, false);
  return fs_max(__uint_as_float(q[0]), __uint_as_float(q[1]));
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

// HPW: attention heads (and FFN hidden slices) per wave, 1 or 2: 4 / HPW waves per workgroup.  The residual-stream
// work (encoding, LayerNorms, out-proj, the FFN2 partial sum, output layer) is repeated by every wave, so fewer waves
// per tile repeat it less, at fewer waves per SIMD.
template <int NT, int HPW>
__global__ __launch_bounds__(256 / HPW) __attribute__((amdgpu_waves_per_eu(HPW == 1 ? 3 : 2, HPW == 1 ? 3 : 2)))
void fa_small_kernel(SolveArgs a, FaArgs f) {
  constexpr int D = 64, NW = 4 / HPW, NTH = 64 * NW;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const KClock kc = kclock_begin(a);
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, n = lane & 15;
  const int h = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave: attention heads / hidden slices HPW h + j
  const int L = f.L, nx = f.nx, nu = f.nu;
  const int Gt = 16 / L, G = NT * Gt;  // samples per tile, per workgroup
  const int gps = (a.K + G - 1) / G;   // workgroups per solve
  const int b = blockIdx.x / gps;
  const int k0 = (blockIdx.x - b * gps) * G;
  if (blockIdx.x == 0 && tid == 0) *a.status = 0u;

  char* VEC = lds;  // the image's fp32 vectors [0, vec_lds)
  char* WO = lds + f.vec_lds;  // out-proj fragments, layer l at l * kFsWoBytes
  f32x4* XP = reinterpret_cast<f32x4*>(WO + f.nlayers * kFsWoBytes);
  char* OB = reinterpret_cast<char*>(XP) + fa_small_xp_bytes(NT);  // (the regions must not alias: a wave writes
  // O of the next layer and XU while slower waves still read XP)
  float* XU = reinterpret_cast<float*>(OB + fa_small_o_bytes(NT));
  for (int i = tid; i < f.vec_lds / 16; i += NTH) reinterpret_cast<int4*>(VEC)[i] = reinterpret_cast<const int4*>(f.img)[i];
  for (int l = 0; l < f.nlayers; ++l)
    for (int i = tid; i < kFsWoBytes / 16; i += NTH)
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
  // One pass: sum and sum of squares together (var = E[x^2] - mean^2, clamped at 0), then y = x rstd - mean rstd as
  // one fma per feature: a shorter chain and fewer VALU than mean -> squared deviations -> (x - mean) rstd, which
  // matters because the kernel is VALU-issue-bound and every wave runs every LayerNorm.  The cancellation error,
  // ~6e-8 (mean / std)^2 relative on the variance, stays far below the bf16 rounding of the output.
  auto layer_norm = [&](const f32x4 (&x)[4], bf16x8 (&xn)[2]) {
    float s0 = 0.0f, s1 = 0.0f, q0 = 0.0f, q1 = 0.0f;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      s0 += x[mt][0] + x[mt][1];
      s1 += x[mt][2] + x[mt][3];
      q0 = fmaf(x[mt][0], x[mt][0], fmaf(x[mt][1], x[mt][1], q0));
      q1 = fmaf(x[mt][2], x[mt][2], fmaf(x[mt][3], x[mt][3], q1));
    }
    float s = s0 + s1, q = q0 + q1;
    fa_group_sum2(s, q);
    const float mean = s * (1.0f / D);
    const float var = fmaxf(fmaf(-mean, mean, q * (1.0f / D)), 0.0f);
    const float rstd = __builtin_amdgcn_rsqf(var + 1e-5f);  // argument >= 1e-5
    const float nb = -mean * rstd;
    f32x4 y[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) y[mt][r] = fmaf(x[mt][r], rstd, nb);
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
  bf16x8 fq[HPW][2], fk[HPW][2], fv[HPW][2], f1[HPW][4][2], f2[HPW][4][2];
  auto load_attn = [&](int l) {
#pragma unroll
    for (int j = 0; j < HPW; ++j) {
      const int o = f.s_wqkv[l] + (HPW * h + j) * 6 * 1024;
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        fq[j][kb] = frag(o + kb * 1024);
        fk[j][kb] = frag(o + (2 + kb) * 1024);
        fv[j][kb] = frag(o + (4 + kb) * 1024);
      }
    }
  };
  auto load_ffn1 = [&](int l) {
#pragma unroll
    for (int j = 0; j < HPW; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) f1[j][i][kb] = frag(f.s_w1[l] + ((4 * (HPW * h + j) + i) * 2 + kb) * 1024);
  };
  auto load_ffn2 = [&](int l) {
#pragma unroll
    for (int j = 0; j < HPW; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) f2[j][i][kb] = frag(f.s_w2[l] + (i * 8 + 2 * (HPW * h + j) + kb) * 1024);
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
      // ---- pre-LN attention, heads HPW h + j of every tile
      f32x4 part[NT][4];
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        bf16x8 xn[2];
        layer_norm(res[nt], xn);
#pragma unroll
        for (int j = 0; j < HPW; ++j) {
          const int hd = HPW * h + j;
          const f32x4 bq = vec4(f.s_bqkv[l], 16 * hd + 4 * g), bk = vec4(f.s_bqkv[l], D + 16 * hd + 4 * g);
          const float bvv = vec1(f.s_bqkv[l], 2 * D + 16 * hd + n);
          f32x4 q = bq, kk = bk, v = {bvv, bvv, bvv, bvv};
#pragma unroll
          for (int kb = 0; kb < 2; ++kb) {
            q = fs_mma32(fq[j][kb], xn[kb], q);    // Q_hd^T [dim][token]
            kk = fs_mma32(fk[j][kb], xn[kb], kk);  // K_hd^T [dim][token]
            v = fs_mma32(xn[kb], fv[j][kb], v);    // V_hd [token][dim]
          }
          // S^T[key][query] = K Q^T (Q pre-scaled by 1/sqrt(16) on the host), softmax over the keys of query n
          f32x4 sc = fs_mma16(fs_pack4(kk), fs_pack4(q), f32x4{0.0f, 0.0f, 0.0f, 0.0f});
          float m = -INFINITY;
#pragma unroll
          for (int r = 0; r < 4; ++r) m = fs_max(m, kval[r] ? sc[r] : -INFINITY);
          m = fs_group_max(m);
          float sum = 0.0f;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            sc[r] = kval[r] ? __expf(sc[r] - m) : 0.0f;
            sum += sc[r];
          }
          sum = fa_group_sum(sum);
          const float inv = sum > 0.0f ? 1.0f / sum : 0.0f;
          // O_hd^T[dim][query] = V^T P^T (P normalised, bf16)
          const f32x4 o = fs_mma16(fs_pack4(v), fs_pack4(sc * inv), f32x4{0.0f, 0.0f, 0.0f, 0.0f});
          // O[query n][16 hd + 4 g + r]: this head's 4 features of row n (one 8-byte store)
          *reinterpret_cast<s16x4*>(OB + (nt * 16 + n) * kFsORow + (16 * hd + 4 * g) * 2) = fs_pack4(o);
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
      // ---- pre-LN FFN: hidden slices HPW h + j (64 rows each) from registers, their K-split share of the second GEMM
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        bf16x8 xn[2];
        layer_norm(res[nt], xn);
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) part[nt][mt] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int j = 0; j < HPW; ++j) {
          const int sl = HPW * h + j;
          f32x4 hid[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            hid[i] = vec4(f.s_b1[l], 64 * sl + 16 * i + 4 * g);
#pragma unroll
            for (int kb = 0; kb < 2; ++kb) hid[i] = fs_mma32(f1[j][i][kb], xn[kb], hid[i]);
          }
          const bf16x8 hb0 = fs_pack8_relu(hid[0], hid[1]), hb1 = fs_pack8_relu(hid[2], hid[3]);
#pragma unroll
          for (int mt = 0; mt < 4; ++mt)
            part[nt][mt] = fs_mma32(f2[j][mt][1], hb1, fs_mma32(f2[j][mt][0], hb0, part[nt][mt]));
        }
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
          res[nt][mt] += (NW == 4 ? (xp(0, nt, mt) + xp(1, nt, mt)) + (xp(2, nt, mt) + xp(3, nt, mt))
                                  : xp(0, nt, mt) + xp(1, nt, mt)) + b2;
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
        cost += fa_cost(a.cost_kind, xr, nu > 0 ? xr[nx] : 0.0f, usq, cx, t + 1);
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
    if (a.terminal_weight != 0.0f) cost += a.terminal_weight * fa_cost(a.cost_kind, XU + cbase, 0.0f, 0.0f, cx, a.H);
    const int ck = k0 + tid;
    if (ck < a.K) a.costs[(long)b * a.Kp + ck] = isfinite(cost) ? cost : INFINITY;
  }
  if (a.xout && k0 == 0 && h == 0 && g == 0 && rvalid && tok < nx && n < L)  // env step: sample 0's final state
    a.xout[(long)b * nx + tok] = xu[0];
}

template <int NT, int HPW>
static hipError_t launch_fa_small_t(const SolveArgs& a, const FaArgs& fa, hipStream_t stream) {
  const int G = NT * (16 / fa.L);
  if (G < 1) return hipErrorInvalidValue;
  const size_t lds = (size_t)fa.vec_lds + fa_small_lds(NT, fa.nlayers);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  auto kern = fa_small_kernel<NT, HPW>;
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)lds);
  if (e != hipSuccess) return e;
  const int gps = (a.K + G - 1) / G;
  hipLaunchKernelGGL(kern, dim3(gps * a.B), dim3(256 / HPW), lds, stream, a, fa);
  return hipGetLastError();
}

static int fa_small_hpw() {  // MPPI_FA_HPW=1|2 (read once)
  static const int v = [] {
    const char* e = getenv("MPPI_FA_HPW");
    return e && atoi(e) == 2 ? 2 : 1;
  }();
  return v;
}

hipError_t launch_fa_small(const SolveArgs& a, const FaArgs& fa, hipStream_t stream) {
  note_kernel("fa_small_kernel");
  return fa_small_hpw() == 2 ? launch_fa_small_t<1, 2>(a, fa, stream) : launch_fa_small_t<1, 1>(a, fa, stream);
}

#ifdef MPPI_STAMPS
int fa_small_stamps(unsigned long long* out, int reset) {
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
