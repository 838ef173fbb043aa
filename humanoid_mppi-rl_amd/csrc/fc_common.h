// fc-stack rollout definitions (kernels_fc.hip): network shapes in m-tiles, the bf16 / fp32 MFMA operand traits,
// lane-group sums, the per-wave layer helpers, the cost-ring chunk map and the per-group LDS layout.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "costs.h"
#include "mppi_internal.h"

namespace mppi {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(2))) float f32x2;
typedef __attribute__((ext_vector_type(2))) short i16x2;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;

constexpr int kSplit = 4;  // waves per sample group (M split)

// Network shapes in m-tiles of 16 rows (the last layer has 4 = the 64 state slots). IN_T = input tiles of
// layer 0 (4 state tiles [+ 2 control tiles]). State slot of state index i: i < QP ? i : 32 + (i - QP).
template <int ARCH>
struct Arch;
template <>
struct Arch<kArchCA> {  // folded CrossAttentionStatePredictor(28, 27, 21, 128), learning/model.py:157-202
  static constexpr int NL = 3, IN_T = 4, MT0 = 16, MT1 = 8, MT2 = 4;
  static constexpr bool LN0 = true;
  static constexpr int BLOCKS0 = 1;  // dense: the LayerNorm fold centres the rows (mppi_nets.cpp)
  static constexpr int QP = 28;
  static constexpr int REG_MASK = kCaRegMask;  // bf16: every layer's fragments in VGPRs (mppi_nets.cpp)
};
template <>
struct Arch<kArchMLP> {  // MLPStatePredictor(nx, nu, 128, hidden_layers=2), learning/model.py:6-46
  static constexpr int NL = 4, IN_T = 6, MT0 = 8, MT1 = 8, MT2 = 8;
  static constexpr bool LN0 = false;
  static constexpr int BLOCKS0 = 1;
  static constexpr int QP = 64;
  static constexpr int REG_MASK = kMlpRegMask;
};

struct FcArgs {
  const char* img;  // packed image in global memory
  int img_bytes, lds_bytes;
  int w_off[4], b_off[4];
  int lnb_off, ln_n;  // beta' of the folded LayerNorm (mppi_nets.cpp)
  int qp, qv;  // state slots: x[0, qp) -> [0, qp); x[qp, qp+qv) -> [32, 32+qv)
  int groups_per_block;
  int g_off;  // FcNet::g_off (the per-wave CA kernel's Gram fragments), -1: none
  int wave;   // FcNet::wave
  int w32_off;  // FcNet::w32_off
  int w32_bd;   // FcNet::w32_bd
  int w0bd_off, gbd_off;  // FcNet::w0bd_off, gbd_off
  int w32x3_off, w32x3_l1lo_off;  // FcNet::w32x3_off, w32x3_l1lo_off
  int wmx3_off, wmx3_lo_off;      // FcNet::wmx3_off, wmx3_lo_off
  int wm32x3_off, wm32x3_lo_off;  // FcNet::wm32x3_off, wm32x3_lo_off
  int x3_l1;                      // FcNet::x3_l1 (the probe's decision for this net)
  int w32f16_off;                 // FcNet::w32f16_off (fc_wave32_x3p_kernel's fp16 form image)
  int wmf16_off, wmf16_x_off;     // FcNet::wmf16_off, wmf16_x_off (fc_rollout_kernel_x3d's fp16 form)
  int wmf16_0_off;                // FcNet::wmf16_0_off
  int wmf16_0b_off;               // FcNet::wmf16_0b_off
  int x3_f16;                     // FcNet::x3_f16 (the probe's decision on the fp16 form)
  int x3_route;                   // FcNet::x3_route (the probe's direct launches: 1 fc_wave32_x3p_kernel, 2 _x3h)
};

// kernels_fc_x3h.hip: whether the few-tiles shards' fp16-form kernel runs this net (the engine's probe checks it too)
bool fc_x3h_wanted(const SolveArgs& a, const FcArgs& fa);

// ------------------------------------------------------------------------------------------------ precision traits

template <int PREC>
struct P;
template <>
struct P<MPPI_PREC_BF16> {
  using Bop = bf16x8;                     // one B-operand k-step per lane (32 features)
  using Wt = bf16x8;                      // one A fragment per lane
  static constexpr int TILE_BYTES = 512;  // one 16-row tile in the exchange buffer (64 lanes x 8 B)
  static constexpr int KS(int mti) { return mti / 2; }
  __device__ static void put_tile(char* buf, int mt, int lane, const f32x4& v) {
    bf16x4 h = {(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
    *reinterpret_cast<bf16x4*>(buf + (mt >> 1) * 1024 + lane * 16 + (mt & 1) * 8) = h;
  }
  // relu(v) stored as bf16: the ReLU on the packed bf16 bit patterns, after the conversion, as two v_pk_max_i16 (a
  // negative bf16 has the sign bit set, i.e. is a negative int16; max(bits, 0) maps it and -0 to +0 and keeps every
  // positive value) instead of four v_med3_f32 before it: bit-identical for every non-NaN input
  __device__ static void put_tile_relu(char* buf, int mt, int lane, const f32x4& v) {
    auto pk = [](float a, float b) {  // one v_cvt_pk_bf16_f32, then one v_pk_max_i16
      const bf16x2 p = __builtin_convertvector(f32x2{a, b}, bf16x2);
      return __builtin_bit_cast(unsigned, __builtin_elementwise_max(__builtin_bit_cast(i16x2, p), i16x2{0, 0}));
    };
    *reinterpret_cast<uint2*>(buf + (mt >> 1) * 1024 + lane * 16 + (mt & 1) * 8) = make_uint2(pk(v[0], v[1]), pk(v[2], v[3]));
  }
  __device__ static Bop get_ks(const char* buf, int ks, int lane) {
    return *reinterpret_cast<const Bop*>(buf + ks * 1024 + lane * 16);
  }
  __device__ static f32x4 mma(const Wt& a, const Bop& b, const f32x4& c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
  // control tiles (registers) as B operands: one bf16 k-step from u tiles {0,1}
  __device__ static void put_u(Bop* bin, const f32x4 (&u)[2]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      bin[0][j] = (__bf16)u[0][j];
      bin[0][4 + j] = (__bf16)u[1][j];
    }
  }
};
template <>
struct P<MPPI_PREC_FP32> {
  using Bop = float;  // one B-operand k-step per lane (4 features)
  using Wt = float;
  static constexpr int TILE_BYTES = 1024;  // 64 lanes x 16 B
  static constexpr int KS(int mti) { return mti * 4; }
  __device__ static void put_tile(char* buf, int mt, int lane, const f32x4& v) {
    *reinterpret_cast<f32x4*>(buf + mt * 1024 + lane * 16) = v;
  }
  __device__ static void put_tile_relu(char* buf, int mt, int lane, const f32x4& v);  // after relu(), below
  __device__ static Bop get_ks(const char* buf, int ks, int lane) {
    return *reinterpret_cast<const float*>(buf + (ks >> 2) * 1024 + lane * 16 + (ks & 3) * 4);
  }
  __device__ static f32x4 mma(const Wt& a, const Bop& b, const f32x4& c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  }
  __device__ static void put_u(Bop* bin, const f32x4 (&u)[2]) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) bin[4 * i + r] = u[i][r];
  }
};

// Split bf16 (MPPI_PREC_BF16X3, fp32-accurate): every weight and activation is a bf16 pair v ~ hi + lo (hi = bf16(v),
// lo = bf16(v - hi): 16 significant bits), and W a = W_hi a_hi + W_hi a_lo + W_lo a_hi (the W_lo a_lo term, ~2^-16 of
// the product, dropped) on three v_mfma_f32_16x16x32_bf16 into one fp32 accumulator, small terms first.  The same k
// layout as bf16; the exchange holds a hi plane and a lo plane per k-step (1 KiB each).
struct BX3 {
  bf16x8 hi, lo;
};
// Layer 1 of the split humanoid CA with two products instead of three (every CA kernel of the split mode, per-wave and
// M-split): W1 = W1_hi + W1_lo against the hi part of its (ReLU'd layer-0) operand only, W1_hi a_lo dropped.  CPU
// emulation against the fp32 oracle over config #4's 64 logged states with checkpoints/model_cross.pth
// (tools/x3_error_budget.py, profiles/r05_x3_error_budget.txt): costs within 4.95e-5 of it at H = 64 (three products
// on every layer: 1.5e-6); the error grows with the horizon (1.1e-4 at H = 96, 4.3e-4 at 200) and depends on the
// weights, so the two-product form is a CHECKED property of the loaded net: mppi_api.hip x3_probe runs the first
// solve's states through both forms and keeps two products only if their costs agree within kX3ProbeTol, and never
// beyond kX3TwoTermMaxH.  Any other layer with two products, or layer 1 without W1_lo, exceeds 1e-4 already at H = 64
// on model_cross, and so does every layer of the MLP, which keeps three.  It takes 64 of the per-wave kernels' 306
// MFMAs per wave-step (M-split: 32 of 168) and layer 0's lo conversions.  MPPI_X3_L1_TERMS=3 / =2 (read per launch)
// forces three / two products without a probe (A/B and tests).
constexpr int kX3TwoTermMaxH = 64;
constexpr float kX3ProbeTol = 7.5e-5f;  // 3/4 of the fp32-accurate bar (costs rtol 1e-4 against the fp32 oracle);
                                        // model_cross.pth on config #4's logged states: 4.95e-5 (CPU emulation)
inline int x3_l1_env() {
  const char* e = std::getenv("MPPI_X3_L1_TERMS");
  return e && (e[0] == '2' || e[0] == '3') ? e[0] - '0' : 0;
}
inline int x3_l1_terms(int H, int decided) {
  if (const int f = x3_l1_env()) return f;
  return H <= kX3TwoTermMaxH && decided == 2 ? 2 : 3;
}
// The fp16 form of the split CA (L1T == 1 in the per-wave kernels, F16 in fc_rollout_kernel_x3d): layer 1 as ONE fp16
// MFMA product per (tile, k-step), fp16 W1 against the fp16 ReLU'd layer-0 output, and the last layer as two (fp16 W hi
// + lo against fp16 activations); the per-wave kernels (fc_wave32_x3p_kernel, fc_wave32_x3_kernel) take layer 0 and the
// statistic to fp16 W hi + lo against ONE fp16 operand too (MPPI_X3_F16_L0: the state rounded to fp16, -mu as an fp16
// pair in two slots), fc_rollout_kernel_x3d keeps them bf16x3.  fp16's 11-bit significand makes one fp16 product about
// as accurate as two bf16 ones: CPU emulation over config #4's 64 logged states (tools/x3_error_budget.py,
// profiles/r06_x3_error_budget_f16.txt) puts the costs within 4.3e-5 ("bf16x3,f16x1,f16x2w") / 2.8e-5
// ("f16x2w,f16x1,f16x2w") of the fp32 oracle at H = 64 (the two-product bf16 form: 4.95e-5).  Per-wave kernels: 140
// MFMAs per wave-step instead of 242 (statistic 18 -> 12, layer 0 48 -> 32, layer 1 128 -> 64, last layer 48 -> 32), no
// W1 lo stream from L2, no hi / lo splits in VALU; x3d: 48 instead of 68.  A CHECKED property of the net like the
// two-product form: x3_probe runs fc_wave32_x3p_kernel's fp16 form against three products and keeps it only within
// kX3ProbeTol, never beyond kX3TwoTermMaxH.  MPPI_X3_F16=0 / =1 (read per launch) forces it off / on without a probe.
inline int x3_f16_env() {
  const char* e = std::getenv("MPPI_X3_F16");
  return e && (e[0] == '0' || e[0] == '1') ? (e[0] == '1' ? 1 : -1) : 0;
}
inline bool x3_f16_on(int H, int decided, int img_off) {
  if (img_off < 0) return false;
  if (const int f = x3_f16_env()) return f > 0;
  return H <= kX3TwoTermMaxH && decided >= 1;
}
// ... with the last layer as ONE fp16 product (fp16 W against the fp16 activations): OPT-IN only, MPPI_X3_F16_L2=1 (read
// per launch).  124 MFMAs per wave-step instead of 140, rollout -6 % (profiles/r06_ab_f16_l2x1.log), but not
// fp32-accurate on every logged state: CPU emulation "f16x2w,f16x1,f16x1" 4.8e-5 from the fp32 oracle over config
// #4's 64 states, while on the GPU one of 34 logged states (H = 64) ended 1.04e-4 from the three-product costs
// (profiles/r06_gpu_tests_f16_l2x1.log) -- the dynamics error is common to all samples of a solve (the CA's action
// encoder never reaches its output), so one state's error is the whole solve's.  The probe does not pick it.
inline bool x3_f16_l2x1(int decided) {
  const char* e = std::getenv("MPPI_X3_F16_L2");
  return (e && e[0] == '1') || decided == 2;
}
// The split CA rollout's form at launch: 0 = fp16 with the one-product last layer, 1 = fp16, 2 = bf16 with the
// two-product layer 1, 3 = bf16 three products (the kernels' L1T template argument)
inline int x3_form(int H, int l1_decided, int f16_decided, int f16_img) {
  if (x3_f16_on(H, f16_decided, f16_img)) return x3_f16_l2x1(f16_decided) ? 0 : 1;
  return x3_l1_terms(H, l1_decided);
}
__device__ __forceinline__ unsigned pk_bf16_x3(float a, float b) {  // one v_cvt_pk_bf16_f32 (RNE)
  return __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{a, b}, bf16x2));
}
template <>
struct P<MPPI_PREC_BF16X3> {
  using Bop = BX3;
  using Wt = BX3;  // the packer writes per lane the hi fragment then the lo fragment (32 B)
  static constexpr int TILE_BYTES = 1024;  // one 16-row tile: 512 B in each plane
  static constexpr int KS(int mti) { return mti / 2; }
  // hi and lo packed pairs of (a, b)
  __device__ static void split2(float a, float b, unsigned& h, unsigned& l) {
    h = pk_bf16_x3(a, b);
    l = pk_bf16_x3(a - __uint_as_float(h << 16), b - __uint_as_float(h & 0xFFFF0000u));
  }
  __device__ static void put_tile(char* buf, int mt, int lane, const f32x4& v) {
    unsigned h0, l0, h1, l1;
    split2(v[0], v[1], h0, l0);
    split2(v[2], v[3], h1, l1);
    char* p = buf + (mt >> 1) * 2048 + lane * 16 + (mt & 1) * 8;
    *reinterpret_cast<uint2*>(p) = make_uint2(h0, h1);
    *reinterpret_cast<uint2*>(p + 1024) = make_uint2(l0, l1);
  }
  __device__ static void put_tile_relu(char* buf, int mt, int lane, const f32x4& v);  // after relu(), below
  __device__ static Bop get_ks(const char* buf, int ks, int lane) {
    return BX3{*reinterpret_cast<const bf16x8*>(buf + ks * 2048 + lane * 16),
               *reinterpret_cast<const bf16x8*>(buf + ks * 2048 + 1024 + lane * 16)};
  }
  __device__ static f32x4 mma(const Wt& a, const Bop& b, const f32x4& c) {
    f32x4 d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.lo, b.hi, c, 0, 0, 0);
    d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.hi, b.lo, d, 0, 0, 0);
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.hi, b.hi, d, 0, 0, 0);
  }
  // The same product with the A fragments read from AccVGPRs.  The M-split kernels hold every layer's fragments of a
  // wave in registers (CA 224); hipcc places them in AGPRs and, since it selects the builtin MFMA with VGPR sources
  // only, copies each fragment back with v_accvgpr_read before every use: 213 copies per wave-step in the CA kernel,
  // a quarter of its VALU issue (PMC: 718 VALU per 168 MFMAs).  The hardware reads A/B from AGPRs, so the three MFMAs
  // go in one asm statement.  hipcc's hazard recognizer does not see into it, so the statement pads its own entry
  // (s_nop 1: a VALU write of a source or of the accumulator right before it) and the caller passes every
  // accumulator through mma_fence() before any other instruction reads it (MFMA write -> VALU read).  Volatile, so
  // the statements keep their order relative to the fences.
  __device__ static f32x4 mma_a(const Wt& a, const Bop& b, f32x4 c) {
    asm volatile(
        "s_nop 1\n\t"
        "v_mfma_f32_16x16x32_bf16 %0, %1, %3, %0\n\t"
        "v_mfma_f32_16x16x32_bf16 %0, %2, %4, %0\n\t"
        "v_mfma_f32_16x16x32_bf16 %0, %2, %3, %0"
        : "+v"(c)
        : "a"(a.lo), "a"(a.hi), "v"(b.hi), "v"(b.lo));
    return c;
  }
  // ... the two-product layer 1 (x3_l1_terms): W_lo b_hi + W_hi b_hi, the same asm form as mma_a
  __device__ static f32x4 mma_a2(const Wt& a, const bf16x8& bh, f32x4 c) {
    asm volatile(
        "s_nop 1\n\t"
        "v_mfma_f32_16x16x32_bf16 %0, %1, %3, %0\n\t"
        "v_mfma_f32_16x16x32_bf16 %0, %2, %3, %0"
        : "+v"(c)
        : "a"(a.lo), "a"(a.hi), "v"(bh));
    return c;
  }
  // ... and its operand: the hi plane of a tile pair only
  __device__ static void put_tile_relu_hi(char* buf, int mt, int lane, const f32x4& v);  // after relu(), below
  __device__ static bf16x8 get_ks_hi(const char* buf, int ks, int lane) {
    return *reinterpret_cast<const bf16x8*>(buf + ks * 2048 + lane * 16);
  }
  __device__ static void put_u(Bop* bin, const f32x4 (&u)[2]) {
    unsigned h[4], l[4];
    split2(u[0][0], u[0][1], h[0], l[0]);
    split2(u[0][2], u[0][3], h[1], l[1]);
    split2(u[1][0], u[1][1], h[2], l[2]);
    split2(u[1][2], u[1][3], h[3], l[3]);
    typedef __attribute__((ext_vector_type(4))) unsigned u4;
    bin[0].hi = __builtin_bit_cast(bf16x8, u4{h[0], h[1], h[2], h[3]});
    bin[0].lo = __builtin_bit_cast(bf16x8, u4{l[0], l[1], l[2], l[3]});
  }
};

// relu as one v_med3_f32 (clamp to [0, FLT_MAX]): fmaxf in IEEE mode first canonicalises an MFMA result
// (v_max x, x), doubling the cost.  (Not inline asm: the hazard recognizer does not pad an asm read of an MFMA
// result, which then reads the accumulator too early.)
__device__ __forceinline__ float relu(float x) { return __builtin_amdgcn_fmed3f(x, 0.0f, 3.402823466e38f); }
__device__ inline void P<MPPI_PREC_FP32>::put_tile_relu(char* buf, int mt, int lane, const f32x4& v) {
  put_tile(buf, mt, lane, f32x4{relu(v[0]), relu(v[1]), relu(v[2]), relu(v[3])});
}
__device__ inline void P<MPPI_PREC_BF16X3>::put_tile_relu(char* buf, int mt, int lane, const f32x4& v) {
  put_tile(buf, mt, lane, f32x4{relu(v[0]), relu(v[1]), relu(v[2]), relu(v[3])});  // relu in fp32, then split
}
__device__ inline void P<MPPI_PREC_BF16X3>::put_tile_relu_hi(char* buf, int mt, int lane, const f32x4& v) {
  P<MPPI_PREC_BF16>::put_tile_relu(buf + (mt >> 1) * 1024, mt, lane, v);  // the bf16 form's packed ReLU, hi plane
}

// Copy n16 16-byte units global -> LDS with THREADS threads, the loads issued in batches of 8 per thread before their
// stores: the plain loop (d[i] = s[i], i += THREADS) waited for every load before its store, one memory round trip per
// unit and thread (18 in a row for the 144 KiB split image at 512 threads) before the horizon loop could start.
template <int THREADS>
__device__ __forceinline__ void stage_lds(int4* __restrict__ d, const int4* __restrict__ s, int n16) {
  constexpr int NB = 8;
  int i = threadIdx.x;
  for (; i + (NB - 1) * THREADS < n16; i += NB * THREADS) {
    int4 t[NB];
#pragma unroll
    for (int j = 0; j < NB; ++j) t[j] = s[i + j * THREADS];
#pragma unroll
    for (int j = 0; j < NB; ++j) d[i + j * THREADS] = t[j];
  }
  for (; i < n16; i += THREADS) d[i] = s[i];
}

// ------------------------------------------------------------------------------------------------ lane groups

// sum over the 4 lanes of a sample (lane groups 0..3), result in every lane; order (g0+g1)+(g2+g3).
__device__ __forceinline__ float group_sum(float v) {
  auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  const float s = __uint_as_float(p[0]) + __uint_as_float(p[1]);
  auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(s), __float_as_uint(s), false, false);
  return __uint_as_float(q[0]) + __uint_as_float(q[1]);
}

// State slots the running cost reads, as whole 4-slot chunks (m-tile, lane group) of the state tiles: the rollouts
// store only these chunks into their cost rings.
template <int ARCH, int COST>
struct CostChunks {
  static constexpr int slot(int xi) { return xi < Arch<ARCH>::QP ? xi : 32 + (xi - Arch<ARCH>::QP); }
  static constexpr bool needed(int tile, int g) {
    const CostIdx ci = cost_idx(COST);
    for (int i = 0; i < ci.n; ++i)
      if (slot(ci.idx[i]) / 4 == 4 * tile + g) return true;
    return false;
  }
  // chunk index of (tile, g) in the ring row, -1 if the cost reads none of its slots
  static constexpr int chunk(int tile, int g) {
    if (!needed(tile, g)) return -1;
    int c = 0;
    for (int e = 0; e < 4 * tile + g; ++e) c += needed(e / 4, e % 4) ? 1 : 0;
    return c;
  }
  static constexpr int count() {
    int c = 0;
    for (int e = 0; e < 16; ++e) c += needed(e / 4, e % 4) ? 1 : 0;
    return c;
  }
  static constexpr int NCH = count() > 0 ? count() : 1;
  static constexpr int HS = 4 * NCH;  // floats per (step, sample) ring row
};


// After a layer's P<BF16X3>::mma_a statements: every accumulator of the layer through one volatile statement, the
// first padded past the MFMA write -> VALU read hazard (16x16x32 bf16: 4 passes, 7 wait states on gfx950's table;
// 12 here), the others ordered behind it, so no instruction reads an accumulator before the pad.
template <bool PAD = true, int N>
__device__ __forceinline__ void mma_fence(f32x4 (&v)[N]) {
  if constexpr (PAD)
    asm volatile("s_nop 7\n\ts_nop 3" : "+v"(v[0]));
  else
    asm volatile("" : "+v"(v[0]));
#pragma unroll
  for (int i = 1; i < N; ++i) asm volatile("" : "+v"(v[i]));
}
template <bool PAD = true, int M, int N>
__device__ __forceinline__ void mma_fence(f32x4 (&v)[M][N]) {
  if constexpr (PAD)
    asm volatile("s_nop 7\n\ts_nop 3" : "+v"(v[0][0]));
  else
    asm volatile("" : "+v"(v[0][0]));
#pragma unroll
  for (int j = 0; j < M; ++j)
#pragma unroll
    for (int i = 0; i < N; ++i)
      if (i + j > 0) asm volatile("" : "+v"(v[j][i]));
}

// ------------------------------------------------------------------------------------------------ layer

// out[i] (own tiles mt = mt0 + i) += W[mt] * in over this wave's KSB k-steps (a block-diagonal layer passes
// only its diagonal block's k-steps).  A fragment (mt, kk) at (mt * KSB + kk) * 64 + lane.
template <int PREC, int KSB, int NOWN>
__device__ __forceinline__ void mfma_rows(f32x4 (&out)[NOWN], const typename P<PREC>::Bop (&bin)[KSB],
                                          const typename P<PREC>::Wt* __restrict__ w, int mt0, int lane) {
#pragma unroll
  for (int kk = 0; kk < KSB; ++kk) {
#pragma unroll
    for (int i = 0; i < NOWN; ++i) out[i] = P<PREC>::mma(w[((mt0 + i) * KSB + kk) * 64 + lane], bin[kk], out[i]);
  }
}

// The same from this wave's fragments held in registers: wr[i][kk] = fragment (mt0 + i, kk).
template <int PREC, int KSB, int NOWN>
__device__ __forceinline__ void load_frags(typename P<PREC>::Wt (&wr)[NOWN][KSB],
                                           const typename P<PREC>::Wt* __restrict__ w, int mt0, int lane) {
#pragma unroll
  for (int i = 0; i < NOWN; ++i)
#pragma unroll
    for (int kk = 0; kk < KSB; ++kk) wr[i][kk] = w[((mt0 + i) * KSB + kk) * 64 + lane];
}
// The running cost is evaluated in batches of kRing steps: at the end of step t the waves owning the state slots
// the cost reads (cost_idx) store them, as whole 4-slot chunks (tile, lane group), into a ring of kRing steps;
// after every kRing steps each lane evaluates the FULL cost of one (step, sample) pair (4 waves x 4 lane groups
// = 16 steps x 16 samples), so no lane computes a cost twice and the per-step loop carries no cost code.
constexpr int kRing = 16;

// LDS per group (bytes): xb (4 state tiles as B operands), act0..act2 (layer outputs), hist (cost ring,
// [kRing steps][16 samples][HS] fp32), st (LN partial stats, S x 16 float2), cp (partial costs, S x 16).
template <int ARCH, int PREC, int COST>
struct Lay {
  using A = Arch<ARCH>;
  static constexpr int TB = P<PREC>::TILE_BYTES;
  static constexpr int XB = 0;
  static constexpr int ACT0 = XB + 4 * TB;
  static constexpr int ACT1 = ACT0 + A::MT0 * TB;
  static constexpr int ACT2 = ACT1 + A::MT1 * TB;
  static constexpr int HIST = ACT2 + (A::NL == 4 ? A::MT2 * TB : 0);
  static constexpr int ST = HIST + kRing * 16 * CostChunks<ARCH, COST>::HS * 4;
  static constexpr int CP = ST + kSplit * 16 * 8;
  static constexpr int BYTES = (CP + kSplit * 16 * 4 + 15) / 16 * 16;
};

}  // namespace mppi
