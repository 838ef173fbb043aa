// Shared by the split (MPPI_PREC_BF16X3) per-wave CA rollouts: fc_wave32_x3_kernel (kernels_fc_x3.hip, one wave per
// SIMD) and fc_wave32_x3p_kernel (kernels_fc_x3p.hip, two waves per SIMD): the LDS image layout, the hi / lo split and
// the three-MFMA product.
#pragma once
#include "fc_rollout.h"

namespace mppi {

typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
__device__ __forceinline__ f32x16 mma32(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ unsigned pk_bf16(float a, float b) {  // one v_cvt_pk_bf16_f32 (RNE)
  typedef __attribute__((ext_vector_type(2))) float f32x2;
  typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
  return __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{a, b}, bf16x2));
}
__device__ __forceinline__ unsigned pk_f16(float a, float b) {  // one v_cvt_pk_f16_f32 (RNE)
  typedef __attribute__((ext_vector_type(2))) float f32x2;
  typedef __attribute__((ext_vector_type(2))) _Float16 f16x2;
  return __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{a, b}, f16x2));
}
__device__ __forceinline__ float f16_hi_value(unsigned p) {  // the fp16 in the upper half of a packed pair, as fp32
  return (float)__builtin_bit_cast(_Float16, (unsigned short)(p >> 16));
}
static inline int x3_device_cus() { return current_device_cus(); }

}  // namespace mppi

// ------------------------------------------------------------------------- split bf16 (MPPI_PREC_BF16X3), per-wave

namespace mppi {

// fc_wave32_kernel's organisation at fp32 accuracy: every product as three 32x32x16 bf16 MFMAs (W_hi a_hi, W_hi a_lo,
// W_lo a_hi; fp32 accumulate), the layer-0 operand, the activations and s split into bf16 hi / lo pairs in registers.
// One wave per SIMD (4 waves, 32 samples each, per CU): the hi / lo activations take ~200 VGPRs, so the 512-entry
// register file of a lone wave is what holds them.  The hi fragments of every layer and the lo fragments of layers 0, 2
// and the statistic factor live in LDS (144 KiB); W1's lo fragments (64 KiB) stream from L2, two k-steps ahead.
// Layer 0 is the block-diagonal, uncentred form with the row mean subtracted through the accumulators (mppi_nets.cpp,
// L0x): b0c against 1.0 in slots 28 / 60, beta' against s in slots 30 / 62.
#ifndef MPPI_X3_L1PF  // W1's lo fragments from L2, this many k-steps ahead
#define MPPI_X3_L1PF 2
#endif
struct WaveX3Lay {
  static constexpr int W0H = 0;                // 16 fragments: D-tiles 0..3 k-steps 0, 1; 4..7 k-steps 2, 3
  static constexpr int W1H = W0H + 16 * 1024;  // 64: T 16 + ks
  static constexpr int WXH = W1H + 64 * 1024;  // 16: T 8 + ks
  static constexpr int RH = WXH + 16 * 1024;   // 8: T 4 + ks
  static constexpr int W0L = RH + 8 * 1024;
  static constexpr int WXL = W0L + 16 * 1024;
  static constexpr int RL = WXL + 16 * 1024;
  static constexpr int IMG = RL + 8 * 1024;  // 144 KiB, one contiguous copy of the image at net.w32x3_off
  static constexpr int B1 = IMG;             // 128 f32
  static constexpr int BX = B1 + 512;        // 64 f32
  static constexpr int RING = BX + 256;
  static constexpr int WAVES = 4;
  template <int COST>
  static constexpr int ring_bytes() { return 2 * 32 * CostChunks<kArchCA, COST>::HS * 4; }
  template <int COST>
  static constexpr int bytes() { return RING + WAVES * ring_bytes<COST>(); }
};

// values 8 HALF .. 8 HALF + 7 of a 32x32 accumulator tile as bf16 hi and lo (lo = v - hi, rounded) B operands
template <int HALF>
__device__ __forceinline__ void split32(const f32x16& v, bf16x8& hi, bf16x8& lo) {
  constexpr int o = 8 * HALF;
  u32x4 hw, lw;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float x0 = v[o + 2 * q], x1 = v[o + 2 * q + 1];
    const unsigned p = pk_bf16(x0, x1);
    hw[q] = p;
    lw[q] = pk_bf16(x0 - __uint_as_float(p << 16), x1 - __uint_as_float(p & 0xFFFF0000u));
  }
  hi = __builtin_bit_cast(bf16x8, hw);
  lo = __builtin_bit_cast(bf16x8, lw);
}
// values 8 HALF .. 8 HALF + 7 of a 32x32 accumulator tile as a bf16 B operand (the hi part only)
template <int HALF>
__device__ __forceinline__ bf16x8 hi32(const f32x16& v) {
  constexpr int o = 8 * HALF;
  u32x4 hw;
#pragma unroll
  for (int q = 0; q < 4; ++q) hw[q] = pk_bf16(v[o + 2 * q], v[o + 2 * q + 1]);
  return __builtin_bit_cast(bf16x8, hw);
}
// ... ReLU'd: relu on the packed bf16 bit patterns after the conversion (one v_pk_max_i16 per pair instead of two
// v_med3_f32 before it; a negative bf16 is a negative int16), bit-identical for every non-NaN input
template <int HALF>
__device__ __forceinline__ bf16x8 hi32_relu(const f32x16& v) {
  typedef __attribute__((ext_vector_type(2))) short i16x2_;
  constexpr int o = 8 * HALF;
  u32x4 hw;
#pragma unroll
  for (int q = 0; q < 4; ++q)
    hw[q] = __builtin_bit_cast(unsigned, __builtin_elementwise_max(
                                             __builtin_bit_cast(i16x2_, pk_bf16(v[o + 2 * q], v[o + 2 * q + 1])),
                                             i16x2_{0, 0}));
  return __builtin_bit_cast(bf16x8, hw);
}
// The fp16 form of fc_wave32_x3p_kernel (L1T == 1, fc_common.h x3_f16_on): fp16 fragments and operands, carried in
// bf16x8 containers (16 B per lane either way), on v_mfma_f32_32x32x16_f16 (fp32 accumulate; fp16 subnormals kept)
__device__ __forceinline__ f32x16 mma32h(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  typedef __attribute__((ext_vector_type(8))) _Float16 f16x8_;
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8_, a), __builtin_bit_cast(f16x8_, b), c, 0, 0, 0);
}
// values 8 HALF .. 8 HALF + 7 of a 32x32 accumulator tile as a ReLU'd fp16 B operand: one v_cvt_pk_f16_f32 (RNE) and
// one v_pk_max_i16 per pair (a negative fp16, like a negative bf16, is a negative int16)
template <int HALF>
__device__ __forceinline__ bf16x8 h16_relu(const f32x16& v) {
  typedef __attribute__((ext_vector_type(2))) short i16x2_;
  typedef __attribute__((ext_vector_type(2))) float f32x2_;
  typedef __attribute__((ext_vector_type(2))) _Float16 f16x2_;
  constexpr int o = 8 * HALF;
  u32x4 hw;
#pragma unroll
  for (int q = 0; q < 4; ++q)
    hw[q] = __builtin_bit_cast(
        unsigned, __builtin_elementwise_max(__builtin_bit_cast(i16x2_, __builtin_convertvector(
                                                                           f32x2_{v[o + 2 * q], v[o + 2 * q + 1]}, f16x2_)),
                                            i16x2_{0, 0}));
  return __builtin_bit_cast(bf16x8, hw);
}
// values 8 HALF .. 8 HALF + 7 of a 32x32 accumulator tile as an fp16 B operand (no ReLU)
template <int HALF>
__device__ __forceinline__ bf16x8 h16(const f32x16& v) {
  constexpr int o = 8 * HALF;
  u32x4 hw;
#pragma unroll
  for (int q = 0; q < 4; ++q) hw[q] = pk_f16(v[o + 2 * q], v[o + 2 * q + 1]);
  return __builtin_bit_cast(bf16x8, hw);
}
// acc += W a with W = wh + wl, a = ah + al (the wl al term dropped)
__device__ __forceinline__ f32x16 mma3(const bf16x8& wh, const bf16x8& wl, const bf16x8& ah, const bf16x8& al,
                                       f32x16 acc) {
  acc = mma32(wl, ah, acc);
  acc = mma32(wh, al, acc);
  return mma32(wh, ah, acc);
}

}  // namespace mppi
