// MFMA operand traits for GEMMs whose A operand (weights) is packed as 16x32 fragments and whose B operand is read
// from a [row][feature] LDS buffer: the FeatureAttention kernels (kernels_fa.hip) and the generic fc-stack kernel
// (kernels_fc_generic.hip).  Fragments are packed by mppi_nets.cpp::pack_frags.
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/mppi.h"

namespace mppi {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;

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
  // relu(v) as bf16: v_pk_max_i16 on the packed bit patterns after the conversion (bit-identical for non-NaN input)
  __device__ static void st4_relu(char* p, const f32x4& v) {
    typedef __attribute__((ext_vector_type(2))) float f2;
    typedef __attribute__((ext_vector_type(2))) __bf16 b2;
    typedef __attribute__((ext_vector_type(2))) short i2;
    auto pk = [](float a, float b) {
      const b2 q = __builtin_convertvector(f2{a, b}, b2);
      return __builtin_bit_cast(unsigned, __builtin_elementwise_max(__builtin_bit_cast(i2, q), i2{0, 0}));
    };
    *reinterpret_cast<uint2*>(p) = make_uint2(pk(v[0], v[1]), pk(v[2], v[3]));
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
  __device__ static void st4_relu(char* p, const f32x4& v) {  // v_med3 against FLT_MAX (no NaN-quieting max)
    const float M = 3.402823466e38f;
    *reinterpret_cast<f32x4*>(p) = f32x4{__builtin_amdgcn_fmed3f(v[0], 0.0f, M), __builtin_amdgcn_fmed3f(v[1], 0.0f, M),
                                         __builtin_amdgcn_fmed3f(v[2], 0.0f, M), __builtin_amdgcn_fmed3f(v[3], 0.0f, M)};
  }
  __device__ static f32x4 ld4(const char* p) { return *reinterpret_cast<const f32x4*>(p); }
};


}  // namespace mppi
