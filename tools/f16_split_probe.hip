// Probe of the split per-wave kernel's fp16 primitives on the GPU (kernels_fc_x3.hip): the hi / lo split of fp32
// values (v_cvt_pk_f16_f32 + v_fma_mix{lo,hi}_f16) against the host's _Float16 arithmetic, and how
// v_mfma_f32_32x32x16_f16 treats fp16 subnormal operands.  Build: hipcc -O3 --offload-arch=gfx950 -o f16_split_probe
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;

__device__ __forceinline__ unsigned pk_f16(float a, float b) {
  typedef __attribute__((ext_vector_type(2))) float f32x2;
  typedef __attribute__((ext_vector_type(2))) _Float16 f16x2;
  return __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{a, b}, f16x2));
}
__device__ __forceinline__ unsigned pk_rem_f16(unsigned hp, float a, float b) {
  unsigned d;
  asm("v_fma_mixlo_f16 %0, -%1, 1.0, %2 op_sel_hi:[1,0,0]" : "=v"(d) : "v"(hp), "v"(a));
  asm("v_fma_mixhi_f16 %0, -%1, 1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "+v"(d) : "v"(hp), "v"(b));
  return d;
}

__global__ void split_k(const float* in, unsigned* hi, unsigned* lo, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float a = in[2 * i], b = in[2 * i + 1];
  const unsigned h = pk_f16(a, b);
  hi[i] = h;
  lo[i] = pk_rem_f16(h, a, b);
}
// D = A B with A = 1.0 on row 0 (k = 0..15: A[0][k] = 1), B[k][n] = the given fp16 bits: D[0][n] = sum_k B[k][n]
__global__ void mfma_k(const unsigned short* bbits, float* out) {
  const int lane = threadIdx.x;
  f16x8 a, b;
  for (int j = 0; j < 8; ++j) {
    const int row = lane & 31, k = 8 * (lane >> 5) + j;
    a[j] = row == 0 ? (_Float16)1.0f : (_Float16)0.0f;
    unsigned short u = bbits[k * 32 + (lane & 31)];
    b[j] = __builtin_bit_cast(_Float16, u);
  }
  f32x16 c = {};
  c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
  // row 0 of the accumulator: lane n (n < 32) value 0
  if (lane < 32) out[lane] = c[0];
}

int main() {
  const int n = 1 << 16;
  std::mt19937 rng(1);
  std::vector<float> in(2 * n);
  for (int i = 0; i < 2 * n; ++i) {
    const float e = std::ldexp(1.0f, (int)(rng() % 30) - 20);
    in[i] = (rng() % 2 ? -1.0f : 1.0f) * e * (1.0f + (rng() % 100000) / 100000.0f);
  }
  float* din;
  unsigned *dh, *dl;
  hipMalloc(&din, 8 * n);
  hipMalloc(&dh, 4 * n);
  hipMalloc(&dl, 4 * n);
  hipMemcpy(din, in.data(), 8 * n, hipMemcpyHostToDevice);
  split_k<<<n / 256, 256>>>(din, dh, dl, n);
  std::vector<unsigned> h(n), l(n);
  hipMemcpy(h.data(), dh, 4 * n, hipMemcpyDeviceToHost);
  hipMemcpy(l.data(), dl, 4 * n, hipMemcpyDeviceToHost);
  int bad_hi = 0, bad_lo = 0;
  double worst = 0.0;
  for (int i = 0; i < n; ++i)
    for (int s = 0; s < 2; ++s) {
      const float v = in[2 * i + s];
      const _Float16 eh = (_Float16)v, el = (_Float16)(v - (float)eh);
      unsigned short gh = (unsigned short)(h[i] >> (16 * s)), gl = (unsigned short)(l[i] >> (16 * s));
      unsigned short ehb, elb;
      std::memcpy(&ehb, &eh, 2);
      std::memcpy(&elb, &el, 2);
      bad_hi += gh != ehb;
      bad_lo += gl != elb;
      _Float16 fh, fl;
      std::memcpy(&fh, &gh, 2);
      std::memcpy(&fl, &gl, 2);
      const double r = std::fabs(((double)(float)fh + (double)(float)fl) - (double)v) / std::fabs((double)v);
      if (std::fabs(v) > 1e-3) worst = std::max(worst, r);
    }
  std::printf("split: %d values, hi mismatches %d, lo mismatches %d, worst rel |hi+lo-v| (|v|>1e-3) %.3g\n", 2 * n,
              bad_hi, bad_lo, worst);
  // MFMA with subnormal fp16 B operands: column n holds 16 copies of one value
  std::vector<unsigned short> bb(16 * 32);
  const float vals[4] = {std::ldexp(1.0f, -15), std::ldexp(1.0f, -20), std::ldexp(1.0f, -24), std::ldexp(1.0f, -13)};
  for (int k = 0; k < 16; ++k)
    for (int c = 0; c < 32; ++c) {
      const _Float16 f = (_Float16)vals[c % 4];
      std::memcpy(&bb[k * 32 + c], &f, 2);
    }
  unsigned short* db;
  float* dout;
  hipMalloc(&db, bb.size() * 2);
  hipMalloc(&dout, 32 * 4);
  hipMemcpy(db, bb.data(), bb.size() * 2, hipMemcpyHostToDevice);
  mfma_k<<<1, 64>>>(db, dout);
  float out[32];
  hipMemcpy(out, dout, 128, hipMemcpyDeviceToHost);
  for (int c = 0; c < 4; ++c)
    std::printf("mfma f16: 16 x %.3g (%s) -> %.6g (expected %.6g)\n", vals[c], c == 3 ? "normal" : "subnormal",
                out[c], 16.0 * vals[c]);
  return 0;
}
