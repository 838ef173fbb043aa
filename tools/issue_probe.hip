// Issue-rate probe for the per-wave rollout's instruction mix on gfx950 (diagnostic, not product code): cycles per
// wave64 instruction of the VALU ops fc_wave32_kernel issues around its MFMAs, alone and beside MFMAs from the same
// wave or from the other wave on the SIMD.
//   hipcc -O3 --offload-arch=gfx950 tools/issue_probe.hip -o /tmp/issue_probe && /tmp/issue_probe
// One block of 512 threads on one CU: waves 0..3 (one per SIMD) run role A, waves 4..7 role B.
#include <hip/hip_runtime.h>

#include <cstdio>

typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;

enum Role { IDLE, FMA, CVT, PKMAX, PKADD, PKFMA, MFMA32, MFMA16, MIX32_FMA, MIX32_CVT, MIX32_CVTMAX, NROLES };
static const char* kName[] = {"idle", "v_fma_f32", "v_cvt_pk_bf16_f32", "v_pk_max_i16", "v_pk_add_f32",
                              "v_pk_fma_f32", "mfma32x32x16", "mfma16x16x32", "4 mfma32 + 16 fma",
                              "4 mfma32 + 16 cvt", "4 mfma32 + 8 cvt + 8 max"};
// VALU instructions and MFMAs per loop iteration of each role
static const int kValu[] = {0, 16, 16, 16, 16, 16, 0, 0, 16, 16, 16};
static const int kMfma[] = {0, 0, 0, 0, 0, 0, 4, 4, 4, 4, 4};

#define V16(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)

template <int role>
__device__ __forceinline__ void valu16(float (&r)[16], unsigned (&u)[16], float s) {
  switch (role) {
    case FMA:
    case MIX32_FMA:
#define OP(i) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(r[i]) : "v"(s));
      V16(OP)
#undef OP
      break;
    case CVT:
    case MIX32_CVT:
#define OP(i) asm volatile("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(u[i]) : "v"(r[i]), "v"(s));
      V16(OP)
#undef OP
      break;
    case PKMAX:
#define OP(i) asm volatile("v_pk_max_i16 %0, %0, 0" : "+v"(u[i]));
      V16(OP)
#undef OP
      break;
    case MIX32_CVTMAX:
#define OP(i) asm volatile("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(u[i]) : "v"(r[i]), "v"(s));
      OP(0) OP(1) OP(2) OP(3) OP(4) OP(5) OP(6) OP(7)
#undef OP
#define OP(i) asm volatile("v_pk_max_i16 %0, %0, 0" : "+v"(u[i]));
      OP(0) OP(1) OP(2) OP(3) OP(4) OP(5) OP(6) OP(7)
#undef OP
      break;
    case PKADD:
#define OP(i) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(*reinterpret_cast<double*>(&r[(2 * i) % 16])) : "v"(1.0));
      V16(OP)
#undef OP
      break;
    case PKFMA:
#define OP(i)                                                                    \
  asm volatile("v_pk_fma_f32 %0, %0, %1, %1"                                    \
               : "+v"(*reinterpret_cast<double*>(&r[(2 * i) % 16]))              \
               : "v"(1.0));
      V16(OP)
#undef OP
      break;
    default:
      break;
  }
}

template <int role>
__device__ __forceinline__ unsigned long long run_role(int iters, float* sink) {
  float r[16];
  unsigned u[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    r[i] = (float)(threadIdx.x + i);
    u[i] = threadIdx.x * 7u + i;
  }
  const float s = 1.0f + 1e-7f * threadIdx.x;
  bf16x8 a, b;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    a[i] = (__bf16)(0.001f * (threadIdx.x + i));
    b[i] = (__bf16)(0.002f * i);
  }
  f32x16 c32[4] = {};
  f32x4 c16[4] = {};
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  if constexpr (role != IDLE) {
    for (int it = 0; it < iters; ++it) {
      if constexpr (role == MFMA32 || role >= MIX32_FMA) {
#pragma unroll
        for (int k = 0; k < 4; ++k) c32[k] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c32[k], 0, 0, 0);
      } else if constexpr (role == MFMA16) {
#pragma unroll
        for (int k = 0; k < 4; ++k) c16[k] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c16[k], 0, 0, 0);
      }
      valu16<role>(r, u, s);
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float acc = 0.0f;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc += r[i] + (float)u[i] + c32[i % 4][i] + c16[i % 4][i % 4];
  sink[threadIdx.x] = acc;
  return t1 - t0;
}

template <int A, int B>
__global__ __launch_bounds__(512) void probe(int iters, unsigned long long* cycles, float* sink) {
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  __syncthreads();
  const unsigned long long c = w < 4 ? run_role<A>(iters, sink) : run_role<B>(iters, sink);
  if ((threadIdx.x & 63) == 0) cycles[w] = c;
}

int main() {
  unsigned long long* dc;
  float* ds;
  if (hipMalloc(&dc, 8 * sizeof(unsigned long long)) != hipSuccess || hipMalloc(&ds, 512 * 4) != hipSuccess) return 1;
  const int iters = 4096;
  auto run = [&](auto kern, int A, int B) {
    unsigned long long c[8];
    for (int rep = 0; rep < 3; ++rep) {  // the last of three (clock ramp)
      hipLaunchKernelGGL(kern, dim3(1), dim3(512), 0, 0, iters, dc, ds);
      if (hipDeviceSynchronize() != hipSuccess) return false;
    }
    if (hipMemcpy(c, dc, sizeof c, hipMemcpyDeviceToHost) != hipSuccess) return false;
    double ca = 0, cb = 0;
    for (int i = 0; i < 4; ++i) ca += c[i] / 4.0;
    for (int i = 4; i < 8; ++i) cb += c[i] / 4.0;
    auto per = [&](int role, double cyc) {
      const int n = kValu[role] + kMfma[role];
      return n ? cyc / iters / n : 0.0;
    };
    printf("A %-26s | B %-26s | A %8.0f cyc/iter (%.2f per instr) | B %8.0f cyc/iter (%.2f per instr)\n", kName[A],
           kName[B], ca / iters, per(A, ca), cb / iters, per(B, cb));
    return true;
  };
  bool ok = true;
#define RUN(A, B) \
  if (ok) ok = run(probe<A, B>, A, B);
  RUN(FMA, IDLE) RUN(CVT, IDLE) RUN(PKMAX, IDLE) RUN(PKADD, IDLE) RUN(PKFMA, IDLE) RUN(MFMA32, IDLE) RUN(MFMA16, IDLE)
  RUN(MIX32_FMA, IDLE) RUN(MIX32_CVT, IDLE) RUN(MIX32_CVTMAX, IDLE)
  RUN(FMA, FMA) RUN(CVT, CVT) RUN(PKMAX, PKMAX) RUN(PKADD, PKADD) RUN(MFMA32, MFMA32) RUN(MFMA16, MFMA16)
  RUN(MIX32_FMA, MIX32_FMA) RUN(MIX32_CVTMAX, MIX32_CVTMAX)
  RUN(MFMA32, FMA) RUN(MFMA32, CVT) RUN(MFMA32, PKMAX) RUN(MFMA32, PKADD) RUN(MFMA16, FMA) RUN(MFMA16, CVT)
#undef RUN
  printf(ok ? "ok\n" : "launch failed\n");
  return ok ? 0 : 1;
}
