// Does the MFMA shape change the clock the chip holds under load (MI355X_MICROARCH.md, DVFS item 7)?  Every CU runs
// 8 waves (two per SIMD) of back-to-back bf16 MFMAs on random operands in registers, either v_mfma_f32_32x32x16_bf16
// or v_mfma_f32_16x16x32_bf16 (the same FLOP per cycle), for ~0.3 s per launch after two warm-up launches; reported: wall time per
// MFMA FLOP and the in-kernel clock (s_memtime ticks / s_memrealtime at 100 MHz, median over workgroups).  The
// split-bf16 per-wave rollouts run on 32x32x16; a 16x16x32 form pays off only if it holds a higher clock.
//   hipcc -O3 --offload-arch=gfx950 -o tools/mfma_clock_probe tools/mfma_clock_probe.hip && tools/mfma_clock_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) float f32x4;

__device__ inline unsigned hash(unsigned x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  return x ^ (x >> 16);
}

template <bool BIG>
__global__ __launch_bounds__(512) void mfma_loop(int iters, float* out, unsigned long long* clk) {
  const unsigned seed = hash(blockIdx.x * 512 + threadIdx.x);
  bf16x8 a[4], b[4];
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 8; ++j) {
      a[i][j] = (__bf16)((float)(hash(seed + 16 * i + j) & 0xFFFF) / 65536.0f - 0.5f);
      b[i][j] = (__bf16)((float)(hash(seed * 3 + 16 * i + j) & 0xFFFF) / 65536.0f - 0.5f);
    }
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  float s = 0.0f;
  if constexpr (BIG) {
    f32x16 c[2] = {};
    for (int it = 0; it < iters; ++it)
#pragma unroll
      for (int i = 0; i < 4; ++i) c[i & 1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[i], c[i & 1], 0, 0, 0);
    for (int i = 0; i < 16; ++i) s += c[0][i] + c[1][i];
  } else {
    f32x4 c[4] = {};
    for (int it = 0; it < iters; ++it)
#pragma unroll
      for (int r = 0; r < 2; ++r)  // twice the instructions of half the size: the same FLOP per iteration
#pragma unroll
        for (int i = 0; i < 4; ++i) c[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[(i + r) & 3], c[i], 0, 0, 0);
    for (int i = 0; i < 4; ++i) s += c[i][0] + c[i][1] + c[i][2] + c[i][3];
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (s == 12345.678f) out[blockIdx.x] = s;
  if (threadIdx.x == 0) {
    clk[2 * blockIdx.x] = t1 - t0;
    clk[2 * blockIdx.x + 1] = r1 - r0;
  }
}

int main() {
  int cus = 256;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  float* out;
  unsigned long long* clk;
  if (hipMalloc(&out, cus * 4) != hipSuccess || hipMalloc(&clk, cus * 16) != hipSuccess) return 1;
  std::vector<unsigned long long> h(2 * cus);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  auto run = [&](bool big, int iters, bool report) {
    (void)hipEventRecord(e0);
    if (big)
      mfma_loop<true><<<cus, 512>>>(iters, out, clk);
    else
      mfma_loop<false><<<cus, 512>>>(iters, out, clk);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0.0f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (!report) return;
    (void)hipMemcpy(h.data(), clk, cus * 16, hipMemcpyDeviceToHost);
    std::vector<double> ghz;
    for (int i = 0; i < cus; ++i) ghz.push_back(h[2 * i] / (h[2 * i + 1] * 10.0));  // ticks / (realtime x 10 ns) in GHz
    std::sort(ghz.begin(), ghz.end());
    const double flop = 2.0 * 4 * 32 * 32 * 16 * (double)iters * 8 * cus;  // per wave: 4 x 32x32x16 per iteration
    std::printf("%-10s %8.2f ms  %7.1f TFLOP/s  in-kernel clock median %.3f GHz (min %.3f, max %.3f)\n",
                big ? "32x32x16" : "16x16x32", ms, flop / (ms * 1e-3) / 1e12, ghz[cus / 2], ghz[0], ghz[cus - 1]);
  };
  const int iters = 1000000;  // ~0.3 s per launch (4 x 32 cycles per iteration, two waves per SIMD: 2.6e8 cycles per SIMD)
  for (int w = 0; w < 2; ++w) run(true, iters, false);  // warm-up / clock ramp
  for (int rep = 0; rep < 3; ++rep) {
    run(true, iters, true);
    run(false, iters, true);
  }
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
