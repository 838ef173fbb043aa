// FETCH_SIZE calibration for the per-wave fc rollouts' noise read pattern (bench.py FETCH_FACTOR).
//
// MI355X_MICROARCH.md §HBM: FETCH_SIZE counts exactly half of a 16-B-per-lane coalesced streaming read on gfx950; other
// widths are uncalibrated.  The per-wave rollouts (fc_wave32_kernel, fc_wave32_x3[p]_kernel) read the noise eps[b][u][t][k]
// (k fastest, Kp = K padded to 64) as 4-byte loads: lane (h, n) of a wave holding samples k0..k0+31 reads control
// u = 2 j + h at step t, so one wave instruction reads two 128-B segments (rows (2j, t) and (2j+1, t)), every eps element
// once per launch.  This probe reads a buffer of exactly config #4's eps (64 solves x 21 x 64 x 1024 floats = 352 MB)
// in that pattern, and, as the control, the same bytes as 16-B-per-lane streaming loads; bench.py's factor for a kernel
// is then known bytes / (FETCH_SIZE x 1024) of its pattern, measured here, not fitted to the kernel itself.
//   hipcc -O3 --offload-arch=gfx950 -o tools/fetch_calib tools/fetch_calib.hip
//   rocprofv3 --pmc FETCH_SIZE -d <dir> -o p --output-format csv -- tools/fetch_calib   (scripts/fetch_calib.sh)
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int B = 64, NU = 21, H = 64, KP = 1024;

// the per-wave pattern: grid = B * KP / 32 waves (one 64-lane block each), every wave sweeps t and j like the rollout
__global__ __launch_bounds__(64) void eps_rows_kernel(const float* __restrict__ eps, float* __restrict__ out) {
  const int wt = blockIdx.x, lane = threadIdx.x, h = lane >> 5, n = lane & 31;
  const int b = wt / (KP / 32), k0 = (wt % (KP / 32)) * 32;
  // the rollout's loads: raw buffer loads, one descriptor per solve, per-lane voffset, out-of-range lanes read 0
  const auto rE = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(eps) + (long)b * NU * H * KP, 0, NU * H * KP * 4,
                                                    0x00020000);
  float acc = 0.0f;
  for (int t = 0; t < H; ++t)
#pragma unroll
    for (int j = 0; j < 11; ++j) {
      const int u = 2 * j + h;
      const int off = u < NU ? ((u * H + t) * KP + k0 + n) * 4 : 0x7FFFFFF0;
      acc += __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rE, off, 0, 0));
    }
  if (acc == 12345.678f) out[wt * 64 + lane] = acc;  // keeps the loads; never true for the zero-filled buffer
}

// the M-split rollout's pattern (fc_rollout_kernel: a group's 16 samples, lane group g of 16 lanes per control slot):
// one wave instruction reads four 64-B segments of four rows; grid = B * KP / 16 waves
__global__ __launch_bounds__(64) void eps_rows16_kernel(const float* __restrict__ eps, float* __restrict__ out) {
  const int wt = blockIdx.x, lane = threadIdx.x, g = lane >> 4, n = lane & 15;
  const int b = wt / (KP / 16), k0 = (wt % (KP / 16)) * 16;
  const auto rE = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(eps) + (long)b * NU * H * KP, 0, NU * H * KP * 4,
                                                    0x00020000);
  float acc = 0.0f;
  for (int t = 0; t < H; ++t)
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      const int u = 4 * j + g;
      const int off = u < NU ? ((u * H + t) * KP + k0 + n) * 4 : 0x7FFFFFF0;
      acc += __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rE, off, 0, 0));
    }
  if (acc == 12345.678f) out[wt * 64 + lane] = acc;
}

// control: the same bytes as coalesced 16-B-per-lane streaming loads
__global__ __launch_bounds__(256) void stream16_kernel(const float4* __restrict__ src, long n4, float* __restrict__ out) {
  float acc = 0.0f;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    const float4 v = src[i];
    acc += v.x + v.y + v.z + v.w;
  }
  if (acc == 12345.678f) out[blockIdx.x] = acc;
}

int main() {
  const long n = (long)B * NU * H * KP;
  const double bytes = 4.0 * n;
  float *eps, *out;
  if (hipMalloc(&eps, n * 4) != hipSuccess || hipMalloc(&out, (long)B * KP * 4 * 2) != hipSuccess) return 1;
  (void)hipMemset(eps, 0, n * 4);
  // evict: a 1 GiB sweep between launches so neither read is served from the Infinity Cache (256 MiB)
  float* big;
  const long nb = 256L << 20;  // floats = 1 GiB
  if (hipMalloc(&big, nb * 4) != hipSuccess) return 1;
  auto evict = [&]() { (void)hipMemset(big, 1, nb * 4); };
  for (int rep = 0; rep < 2; ++rep) {
    evict();
    eps_rows_kernel<<<B * KP / 32, 64>>>(eps, out);
    evict();
    eps_rows16_kernel<<<B * KP / 16, 64>>>(eps, out);
    evict();
    stream16_kernel<<<2048, 256>>>(reinterpret_cast<const float4*>(eps), n / 4, out);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  std::printf("known bytes per launch: %.0f (config #4 eps, 64 solves)\n", bytes);
  return 0;
}
