// The HBM ceiling of the chained solve's reduce: reduce_kernel<GEN> reads this solve's noise
// (config #4, 64 solves: 352 MB) and writes the next solve's (352 MB) in one pass.  This probe times the same byte
// streams with no arithmetic on them, on the same box: a read-only sweep, a write-only sweep and a copy (read one
// 352 MB buffer, write another), float4 per lane, plain and nontemporal, grid-stride, a 1 GiB eviction sweep before
// each launch so nothing is served from the Infinity Cache (256 MiB).  The copy's time is the floor for the reduce.
//   hipcc -O3 --offload-arch=gfx950 -o tools/copy_probe tools/copy_probe.hip && tools/copy_probe
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f4 __attribute__((ext_vector_type(4)));

template <bool NT>
__global__ __launch_bounds__(256) void read_kernel(const f4* __restrict__ src, long n4, float* __restrict__ out) {
  f4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long)gridDim.x * 256)
    acc += NT ? __builtin_nontemporal_load(src + i) : src[i];
  if (acc.x + acc.y + acc.z + acc.w == 12345.678f) out[blockIdx.x] = 1.0f;  // never true for the zero buffer
}

template <bool NT>
__global__ __launch_bounds__(256) void write_kernel(f4* __restrict__ dst, long n4) {
  const f4 v = {1.0f, 2.0f, 3.0f, (float)blockIdx.x};
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    if constexpr (NT)
      __builtin_nontemporal_store(v, dst + i);
    else
      dst[i] = v;
  }
}

template <bool NT>
__global__ __launch_bounds__(256) void copy_kernel(const f4* __restrict__ src, f4* __restrict__ dst, long n4) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    if constexpr (NT)
      __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
    else
      dst[i] = src[i];
  }
}

int main() {
  const long bytes = 64L * 21 * 64 * 1024 * 4;  // config #4's noise at 64 solves: 352,321,536 B
  const long n4 = bytes / 16;
  f4 *a, *b;
  float *out, *big;
  const long nb = 1L << 30;
  if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&b, bytes) != hipSuccess || hipMalloc(&out, 1 << 20) != hipSuccess ||
      hipMalloc(&big, nb) != hipSuccess)
    return 1;
  (void)hipMemset(a, 0, bytes);
  (void)hipMemset(b, 0, bytes);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  auto timed = [&](const char* name, double moved, auto launch) {
    double best = 1e30, sum = 0.0;
    const int reps = 10;
    for (int r = 0; r < reps + 2; ++r) {
      (void)hipMemset(big, r & 1, nb);  // evict L2 / the Infinity Cache
      (void)hipEventRecord(e0);
      launch();
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms = 0.0f;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (r >= 2) {  // the first two: clock ramp
        best = ms < best ? ms : best;
        sum += ms;
      }
    }
    std::printf("%-28s %8.1f us avg  %8.1f us best  %5.2f TB/s avg (%.0f MB moved)\n", name, 1e3 * sum / reps, 1e3 * best,
                moved / (sum / reps * 1e-3) / 1e12, moved / 1e6);
  };
  for (int grid : {1024, 2048, 4096}) {
    std::printf("grid %d x 256 threads\n", grid);
    timed("read (plain)", bytes, [&] { read_kernel<false><<<grid, 256>>>(a, n4, out); });
    timed("read (nontemporal)", bytes, [&] { read_kernel<true><<<grid, 256>>>(a, n4, out); });
    timed("write (plain)", bytes, [&] { write_kernel<false><<<grid, 256>>>(b, n4); });
    timed("write (nontemporal)", bytes, [&] { write_kernel<true><<<grid, 256>>>(b, n4); });
    timed("copy (plain)", 2.0 * bytes, [&] { copy_kernel<false><<<grid, 256>>>(a, b, n4); });
    timed("copy (nontemporal)", 2.0 * bytes, [&] { copy_kernel<true><<<grid, 256>>>(a, b, n4); });
  }
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
