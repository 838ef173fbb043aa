// Accuracy of gfx950's native v_sin_f32 / v_cos_f32 (via __sinf / __cosf) and of costs.h::sincos_fast against
// double-precision libm, over |x| <= R (diagnostic: may the analytic cartpole use the native ops?).
//   hipcc -O3 --offload-arch=gfx950 -I../include tools/native_trig_probe.hip -o /tmp/trig && /tmp/trig
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <vector>

#include "../humanoid_mppi-rl_amd/csrc/costs.h"

__global__ void trig(const float* x, float* out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float s, c;
  mppi::sincos_fast(x[i], &s, &c);
  out[4 * i + 0] = __sinf(x[i]);
  out[4 * i + 1] = __cosf(x[i]);
  out[4 * i + 2] = s;
  out[4 * i + 3] = c;
}

int main() {
  const float R[] = {4.0f, 8.0f, 32.0f, 256.0f};
  for (float r : R) {
    const int n = 1 << 22;
    std::vector<float> x(n), o(4 * (size_t)n);
    for (int i = 0; i < n; ++i) x[i] = -r + 2.0f * r * (float)i / (float)(n - 1);
    float *dx, *dout;
    if (hipMalloc(&dx, n * 4) != hipSuccess || hipMalloc(&dout, 16 * (size_t)n) != hipSuccess) return 1;
    hipMemcpy(dx, x.data(), n * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(trig, dim3((n + 255) / 256), dim3(256), 0, 0, dx, dout, n);
    hipMemcpy(o.data(), dout, 16 * (size_t)n, hipMemcpyDeviceToHost);
    double e[4] = {0, 0, 0, 0};
    for (int i = 0; i < n; ++i) {
      const double s = std::sin((double)x[i]), c = std::cos((double)x[i]);
      e[0] = std::fmax(e[0], std::fabs(o[4 * i + 0] - s));
      e[1] = std::fmax(e[1], std::fabs(o[4 * i + 1] - c));
      e[2] = std::fmax(e[2], std::fabs(o[4 * i + 2] - s));
      e[3] = std::fmax(e[3], std::fabs(o[4 * i + 3] - c));
    }
    printf("|x| <= %g: native sin %.3g cos %.3g | sincos_fast sin %.3g cos %.3g (max abs err vs double)\n", r, e[0],
           e[1], e[2], e[3]);
    hipFree(dx);
    hipFree(dout);
  }
  return 0;
}
