// Host build of csrc/costs.h's branch-free sincos_fast / cos_fast (the analytic cartpole dynamics and the cartpole
// costs use them on the device) against double-precision libm: prints the max abs errors over a dense grid per
// range, then sin/cos of NaN and inf.  Driven by tests/test_native_math.py.
#include <cmath>
#include <cstdio>

#include "../../humanoid_mppi-rl_amd/csrc/costs.h"

int main() {
  const double lims[] = {4.0, 64.0, 8192.0};
  for (double lim : lims) {
    double es = 0.0, ec = 0.0, e1 = 0.0;
    const long n = 2000000;
    for (long i = 0; i <= n; ++i) {
      const float x = (float)(-lim + 2.0 * lim * (double)i / (double)n);
      float s, c;
      mppi::sincos_fast(x, &s, &c);
      es = std::fmax(es, std::fabs((double)s - std::sin((double)x)));
      ec = std::fmax(ec, std::fabs((double)c - std::cos((double)x)));
      e1 = std::fmax(e1, std::fabs((double)mppi::cos_fast(x) - (double)c));
    }
    std::printf("%g %.3e %.3e %.3e\n", lim, es, ec, e1);
  }
  float s, c;
  mppi::sincos_fast(NAN, &s, &c);
  const bool nan_ok = std::isnan(s) && std::isnan(c);
  mppi::sincos_fast(INFINITY, &s, &c);
  std::printf("nonfinite %d\n", (int)(nan_ok && std::isnan(s) && std::isnan(c)));
  return 0;
}
