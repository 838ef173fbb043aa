// Counter-based Gaussian noise for the MPPI sample step.
//
// Replaces the reference's stateful global RNG draws (np.random.randn(nu,T,K)*sigma at
// src/cartpole_mppi.py:89, randn(nu,H,K)*Σ at src/Humanoid_mppi_v3.jl:156, torch.randn at
// src/cartpole_mppi_estimator.py:127) with Philox4x32-10 (Salmon et al., SC'11) + Box-Muller, so every
// element eps[b][u][t][k] is a pure function of (seed, b, u, t, k): any kernel can regenerate it and
// the result is independent of launch geometry. Bitwise parity with numpy/Julia streams is impossible;
// parity runs inject the reference's seeded noise instead (mppi_io.noise).
//
// Counter layout for one call: c = (k/4, t, u, b), key = (seed_lo, seed_hi); the 4 outputs feed
// 2 Box-Muller pairs -> normals for k = 4*(k/4) + {0,1,2,3}.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define MPPI_HD __host__ __device__ __forceinline__
#else
#define MPPI_HD inline
#endif

struct mppi_u4 {
  uint32_t x, y, z, w;
};

MPPI_HD void philox_mulhilo(uint32_t a, uint32_t b, uint32_t* hi, uint32_t* lo) {
  const uint64_t p = (uint64_t)a * (uint64_t)b;
  *hi = (uint32_t)(p >> 32);
  *lo = (uint32_t)p;
}

MPPI_HD mppi_u4 philox4x32_10(mppi_u4 c, uint32_t k0, uint32_t k1) {
#if defined(__HIPCC__)
#pragma unroll
#endif
  for (int r = 0; r < 10; ++r) {
    uint32_t hi0, lo0, hi1, lo1;
    philox_mulhilo(0xD2511F53u, c.x, &hi0, &lo0);
    philox_mulhilo(0xCD9E8D57u, c.z, &hi1, &lo1);
    mppi_u4 n;
#if defined(__HIP_DEVICE_COMPILE__)
    // gfx950's three-input bitwise op (truth table 0x96 = a ^ b ^ c): one VALU op instead of two v_xor_b32
    n.x = __builtin_amdgcn_bitop3_b32(hi1, c.y, k0, 0x96);
    n.z = __builtin_amdgcn_bitop3_b32(hi0, c.w, k1, 0x96);
#else
    n.x = hi1 ^ c.y ^ k0;
    n.z = hi0 ^ c.w ^ k1;
#endif
    n.y = lo1;
    n.w = lo0;
    c = n;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// 24-bit uniforms: u1 in (0,1] (log-safe), u2 in [0,1).
MPPI_HD float philox_u01_open0(uint32_t v) { return (float)((v >> 8) + 1u) * (1.0f / 16777216.0f); }
MPPI_HD float philox_u01(uint32_t v) { return (float)(v >> 8) * (1.0f / 16777216.0f); }

// Four N(0,1) normals for counter (kq, t, u, b).
#if defined(__HIPCC__)
__device__ __forceinline__ void philox_normal4(uint32_t kq, uint32_t t, uint32_t u, uint32_t b, uint32_t k0,
                                               uint32_t k1, float out[4]) {
  mppi_u4 c = {kq, t, u, b};
  mppi_u4 r = philox4x32_10(c, k0, k1);
  // native v_log_f32 (log2), v_sqrt_f32, v_sin/v_cos_f32 (argument in revolutions): Box-Muller needs
  // sin(2*pi*u) for u in [0,1), exactly the hardware form; ~1e-6 accuracy, no libm slow paths.
  const float ln2x2 = 2.0f * 0.69314718055994531f;
  const float r0 = __builtin_amdgcn_sqrtf(-ln2x2 * __builtin_amdgcn_logf(philox_u01_open0(r.x)));
  const float r1 = __builtin_amdgcn_sqrtf(-ln2x2 * __builtin_amdgcn_logf(philox_u01_open0(r.z)));
  const float a0 = philox_u01(r.y), a1 = philox_u01(r.w);
  out[0] = r0 * __builtin_amdgcn_cosf(a0);
  out[1] = r0 * __builtin_amdgcn_sinf(a0);
  out[2] = r1 * __builtin_amdgcn_cosf(a1);
  out[3] = r1 * __builtin_amdgcn_sinf(a1);
}
#endif
