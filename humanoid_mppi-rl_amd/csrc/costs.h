// Running costs of the reference controllers, evaluated per (sample, step) in fp32.
// Each cost reads a small, fixed set of state entries (cost_idx); the rollout kernels gather exactly those
// and call cost_eval<KIND>().  Trigonometry is branch-free minimax (Cephes single-precision coefficients,
// |rel err| ~1e-7): libm's atan2f/asinf/hypotf expand to branchy slow paths that dominated the horizon step.
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/mppi.h"

namespace mppi {

constexpr int kCostMaxIdx = 10;

// State indices (0-based, x = [qpos, qvel]) each cost reads, in the order cost_eval expects them.
struct CostIdx {
  int n;
  int idx[kCostMaxIdx];
};

__host__ __device__ constexpr CostIdx cost_idx(int kind) {
  return kind == MPPI_COST_CARTPOLE || kind == MPPI_COST_CARTPOLE_EST ? CostIdx{4, {0, 1, 2, 3}}
         // root xyz, quat wxyz, root vx vy  (src/Humanoid_mppi_v3.jl:30-35; nq = 28)
         : kind == MPPI_COST_HUMANOID_V3 || kind == MPPI_COST_HUMANOID_V1 ? CostIdx{9, {0, 1, 2, 3, 4, 5, 6, 28, 29}}
         // qpos[2:3], qpos[7:8] (1-based), qvel[1:2], qvel[7:9]  (src/mppi.jl:34-37; nq = 19)
         : kind == MPPI_COST_QUAD_JL ? CostIdx{9, {1, 2, 6, 7, 19, 20, 25, 26, 27}}
         : kind == MPPI_COST_QUAD_EST ? CostIdx{3, {0, 1, 2}}
                                      : CostIdx{0, {}};
}

// ---- branch-free trig (selects, one reciprocal). Hardware v_rcp_f32 / v_sqrt_f32 (~1 ulp): HIP's __fdividef
// and sqrtf expand to IEEE division / denormal-scaling sequences (~10 VALU each) in this issue-bound loop.
__device__ __forceinline__ float fast_div(float a, float b) { return a * __builtin_amdgcn_rcpf(b); }
__device__ __forceinline__ float fast_sqrt(float a) { return __builtin_amdgcn_sqrtf(a); }

__device__ __forceinline__ float atan_cephes(float x) {
  const float a = fabsf(x);
  const bool big = a > 2.414213562373095f, mid = a > 0.4142135623730950f;
  const float num = big ? -1.0f : (mid ? a - 1.0f : a);
  const float den = big ? a : (mid ? a + 1.0f : 1.0f);
  const float y0 = big ? 1.5707963267948966f : (mid ? 0.7853981633974483f : 0.0f);
  const float r = fast_div(num, den);
  const float z = r * r;
  const float p =
      fmaf(fmaf(fmaf(fmaf(8.05374449538e-2f, z, -1.38776856032e-1f), z, 1.99777106478e-1f), z, -3.33329491539e-1f),
           z * r, r);
  return copysignf(y0 + p, x);
}

__device__ __forceinline__ float atan2_fast(float y, float x) {
  float t = atan_cephes(fast_div(y, x));
  const float pi = 3.14159265358979323846f;
  t = x < 0.0f ? t + copysignf(pi, y) : t;
  // x == 0: (y == 0 ? 0 : +-pi/2), selected through a lane mask -- the plain nested select became a divergent branch
  // (exec-mask save / skip), a basic-block boundary the scheduler does not move the rest of the cost across
  const float z0 = y == 0.0f ? 0.0f : copysignf(0.5f * pi, y);
  const unsigned m = 0u - (unsigned)(x == 0.0f);
  return __uint_as_float((__float_as_uint(z0) & m) | (__float_as_uint(t) & ~m));
}

__device__ __forceinline__ float asin_fast(float x) {  // x clamped to [-1, 1] by the caller
  const float a = fabsf(x);
  const bool hi = a > 0.5f;
  const float z = hi ? 0.5f * (1.0f - a) : a * a;
  const float s = hi ? fast_sqrt(z) : a;
  const float p =
      fmaf(fmaf(fmaf(fmaf(fmaf(4.2163199048e-2f, z, 2.4181311049e-2f), z, 4.5470025998e-2f), z, 7.4953002686e-2f), z,
                1.6666752422e-1f),
           z * s, s);
  return copysignf(hi ? 1.5707963267948966f - 2.0f * p : p, x);
}

// sin(x), cos(x) branch-free: Cephes sinf/cosf's 3-part Cody-Waite reduction by pi/2 and their minimax polynomials on
// [-pi/4, pi/4]; max abs err 7e-8 for |x| <= 8192 (libm: 3e-8, through a branchy path whose Payne-Hanek large-argument
// reduction is ~200 instructions).  NaN / inf -> NaN.  The analytic cartpole carries sin/cos of theta in its per-step
// dependency chain, the FA kernels' single cost-evaluating wave ran libm cosf every step
__host__ __device__ __forceinline__ void sincos_fast(float x, float* sn, float* cs) {
  // nearest multiple j of pi/2 by the 1.5 * 2^23 shifter: t's low mantissa bits ARE j (two's complement, |j| < 2^22),
  // so the quadrant needs no float -> int conversion (undefined for NaN); NaN / inf still flow into r below
  const float t = fmaf(x, 0.63661977236758134f, 12582912.0f);
  const float j = t - 12582912.0f;
  float r = fmaf(j, -1.5703125f, x);
  r = fmaf(j, -4.837512969970703125e-4f, r);
  r = fmaf(j, -7.54978995489188216e-8f, r);
  const float z = r * r;
  const float c =
      fmaf(fmaf(fmaf(fmaf(2.443315711809948e-5f, z, -1.388731625493765e-3f), z, 4.166664568298827e-2f), z, -0.5f), z,
           1.0f);
  const float s = fmaf(fmaf(fmaf(-1.9515295891e-4f, z, 8.3321608736e-3f), z, -1.6666654611e-1f), z * r, r);
  const int q = __builtin_bit_cast(int, t) & 3;  // quadrant: (sin, cos) = (s, c), (c, -s), (-s, -c), (-c, s)
  const float sv = (q & 1) ? c : s, cv = (q & 1) ? s : c;
  *sn = (q & 2) ? -sv : sv;
  *cs = ((q + 1) & 2) ? -cv : cv;
}
__host__ __device__ __forceinline__ float cos_fast(float x) {
  float s, c;
  sincos_fast(x, &s, &c);
  return c;
}

// v: the gathered state entries (cost_idx order); usq = sum_u u^2 of the control used in this step
// (0 for the terminal term); u0 = first control (cartpole ctrl term); ctx: per-solve context row; t1: the reference's
// 1-based rollout step t (1..H; the terminal term passes H, src/Humanoid_mppi.jl:135,158-160) -- only humanoid_v1
// reads it.
// The cartpole costs from cos(theta) (the analytic rollout carries cos from its dynamics step).
template <int KIND>
__device__ __forceinline__ float cartpole_cost_c(float x, float cth, float xd, float thd, float u0) {
  if constexpr (KIND == MPPI_COST_CARTPOLE) {  // src/cartpole_mppi.py:44-50
    const float c = cth - 1.0f;
    return x * x + 20.0f * c * c + 0.1f * xd * xd + 0.1f * thd * thd + 0.01f * u0 * u0;
  } else {  // MPPI_COST_CARTPOLE_EST, src/cartpole_mppi_estimator.py:46-52
    return x * x + 50.0f * fabsf(cth - 1.0f) + 0.1f * xd * xd + 0.1f * thd * thd;
  }
}

template <int KIND>
__device__ __forceinline__ float cost_eval_t(const float* v, float u0, float usq, const float* ctx, int t1) {
  if constexpr (KIND == MPPI_COST_CARTPOLE || KIND == MPPI_COST_CARTPOLE_EST) {
    (void)t1;
    return cartpole_cost_c<KIND>(v[0], cos_fast(v[1]), v[2], v[3], u0);
  } else if constexpr (KIND == MPPI_COST_HUMANOID_V3) {  // src/Humanoid_mppi_v3.jl:27-105 (real-env terms in ctx)
    const float px = v[0], py = v[1], pz = v[2];
    const float q0 = v[3], q1 = v[4], q2 = v[5], q3 = v[6];
    const float roll = atan2_fast(2.0f * (q0 * q1 + q2 * q3), 1.0f - 2.0f * (q1 * q1 + q2 * q2));
    const float pitch = asin_fast(fminf(1.0f, fmaxf(-1.0f, 2.0f * (q0 * q2 - q3 * q1))));
    const float yaw = atan2_fast(2.0f * (q0 * q3 + q1 * q2), 1.0f - 2.0f * (q2 * q2 + q3 * q3));
    float c = 5.0f * (roll * roll + pitch * pitch) + 0.075f * yaw * yaw;
    const float dx = px - ctx[0], dy = py - ctx[1];
    c += 12.5f * fast_sqrt(dx * dx + dy * dy);
    c += 5.0f * fabsf(ctx[2] - pz);
    const float vx = v[7] - 0.3f, vy = v[8];
    c += fast_sqrt(vx * vx + vy * vy);
    const float ftx = px + 0.5f;
    c += 8.0f * fabsf(ctx[3] - ftx);
    const float dk = ctx[4] - ftx;
    c += 3.0f * dk * dk + ctx[5];
    return c + 0.01f * usq;
  } else if constexpr (KIND == MPPI_COST_HUMANOID_V1) {  // src/Humanoid_mppi.jl:31-121 (real-env terms in ctx)
    // ctx = [tx, ty, tz, left_foot_x, right_foot_x, 0.01 (right_foot_z - left_foot_z), 0.1 |left_y - right_y|, 0]
    // (mppi_hip.controller.humanoid_v1_context); the swing foot is the left one while (t mod 100) < 50 (:76-87)
    const float px = v[0], py = v[1], pz = v[2];
    const float q0 = v[3], q1 = v[4], q2 = v[5], q3 = v[6];
    const float roll = atan2_fast(2.0f * (q0 * q1 + q2 * q3), 1.0f - 2.0f * (q1 * q1 + q2 * q2));
    const float pitch = asin_fast(fminf(1.0f, fmaxf(-1.0f, 2.0f * (q0 * q2 - q3 * q1))));
    float c = 5.0f * (roll * roll + pitch * pitch);  // :47-50
    const float dx = px - ctx[0], dy = py - ctx[1];
    c += 12.0f * fast_sqrt(dx * dx + dy * dy);   // :53
    c += 2.25f * (ctx[2] - pz);                 // :57 (signed, not an absolute value)
    const float vx = v[7] - 0.5f, vy = v[8];
    c += fast_sqrt(vx * vx + vy * vy);           // :60
    const bool left = (t1 % 100) < 50;           // :76-87
    const float sw = (left ? ctx[3] : ctx[4]) - (px + 0.5f);
    c += 10.0f * sw * sw;                        // :89-92
    c += left ? ctx[5] : -ctx[5];                // :94-98, 0.01 (stance_z - swing_z)
    c += ctx[6];                                 // :103-106, 0.1 |stance_y - swing_y| (side-independent)
    return c + 0.01f * usq;                      // :118
  } else if constexpr (KIND == MPPI_COST_QUAD_JL) {  // src/mppi.jl:18-62
    const float h = v[1] - 0.45f, vx = v[4] - 0.6f;
    return 500.0f * h * h + 1000.0f * vx * vx + 500.0f * (v[2] * v[2] + v[3] * v[3]) +
           20.0f * (v[6] * v[6] + v[7] * v[7] + v[8] * v[8]) + 1000.0f * (v[0] * v[0] + v[5] * v[5]) + 0.1f * usq;
  } else if constexpr (KIND == MPPI_COST_QUAD_EST) {  // src/quadruped_mppi_estimator.py:48-52
    const float a = v[0] - ctx[0], b = v[1] - ctx[1], c = v[2] - ctx[2];
    return a * a + b * b + c * c + 0.1f * usq;
  } else {
    return __builtin_nanf("");
  }
}

// Control term of the running cost (the part that depends on u only): cost_eval_t(v, u0, usq, ., t) ==
// cost_eval_t(v, 0, 0, ., t) + ctrl_term_t(u0, usq) for every kind.  The fc rollouts add it at their cost-ring flush from
// U and the noise of the flushed (step, sample), so their per-step loop never touches u.
template <int KIND>
__device__ __forceinline__ float ctrl_term_t(float u0, float usq) {
  if constexpr (KIND == MPPI_COST_CARTPOLE) return 0.01f * u0 * u0;               // src/cartpole_mppi.py:50
  else if constexpr (KIND == MPPI_COST_HUMANOID_V3) return 0.01f * usq;            // src/Humanoid_mppi_v3.jl:102
  else if constexpr (KIND == MPPI_COST_HUMANOID_V1) return 0.01f * usq;            // src/Humanoid_mppi.jl:118
  else if constexpr (KIND == MPPI_COST_QUAD_JL || KIND == MPPI_COST_QUAD_EST) return 0.1f * usq;
  else return 0.0f;                                                                // cartpole_est: no ctrl term
}

}  // namespace mppi
