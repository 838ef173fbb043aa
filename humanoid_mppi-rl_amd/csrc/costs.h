// Running costs of the reference controllers, evaluated per (sample, step) in fp32.
// Each cost reads a small, fixed set of state entries (kCostIdx); the rollout kernels gather
// exactly those (register shuffles in the fc-stack kernel) and call cost_eval().
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
         : kind == MPPI_COST_HUMANOID_V3 ? CostIdx{9, {0, 1, 2, 3, 4, 5, 6, 28, 29}}
         // qpos[2:3], qpos[7:8] (1-based), qvel[1:2], qvel[7:9]  (src/mppi.jl:34-37; nq = 19)
         : kind == MPPI_COST_QUAD_JL ? CostIdx{9, {1, 2, 6, 7, 19, 20, 25, 26, 27}}
         : kind == MPPI_COST_QUAD_EST ? CostIdx{3, {0, 1, 2}}
                                      : CostIdx{0, {}};
}

// v: the gathered state entries (cost_idx order); usq = sum_u u^2 of the control used in this step
// (0 for the terminal term); u0 = first control (cartpole ctrl term); ctx: per-solve context row.
__device__ __forceinline__ float cost_eval(int kind, const float* v, float u0, float usq, const float* ctx) {
  switch (kind) {
    case MPPI_COST_CARTPOLE: {  // src/cartpole_mppi.py:44-50
      const float c = cosf(v[1]) - 1.0f;
      return v[0] * v[0] + 20.0f * c * c + 0.1f * v[2] * v[2] + 0.1f * v[3] * v[3] + 0.01f * u0 * u0;
    }
    case MPPI_COST_CARTPOLE_EST: {  // src/cartpole_mppi_estimator.py:46-52
      return v[0] * v[0] + 50.0f * fabsf(cosf(v[1]) - 1.0f) + 0.1f * v[2] * v[2] + 0.1f * v[3] * v[3];
    }
    case MPPI_COST_HUMANOID_V3: {  // src/Humanoid_mppi_v3.jl:27-105 (real-env terms folded into ctx)
      const float px = v[0], py = v[1], pz = v[2];
      const float q0 = v[3], q1 = v[4], q2 = v[5], q3 = v[6];
      const float roll = atan2f(2.0f * (q0 * q1 + q2 * q3), 1.0f - 2.0f * (q1 * q1 + q2 * q2));
      const float pitch = asinf(fminf(1.0f, fmaxf(-1.0f, 2.0f * (q0 * q2 - q3 * q1))));
      const float yaw = atan2f(2.0f * (q0 * q3 + q1 * q2), 1.0f - 2.0f * (q2 * q2 + q3 * q3));
      float c = 5.0f * (roll * roll + pitch * pitch) + 0.075f * yaw * yaw;
      c += 12.5f * hypotf(px - ctx[0], py - ctx[1]);
      c += 5.0f * fabsf(ctx[2] - pz);
      c += hypotf(v[7] - 0.3f, v[8]);
      const float ftx = px + 0.5f;
      c += 8.0f * fabsf(ctx[3] - ftx);
      const float dk = ctx[4] - ftx;
      c += 3.0f * dk * dk + ctx[5];
      return c + 0.01f * usq;
    }
    case MPPI_COST_QUAD_JL: {  // src/mppi.jl:18-62
      const float h = v[1] - 0.45f, vx = v[4] - 0.6f;
      return 500.0f * h * h + 1000.0f * vx * vx + 500.0f * (v[2] * v[2] + v[3] * v[3]) +
             20.0f * (v[6] * v[6] + v[7] * v[7] + v[8] * v[8]) + 1000.0f * (v[0] * v[0] + v[5] * v[5]) + 0.1f * usq;
    }
    case MPPI_COST_QUAD_EST: {  // src/quadruped_mppi_estimator.py:48-52
      const float a = v[0] - ctx[0], b = v[1] - ctx[1], c = v[2] - ctx[2];
      return a * a + b * b + c * c + 0.1f * usq;
    }
    default:
      return __builtin_nanf("");
  }
}

}  // namespace mppi
