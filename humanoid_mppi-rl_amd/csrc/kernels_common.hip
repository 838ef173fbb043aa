// Dynamics-independent MPPI kernels: device noise, softmin + weighted-noise reduce, U update/shift,
// and the analytic cartpole rollout.
//
// HBM layout (k fastest = "state-major", numpy's (nu,T,K) C order of src/cartpole_mppi.py:89):
//   noise [B][nu][H][Kp]   costs [B][Kp]   U/dU [B][nu][H]   x0 [B][nx]
#include <hip/hip_runtime.h>

#include "costs.h"
#include "mppi_internal.h"
#include "philox.h"

namespace mppi {

// ------------------------------------------------------------------------------------------------
// a1: eps[b][u][t][k] = sigma * N(0,1) (Philox4x32-10); one thread = 4 consecutive k, 16-B store.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void noise_kernel(float* __restrict__ noise, int rows /*B*nu*H*/, int nu, int H,
                                                    int Kp, uint32_t k0, uint32_t k1, float sigma) {
  const int q_per_row = Kp >> 2;
  const long total = (long)rows * q_per_row;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int row = (int)(i / q_per_row);
    const int kq = (int)(i - (long)row * q_per_row);
    const int t = row % H;
    const int bu = row / H;
    const int u = bu % nu;
    const int b = bu / nu;
    float z[4];
    philox_normal4((uint32_t)kq, (uint32_t)t, (uint32_t)u, (uint32_t)b, k0, k1, z);
    float4 v = make_float4(sigma * z[0], sigma * z[1], sigma * z[2], sigma * z[3]);
    *reinterpret_cast<float4*>(noise + (long)row * Kp + 4 * kq) = v;
  }
}

hipError_t launch_noise(const SolveArgs& a, uint64_t seed, float sigma, hipStream_t stream) {
  const int rows = a.B * a.nu * a.H;
  const long work = (long)rows * (a.Kp / 4);
  int grid = (int)((work + 255) / 256);
  if (grid > 8192) grid = 8192;
  hipLaunchKernelGGL(noise_kernel, dim3(grid), dim3(256), 0, stream, a.noise, rows, a.nu, a.H, a.Kp,
                     (uint32_t)seed, (uint32_t)(seed >> 32), sigma);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// Wave / block reductions (fixed order -> bitwise deterministic).
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ __forceinline__ float wave_min(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o));
  return v;
}

// ------------------------------------------------------------------------------------------------
// a7 + a8: softmin weights and dU[b][u][t] = sum_k w_k eps[b][u][t][k] / (sum_k w_k + eps_norm).
// grid = (row chunks, B), 256 threads. Every block recomputes beta and sum(w) for its solve from the
// K costs (<= 128 KiB, L2-resident) and stages w in LDS; then each wave streams whole noise rows
// with 16-B loads (the HBM-bound part: each noise element is read exactly once).
// References: src/cartpole_mppi.py:92-98, src/mppi.jl:87-94, src/cartpole_mppi_estimator.py:131-143.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void reduce_kernel(SolveArgs a, int rows_per_block) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* w = smem;                // [Kp]
  float* red = smem + a.Kp;       // [8] scratch
  const int b = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const float* c = a.costs + (long)b * a.Kp;

  // beta = min over finite costs (non-finite -> +inf -> weight 0: the documented NaN guard)
  float m = INFINITY;
  for (int k = tid; k < a.K; k += 256) {
    const float ck = c[k];
    m = fminf(m, isfinite(ck) ? ck : INFINITY);
  }
  m = wave_min(m);
  if (lane == 0) red[wv] = m;
  __syncthreads();
  const float beta = fminf(fminf(red[0], red[1]), fminf(red[2], red[3]));
  __syncthreads();
  const float inv_lam = 1.0f / a.lambda;
  float s = 0.0f;
  for (int k = tid; k < a.Kp; k += 256) {
    float wk = 0.0f;
    if (k < a.K) {
      const float ck = c[k];
      wk = (isfinite(ck) && beta < INFINITY) ? __expf(-inv_lam * (ck - beta)) : 0.0f;
    }
    w[k] = wk;
    s += wk;
  }
  s = wave_sum(s);
  if (lane == 0) red[4 + wv] = s;
  __syncthreads();
  const float S = (red[4] + red[5]) + (red[6] + red[7]);
  const float inv_S = 1.0f / (S + a.norm_eps);
  if (blockIdx.x == 0) {
    if (a.weights)
      for (int k = tid; k < a.Kp; k += 256) a.weights[(long)b * a.Kp + k] = w[k] * inv_S;
    if (tid == 0 && !(beta < INFINITY)) atomicOr(a.status, 1u);
  }

  const int rows = a.nu * a.H;
  const int r0 = blockIdx.x * rows_per_block;
  const int r1 = min(rows, r0 + rows_per_block);
  typedef float f4 __attribute__((ext_vector_type(4)));
  const f4* w4 = reinterpret_cast<const f4*>(w);
  const int nq = a.Kp >> 2;
  for (int r = r0 + wv; r < r1; r += 4) {
    const f4* e4 = reinterpret_cast<const f4*>(a.noise + ((long)b * rows + r) * a.Kp);
    float acc = 0.0f;
    for (int q = lane; q < nq; q += 64) {
      const f4 e = __builtin_nontemporal_load(e4 + q);
      const f4 ww = w4[q];
      acc = fmaf(e.x, ww.x, acc);
      acc = fmaf(e.y, ww.y, acc);
      acc = fmaf(e.z, ww.z, acc);
      acc = fmaf(e.w, ww.w, acc);
    }
    acc = wave_sum(acc);
    if (lane == 0) a.dU[(long)b * rows + r] = acc * inv_S;
  }
}

hipError_t launch_reduce(const SolveArgs& a, hipStream_t stream) {
  const int rows = a.nu * a.H;
  // ~1 row per wave when rows are few (small solves are latency-bound), up to 16 per block otherwise.
  int rpb = rows >= 4096 ? 16 : (rows >= 1024 ? 8 : 4);
  const dim3 grid((rows + rpb - 1) / rpb, a.B);
  const size_t lds = (size_t)(a.Kp + 8) * sizeof(float);
  hipLaunchKernelGGL(reduce_kernel, grid, dim3(256), lds, stream, a, rpb);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// a8 (update) + a9 (controller shift). One block per solve; in place (all reads before the barrier).
//   ADD:     U = clamp(U + dU)      REPLACE: U = clamp(dU)
//   SHIFT:   u0 = U[:,0]; U[:,t] = U[:,t+1]; U[:,H-1] = fill * U[:,H-1]     (src/cartpole_mppi.py:101-106)
//   U0_BEFORE: u0 = U_old[:,0]   (src/quadruped_datacollection.py:170)
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void update_kernel(SolveArgs a) {
  extern __shared__ __attribute__((aligned(16))) float su[];  // [nu*H]
  const int b = blockIdx.x;
  const int rows = a.nu * a.H;
  float* U = a.U + (long)b * rows;
  const float* dU = a.dU + (long)b * rows;
  const bool before = (a.flags & MPPI_FLAG_U0_BEFORE) != 0;
  for (int r = threadIdx.x; r < rows; r += blockDim.x) {
    const float old = U[r];
    float v = (a.update_mode == MPPI_UPDATE_REPLACE ? 0.0f : old) + dU[r];
    if (a.U_clamp > 0.0f) v = fminf(a.U_clamp, fmaxf(-a.U_clamp, v));
    su[r] = v;
    const int t = r % a.H;
    if (t == 0 && a.u0) a.u0[(long)b * a.nu + r / a.H] = before ? old : v;
  }
  __syncthreads();
  const bool shift = (a.flags & MPPI_FLAG_SHIFT) != 0;
  for (int r = threadIdx.x; r < rows; r += blockDim.x) {
    const int t = r % a.H;
    float v = su[r];
    // after U[:, :-1] = U[:, 1:], the reference's U[:, -2] is the old last column: fill * su[t = H-1]
    if (shift) v = (t < a.H - 1) ? su[r + 1] : a.shift_fill * su[r];
    U[r] = v;
  }
}

hipError_t launch_update(const SolveArgs& a, hipStream_t stream) {
  const size_t lds = (size_t)a.nu * a.H * sizeof(float);
  hipLaunchKernelGGL(update_kernel, dim3(a.B), dim3(256), lds, stream, a);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// a2-a6 for the analytic cartpole (models/cartpole.xml): one lane per sample, the H loop in
// registers, U[b] staged in LDS; writes costs[b][k]. Dynamics = oracle/mppi_ref.py::cartpole_step,
// which reproduces the recorded MuJoCo trajectory data/2025-04-21_011138 to 1.1e-16 (fp64).
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void cartpole_rollout_kernel(SolveArgs a, CartpoleParams p) {
  extern __shared__ __attribute__((aligned(16))) float sU[];  // [H]
  const int b = blockIdx.y;
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  for (int t = threadIdx.x; t < a.H; t += blockDim.x) sU[t] = a.U[(long)b * a.H + t];  // nu == 1
  __syncthreads();
  if (k >= a.Kp) return;
  const float* xb = a.x0 + (long)b * a.nx;
  float pos = xb[0], th = xb[1], xd = xb[2], thd = xb[3];
  const float dt = p.dt, D = p.damping, mp = p.m_pole, l = p.l;
  const float m11 = p.m_cart + mp + dt * D;
  const float m22 = mp * l * l + p.inertia + dt * D;
  const float mpl = mp * l;
  const float* e = a.noise + (long)b * a.H * a.Kp + k;
  float ctx[MPPI_CTX_MAX];
#pragma unroll
  for (int i = 0; i < MPPI_CTX_MAX; ++i) ctx[i] = a.ctx ? a.ctx[(long)b * MPPI_CTX_MAX + i] : a.ctx_default[i];
  float cost = 0.0f;
  float v[4];
  for (int t = 0; t < a.H; ++t) {
    float u = sU[t] + e[(long)t * a.Kp];
    if (a.ctrl_clamp > 0.0f) u = fminf(a.ctrl_clamp, fmaxf(-a.ctrl_clamp, u));
    const float F = p.gear * fminf(p.ctrl_hi, fmaxf(p.ctrl_lo, u));
    float s, c;
    sincosf(th, &s, &c);
    const float m12 = mpl * c;
    const float f1 = F + mpl * s * thd * thd - D * xd;
    const float f2 = mpl * p.g * s - D * thd;
    const float inv_det = 1.0f / (m11 * m22 - m12 * m12);
    const float a1 = (m22 * f1 - m12 * f2) * inv_det;
    const float a2 = (m11 * f2 - m12 * f1) * inv_det;
    xd = xd + dt * a1;
    thd = thd + dt * a2;
    pos = pos + dt * xd;
    th = th + dt * thd;
    v[0] = pos; v[1] = th; v[2] = xd; v[3] = thd;
    cost += cost_eval(a.cost_kind, v, u, u * u, ctx);
  }
  if (a.terminal_weight != 0.0f) cost += a.terminal_weight * cost_eval(a.cost_kind, v, 0.0f, 0.0f, ctx);
  if (k < a.K) a.costs[(long)b * a.Kp + k] = isfinite(cost) ? cost : INFINITY;
}

hipError_t launch_cartpole_rollout(const SolveArgs& a, const CartpoleParams& p, hipStream_t stream) {
  const dim3 grid((a.Kp + 255) / 256, a.B);
  hipLaunchKernelGGL(cartpole_rollout_kernel, grid, dim3(256), (size_t)a.H * sizeof(float), stream, a, p);
  return hipGetLastError();
}

}  // namespace mppi
