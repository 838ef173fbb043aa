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
// a1: eps[b][u][t][k] = sigma * N(0,1) (Philox4x32-10, counter (k/4, t, u, b)).  A block = 64 quads of k (one
// wave-wide 1 KiB store per control row) x 4 control groups; thread (uq, kq) generates rows u = uq, uq+4, ... of
// one (b, t) with 16-B nontemporal stores.  For the fc rollouts the same pass emits the control term of the
// running cost, ctrl_cost[b][t][k] = ctrl_term(clamp(U + eps)) (costs.h; sum over u combined in LDS), so those
// rollouts never load u.  GEN = false: eps was injected (parity runs); only ctrl_cost.
// seed_ctr (graph-replayable solves, MPPI_FLAG_SEED_COUNTER): key = seed + *seed_ctr.
// ------------------------------------------------------------------------------------------------
constexpr int kNoiseUG = 4;  // control groups per block
template <bool GEN>
__global__ __launch_bounds__(256) void noise_kernel(SolveArgs a, uint64_t seed, float sigma) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  __shared__ f4 part[kNoiseUG][64];
  const int row = blockIdx.z * 65535 + blockIdx.y;  // b*H + t
  const int uq = threadIdx.x >> 6;
  const int kq = blockIdx.x * 64 + (threadIdx.x & 63);
  const bool live = row < a.B * a.H && 4 * kq < a.Kp;
  const int b = row / a.H, t = row - b * a.H;
  const uint64_t key = seed + (a.seed_ctr ? *a.seed_ctr : 0ull);
  const uint32_t k0 = (uint32_t)key, k1 = (uint32_t)(key >> 32);
  f4 usq = {0.0f, 0.0f, 0.0f, 0.0f}, u0 = usq;
  const bool cc = a.ctrl_cost != nullptr;
  if (live) {
    for (int u = uq; u < a.nu; u += kNoiseUG) {
      f4* p = reinterpret_cast<f4*>(a.noise + (((long)b * a.nu + u) * a.H + t) * a.Kp) + kq;
      f4 e;
      if constexpr (GEN) {
        float z[4];
        philox_normal4((uint32_t)kq, (uint32_t)t, (uint32_t)u, (uint32_t)b, k0, k1, z);
        e = f4{sigma * z[0], sigma * z[1], sigma * z[2], sigma * z[3]};
        __builtin_nontemporal_store(e, p);
      } else {
        e = *p;
      }
      if (cc) {
        const float Ut = a.U[((long)b * a.nu + u) * a.H + t];
        f4 uc = Ut + e;
        if (a.ctrl_clamp > 0.0f)
          for (int i = 0; i < 4; ++i) uc[i] = fminf(a.ctrl_clamp, fmaxf(-a.ctrl_clamp, uc[i]));
        if (u == 0) u0 = uc;
        usq = uc * uc + usq;
      }
    }
  }
  if (!cc) return;  // uniform
  part[uq][threadIdx.x & 63] = usq;
  __syncthreads();
  if (uq == 0 && live) {
    for (int j = 1; j < kNoiseUG; ++j) usq += part[j][threadIdx.x];  // fixed order
    f4 c;
    for (int i = 0; i < 4; ++i) c[i] = ctrl_term(a.cost_kind, u0[i], usq[i]);
    reinterpret_cast<f4*>(a.ctrl_cost + ((long)b * a.H + t) * a.Kp)[kq] = c;
  }
}

hipError_t launch_noise(const SolveArgs& a, uint64_t seed, float sigma, bool gen, hipStream_t stream) {
  const int rows = a.B * a.H;
  const dim3 grid((a.Kp / 4 + 63) / 64, rows < 65535 ? rows : 65535, (rows + 65534) / 65535);
  if (gen)
    hipLaunchKernelGGL(noise_kernel<true>, grid, dim3(64 * kNoiseUG), 0, stream, a, seed, sigma);
  else
    hipLaunchKernelGGL(noise_kernel<false>, grid, dim3(64 * kNoiseUG), 0, stream, a, seed, sigma);
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

// a8 (update) + a9 (controller shift) for solve b, run by one block; in place (all reads before the barrier).
//   ADD: U = clamp(U + dU)   REPLACE: U = clamp(dU)   SHIFT: u0 = U[:,0]; U[:,t] = U[:,t+1]; U[:,H-1] = fill * U[:,H-1]
//   (src/cartpole_mppi.py:101-106)   U0_BEFORE: u0 = U_old[:,0] (src/quadruped_datacollection.py:170)
__device__ void update_solve(const SolveArgs& a, int b, float* su /* LDS, >= nu*H floats */) {
  const int rows = a.nu * a.H;
  float* U = a.U + (long)b * rows;
  float* dU = a.dU + (long)b * rows;
  const bool before = (a.flags & MPPI_FLAG_U0_BEFORE) != 0;
  __syncthreads();  // su may alias scratch the caller used
  for (int r = threadIdx.x; r < rows; r += blockDim.x) {
    const float old = U[r];
    const float d = __hip_atomic_load(dU + r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // sc1: other blocks' rows
    float v = (a.update_mode == MPPI_UPDATE_REPLACE ? 0.0f : old) + d;
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

// ------------------------------------------------------------------------------------------------
// a7 + a8: softmin weights and dU[b][u][t] = sum_k w_k eps[b][u][t][k] / (sum_k w_k + eps_norm).
// grid = (row chunks, B), 512 threads. Every block recomputes beta and sum(w) for its solve from the
// K costs (<= 128 KiB, L2-resident) and stages w in LDS; then each wave streams whole noise rows
// with 16-B loads (the HBM-bound part: each noise element is read exactly once).
// References: src/cartpole_mppi.py:92-98, src/mppi.jl:87-94, src/cartpole_mppi_estimator.py:131-143.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(512) void reduce_kernel(SolveArgs a, int rows_per_block) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* w = smem;                // [max(Kp, nu*H)]
  float* red = smem + (a.Kp > a.nu * a.H ? a.Kp : a.nu * a.H);  // [8] scratch
  const int b = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, nw = blockDim.x >> 6, nt = blockDim.x;
  const float* c = a.costs + (long)b * a.Kp;
  const int rows = a.nu * a.H;
  const int r0 = blockIdx.x * rows_per_block;
  const int r1 = min(rows, r0 + rows_per_block);
  typedef float f4 __attribute__((ext_vector_type(4)));
  const int nq = a.Kp >> 2;
  // each wave streams kRR rows at once, kRU quads per lane in flight per row (kRR * kRU 16-B loads outstanding)
  constexpr int kRR = 2, kRU = 4;
  f4 e[kRR][kRU];
  auto issue = [&](int r, int q0) {
#pragma unroll
    for (int j = 0; j < kRU; ++j) {
      const int q = min(q0 + 64 * j, nq - 1);
#pragma unroll
      for (int i = 0; i < kRR; ++i)
        e[i][j] = __builtin_nontemporal_load(
            reinterpret_cast<const f4*>(a.noise + ((long)b * rows + min(r + i, r1 - 1)) * a.Kp) + q);
    }
  };
  // the first tile of this wave's first rows does not depend on the weights: in flight during the softmin pass
  const int rfirst = r0 + wv * kRR;
  if (rfirst < r1) issue(rfirst, lane);

  // beta = min over finite costs (non-finite -> +inf -> weight 0: the documented NaN guard)
  float m = INFINITY;
  for (int k = tid; k < a.K; k += nt) {
    const float ck = c[k];
    m = fminf(m, isfinite(ck) ? ck : INFINITY);
  }
  m = wave_min(m);
  if (lane == 0) red[wv] = m;
  __syncthreads();
  float beta = red[0];
  for (int i = 1; i < nw; ++i) beta = fminf(beta, red[i]);
  __syncthreads();
  const float inv_lam = 1.0f / a.lambda;
  float s = 0.0f;
  for (int k = tid; k < a.Kp; k += nt) {
    float wk = 0.0f;
    if (k < a.K) {
      const float ck = c[k];
      wk = (isfinite(ck) && beta < INFINITY) ? __expf(-inv_lam * (ck - beta)) : 0.0f;
    }
    w[k] = wk;
    s += wk;
  }
  s = wave_sum(s);
  if (lane == 0) red[nw + wv] = s;
  __syncthreads();
  float S = 0.0f;
  for (int i = 0; i < nw; ++i) S += red[nw + i];  // fixed order: deterministic
  const float inv_S = 1.0f / (S + a.norm_eps);
  if (blockIdx.x == 0) {
    if (a.weights)
      for (int k = tid; k < a.Kp; k += nt) a.weights[(long)b * a.Kp + k] = w[k] * inv_S;
    if (tid == 0 && !(beta < INFINITY)) atomicOr(a.status, 1u);
  }

  const f4* w4 = reinterpret_cast<const f4*>(w);
  for (int r = rfirst; r < r1; r += nw * kRR) {
    float acc[kRR];
#pragma unroll
    for (int i = 0; i < kRR; ++i) acc[i] = 0.0f;
    for (int q0 = lane; q0 < nq; q0 += 64 * kRU) {
      if (r != rfirst || q0 != lane) issue(r, q0);  // (the first tile is already in flight)
#pragma unroll
      for (int j = 0; j < kRU; ++j) {
        if (q0 + 64 * j < nq) {
          const f4 ww = w4[q0 + 64 * j];
#pragma unroll
          for (int i = 0; i < kRR; ++i) {
            acc[i] = fmaf(e[i][j].x, ww.x, acc[i]);
            acc[i] = fmaf(e[i][j].y, ww.y, acc[i]);
            acc[i] = fmaf(e[i][j].z, ww.z, acc[i]);
            acc[i] = fmaf(e[i][j].w, ww.w, acc[i]);
          }
        }
      }
    }
#pragma unroll
    for (int i = 0; i < kRR; ++i) {
      const float sum = wave_sum(acc[i]);
      // write-through (sc1) store: visible to the last-arriving block of this solve without a release fence
      if (lane == 0 && r + i < r1)
        __hip_atomic_store(a.dU + (long)b * rows + r + i, sum * inv_S, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }

  // ---- a8/a9 fused: the last block to finish solve b applies the update + shift (guide G16, sc1 counter
  // form: sc1 payload stores drained by every storing wave, block barrier, one relaxed agent ticket; the last
  // arriver reads every dU row with sc1 loads, so no release/acquire fences). Ticket reset for the next solve.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // the arrival flag lives in the dynamic LDS scratch (a static __shared__ would shift the 16-B-aligned base)
  unsigned* last_flag = reinterpret_cast<unsigned*>(red + 2 * nw);
  if (tid == 0) {
    const unsigned prev = __hip_atomic_fetch_add(a.tickets + b, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *last_flag = (prev == gridDim.x - 1) ? 1u : 0u;
  }
  __syncthreads();
  if (!*last_flag) return;
  update_solve(a, b, w);  // w (softmin weights) is dead here; the LDS region holds max(Kp, nu*H) floats
  if (tid == 0) {
    __hip_atomic_store(a.tickets + b, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // next solve's noise key (this solve's noise kernel has completed: stream order)
    if (b == 0 && a.seed_ctr) atomicAdd(a.seed_ctr, 1ull);
  }
}

hipError_t launch_reduce(const SolveArgs& a, hipStream_t stream) {
  const int rows = a.nu * a.H;
  // ~512 blocks of 8 waves in total (2 per CU), each wave streaming up to 2 rows with 8 16-B loads in flight
  // per lane; enough rows per block to amortise each block's softmin pass over the K costs.
  int rpb = (rows * a.B + 511) / 512;
  rpb = rpb < 1 ? 1 : rpb;
  const dim3 grid((rows + rpb - 1) / rpb, a.B);
  const size_t lds = (size_t)((a.Kp > a.nu * a.H ? a.Kp : a.nu * a.H) + 32) * sizeof(float);
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(reduce_kernel),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(reduce_kernel, grid, dim3(512), lds, stream, a, rpb);
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
  if (k == 0 && b == 0) *a.status = 0u;  // per-solve status word (read by the host after the reduce)
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
  if (a.xout && k == 0) {
    float* xo = a.xout + (long)b * a.nx;
    xo[0] = pos;
    xo[1] = th;
    xo[2] = xd;
    xo[3] = thd;
  }
}

// ------------------------------------------------------------------------------------------------
// Trajectory logging (mppi_graph_capture_traj): copy x_t [B][nx] and u_t [B][nu] into the log before the env
// step advances x.  Its own tiny launch, so the rollout kernels carry no logging code.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void record_kernel(const float* __restrict__ x, const float* __restrict__ u,
                                                     float* __restrict__ rx, float* __restrict__ ru, int nxB, int nuB) {
  for (int i = blockIdx.x * 256 + threadIdx.x; i < nxB + nuB; i += gridDim.x * 256) {
    if (i < nxB) rx[i] = x[i];
    else ru[i - nxB] = u[i - nxB];
  }
}

hipError_t launch_record(const float* x, const float* u, float* rx, float* ru, int nxB, int nuB, hipStream_t s) {
  hipLaunchKernelGGL(record_kernel, dim3((nxB + nuB + 255) / 256), dim3(256), 0, s, x, u, rx, ru, nxB, nuB);
  return hipGetLastError();
}

hipError_t launch_cartpole_rollout(const SolveArgs& a, const CartpoleParams& p, hipStream_t stream) {
  const dim3 grid((a.Kp + 255) / 256, a.B);
  hipLaunchKernelGGL(cartpole_rollout_kernel, grid, dim3(256), (size_t)a.H * sizeof(float), stream, a, p);
  return hipGetLastError();
}

}  // namespace mppi
