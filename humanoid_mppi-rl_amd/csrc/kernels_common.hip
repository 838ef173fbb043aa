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
// a1: eps[b][u][t][k] = sigma * N(0,1) (Philox4x32-10, counter (k/4, t, u, b)); one thread = 4 consecutive k of one
// (b, u, t) row, one 16-B nontemporal store.  grid = (Kp/4/256 chunks, rows): no 64-bit div/mod per element.
// The kernel depends on nothing but the seed, so a captured stream of solves generates solve i+1's noise
// concurrently with solve i's rollout (mppi_api.hip, double-buffered).
// seed_ctr (MPPI_FLAG_SEED_COUNTER): key = seed + *seed_ctr.  The counter advances once per solve: in the reduce's
// last block for a plain solve, in bump_kernel right behind a graph's prefetched noise (mppi_api.hip).
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void noise_kernel(float* __restrict__ noise, int rows, int nu, int H, int Kp,
                                                    uint64_t seed, const unsigned long long* seed_ctr, float sigma) {
  const int row = blockIdx.z * 65535 + blockIdx.y;  // (b*nu + u)*H + t
  const int kq = blockIdx.x * 256 + threadIdx.x;
  const uint64_t key = seed + (seed_ctr ? *seed_ctr : 0ull);
  if (row < rows && 4 * kq < Kp) {
    const uint32_t k0 = (uint32_t)key, k1 = (uint32_t)(key >> 32);
    const int t = row % H;
    const int bu = row / H;
    const int u = bu % nu;
    const int b = bu / nu;
    float z[4];
    philox_normal4((uint32_t)kq, (uint32_t)t, (uint32_t)u, (uint32_t)b, k0, k1, z);
    typedef float f4 __attribute__((ext_vector_type(4)));
    f4 v = {sigma * z[0], sigma * z[1], sigma * z[2], sigma * z[3]};
    __builtin_nontemporal_store(v, reinterpret_cast<f4*>(noise + (long)row * Kp) + kq);
  }
}

__global__ void bump_kernel(unsigned long long* seed_ctr, long long delta) { *seed_ctr += (unsigned long long)delta; }

hipError_t launch_noise(float* noise, int B, int nu, int H, int Kp, uint64_t seed, const unsigned long long* seed_ctr,
                        float sigma, hipStream_t stream) {
  const int rows = B * nu * H;
  const dim3 grid((Kp / 4 + 255) / 256, rows < 65535 ? rows : 65535, (rows + 65534) / 65535);
  hipLaunchKernelGGL(noise_kernel, grid, dim3(256), 0, stream, noise, rows, nu, H, Kp, seed, seed_ctr, sigma);
  return hipGetLastError();
}

hipError_t launch_seed_bump(unsigned long long* seed_ctr, long long delta, hipStream_t stream) {
  hipLaunchKernelGGL(bump_kernel, dim3(1), dim3(1), 0, stream, seed_ctr, delta);
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
// GEN (graph streams): the same pass also generates the NEXT solve's noise rows into `gen.next` (same rows, same
// Philox counters as noise_kernel, key = gen.seed + *seed_ctr): the VALU-bound generation hides under the
// HBM-bound stream, and the next solve needs no noise launch.  The counter advances once every block of every
// solve has read it (the last solve to finish, global ticket).

template <bool GEN>
__global__ __launch_bounds__(512) void reduce_kernel(SolveArgs a, int rows_per_block, NoiseGen gen) {
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
  uint32_t gk0 = 0, gk1 = 0;
  if constexpr (GEN) {
    const uint64_t key = gen.seed + *a.seed_ctr;
    gk0 = (uint32_t)key;
    gk1 = (uint32_t)(key >> 32);
  }
  // next solve's noise for the tile (rows r, r+1; quads q0 + 64 j)
  auto generate = [&](int r, int q0) {
#pragma unroll
    for (int i = 0; i < kRR; ++i) {
      const int row = r + i;
      if (row >= r1) continue;
      const int u = row / a.H, t = row - u * a.H;
      f4* dst = reinterpret_cast<f4*>(gen.next + ((long)b * rows + row) * a.Kp);
#pragma unroll
      for (int j = 0; j < kRU; ++j) {
        const int q = q0 + 64 * j;
        if (q >= nq) continue;
        float z[4];
        philox_normal4((uint32_t)q, (uint32_t)t, (uint32_t)u, (uint32_t)b, gk0, gk1, z);
        __builtin_nontemporal_store(f4{gen.sigma * z[0], gen.sigma * z[1], gen.sigma * z[2], gen.sigma * z[3]},
                                    dst + q);
      }
    }
  };

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
      if constexpr (GEN) generate(r, q0);  // VALU work while the tile's loads are in flight
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
    // next solve's noise key (plain solves; this solve's noise kernel has completed: stream order)
    if (b == 0 && a.seed_bump) atomicAdd(a.seed_bump, 1ull);
    if constexpr (GEN) {  // every block of every solve has read the counter: advance it once
      if (__hip_atomic_fetch_add(gen.gticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.y - 1) {
        __hip_atomic_store(gen.gticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        atomicAdd(a.seed_ctr, 1ull);
      }
    }
  }
}

hipError_t launch_reduce(const SolveArgs& a, const NoiseGen* gen, hipStream_t stream) {
  const int rows = a.nu * a.H;
  // ~512 blocks of 8 waves in total (2 per CU), each wave streaming up to 2 rows with 8 16-B loads in flight
  // per lane; enough rows per block to amortise each block's softmin pass over the K costs.
  int rpb = (rows * a.B + 511) / 512;
  rpb = rpb < 1 ? 1 : rpb;
  const dim3 grid((rows + rpb - 1) / rpb, a.B);
  const size_t lds = (size_t)((a.Kp > a.nu * a.H ? a.Kp : a.nu * a.H) + 32) * sizeof(float);
  auto kern = gen ? reduce_kernel<true> : reduce_kernel<false>;
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(kern, grid, dim3(512), lds, stream, a, rpb, gen ? *gen : NoiseGen{nullptr, 0, 0.0f, nullptr});
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// a2-a6 for the analytic cartpole (models/cartpole.xml): one lane per sample, the H loop in
// registers, U[b] staged in LDS; writes costs[b][k]. Dynamics = oracle/mppi_ref.py::cartpole_step,
// which reproduces the recorded MuJoCo trajectory data/2025-04-21_011138 to 1.1e-16 (fp64).
// ------------------------------------------------------------------------------------------------
// The horizon is a dependent chain per sample (one lane each), so the kernel is latency-bound: the noise of the
// next 8 steps is loaded while the current 8 run (chunked register ring), the cost kind is a template parameter
// (no per-step switch) and the 2x2 solve uses the hardware reciprocal.
template <int COST>
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
  float v[4] = {pos, th, xd, thd};
  constexpr int kC = 8;  // steps per chunk
  float en[kC];
  auto load_chunk = [&](int t0) {
#pragma unroll
    for (int j = 0; j < kC; ++j) en[j] = e[(long)min(t0 + j, a.H - 1) * a.Kp];
  };
  load_chunk(0);
  for (int t0 = 0; t0 < a.H; t0 += kC) {
    float ec[kC];
#pragma unroll
    for (int j = 0; j < kC; ++j) ec[j] = en[j];
    if (t0 + kC < a.H) load_chunk(t0 + kC);
#pragma unroll
    for (int j = 0; j < kC; ++j) {
      const int t = t0 + j;
      if (t >= a.H) break;
      float u = sU[t] + ec[j];
      if (a.ctrl_clamp > 0.0f) u = fminf(a.ctrl_clamp, fmaxf(-a.ctrl_clamp, u));
      const float F = p.gear * fminf(p.ctrl_hi, fmaxf(p.ctrl_lo, u));
      float s, c;
      sincosf(th, &s, &c);
      const float m12 = mpl * c;
      const float f1 = F + mpl * s * thd * thd - D * xd;
      const float f2 = mpl * p.g * s - D * thd;
      const float inv_det = __builtin_amdgcn_rcpf(m11 * m22 - m12 * m12);
      const float a1 = (m22 * f1 - m12 * f2) * inv_det;
      const float a2 = (m11 * f2 - m12 * f1) * inv_det;
      xd = xd + dt * a1;
      thd = thd + dt * a2;
      pos = pos + dt * xd;
      th = th + dt * thd;
      v[0] = pos; v[1] = th; v[2] = xd; v[3] = thd;
      cost += cost_eval_t<COST>(v, u, u * u, ctx);
    }
  }
  if (a.terminal_weight != 0.0f) cost += a.terminal_weight * cost_eval_t<COST>(v, 0.0f, 0.0f, ctx);
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
  const size_t lds = (size_t)a.H * sizeof(float);
  switch (a.cost_kind) {
    case MPPI_COST_CARTPOLE:
      hipLaunchKernelGGL(cartpole_rollout_kernel<MPPI_COST_CARTPOLE>, grid, dim3(256), lds, stream, a, p);
      break;
    case MPPI_COST_CARTPOLE_EST:
      hipLaunchKernelGGL(cartpole_rollout_kernel<MPPI_COST_CARTPOLE_EST>, grid, dim3(256), lds, stream, a, p);
      break;
    default: return hipErrorInvalidValue;  // the analytic cartpole carries a cartpole cost (mppi_set_cost checks)
  }
  return hipGetLastError();
}

}  // namespace mppi
