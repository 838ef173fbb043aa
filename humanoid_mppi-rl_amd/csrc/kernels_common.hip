// Dynamics-independent MPPI kernels: device noise, softmin + weighted-noise reduce, U update/shift, trajectory
// logging (the analytic cartpole rollout: kernels_cartpole.hip).
//
// HBM layout (k fastest = "state-major", numpy's (nu,T,K) C order of src/cartpole_mppi.py:89):
//   noise [B][nu][H][Kp]   costs [B][Kp]   U/dU [B][nu][H]   x0 [B][nx]
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <algorithm>
#include "costs.h"
#include "mppi_internal.h"
#include "philox.h"
#include "wave_reduce.h"

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
    if (a.Umirror) a.Umirror[(long)b * rows + r] = v;
  }
}

// ------------------------------------------------------------------------------------------------
// a7 + a8: softmin weights and dU[b][u][t] = sum_k w_k eps[b][u][t][k] / (sum_k w_k + eps_norm).
// grid = (row chunks, B), 512 threads (1024 for LOCAL and GEN). Every block recomputes beta and sum(w) for its solve from the
// K costs (<= 128 KiB, L2-resident) and stages w in LDS; then each wave streams whole noise rows
// with 16-B loads (the HBM-bound part: each noise element is read exactly once).
// References: src/cartpole_mppi.py:92-98, src/mppi.jl:87-94, src/cartpole_mppi_estimator.py:131-143.
// ------------------------------------------------------------------------------------------------
// GEN (graph streams): the same pass also generates the NEXT solve's noise rows into `gen.next` (same rows, same
// Philox counters as noise_kernel, key = gen.seed + *seed_ctr): the VALU-bound generation hides under the
// HBM-bound stream, and the next solve needs no noise launch.  The counter advances once every block of every
// solve has read it (the last solve to finish, global ticket).

// LOCAL (B*nu large enough to fill the chip with one u-row per block): block (u, b) owns the whole row U[b][u][:],
// so update + clamp + u0 + shift are block-local: no per-solve ticket, no sc1 re-read of dU (config #4: the ticketed
// tail cost ~2.3 us of a 16.6 us reduce).
// NT: nontemporal noise loads, for batches whose noise (> 128 MB) no longer sits in L2 / the Infinity Cache after the
// rollout read it (config #4 at 64 solves: 352 MB; step 0.5017 / 0.5032 -> 0.4918 / 0.4920 ms, same box; 8 solves,
// 44 MB: no change either way -- round 2 had measured nontemporal loads 2 us slower there)
template <bool GEN, bool LOCAL, bool NT = false>
__global__ __launch_bounds__(1024) void reduce_kernel(SolveArgs a, int rows_per_block, NoiseGen gen) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* w = smem;                // [max(Kp, nu*H)]
  float* red = smem + (a.Kp > a.nu * a.H ? a.Kp : a.nu * a.H);  // [40] scratch (2 per wave + the arrival flag)
  float* du_l = red + 40;         // LOCAL: dU of the block's rows [rows_per_block]
  const int b = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, nw = blockDim.x >> 6, nt = blockDim.x;
  const float* c = a.costs + (long)b * a.Kp;
  const int rows = a.nu * a.H;
  const int r0 = blockIdx.x * rows_per_block;
  const int r1 = min(rows, r0 + rows_per_block);
  typedef float f4 __attribute__((ext_vector_type(4)));
  const int nq = a.Kp >> 2;
  // each wave streams kRR rows at once, kRU quads per lane in flight per row (kRR * kRU 16-B loads outstanding)
  constexpr int kRR = 1, kRU = 4;
  f4 e[kRR][kRU];
  auto issue = [&](int r, int q0) {
#pragma unroll
    for (int j = 0; j < kRU; ++j) {
      const int q = min(q0 + 64 * j, nq - 1);
#pragma unroll
      for (int i = 0; i < kRR; ++i) {
        // plain (cached) load while the rollout's read of this noise is still in L2 / the Infinity Cache (NT: the
        // large batches, where it is not)
        const f4* src = reinterpret_cast<const f4*>(a.noise + ((long)b * rows + min(r + i, r1 - 1)) * a.Kp) + q;
        if constexpr (NT)
          e[i][j] = __builtin_nontemporal_load(src);
        else
          e[i][j] = *src;
      }
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
      if (lane == 0 && r + i < r1) {
        if constexpr (LOCAL) du_l[r + i - r0] = sum * inv_S;
        __hip_atomic_store(a.dU + (long)b * rows + r + i, sum * inv_S, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }

  if constexpr (LOCAL) {  // a8/a9 on the block's own u-row(s) [r0, r1) (whole rows: r0 % H == 0, r1 % H == 0)
    __syncthreads();        // du_l complete, w dead
    float* su = w;
    const bool before = (a.flags & MPPI_FLAG_U0_BEFORE) != 0, shift = (a.flags & MPPI_FLAG_SHIFT) != 0;
    float* U = a.U + (long)b * rows;
    for (int r = r0 + tid; r < r1; r += nt) {
      const float old = U[r];
      float v = (a.update_mode == MPPI_UPDATE_REPLACE ? 0.0f : old) + du_l[r - r0];
      if (a.U_clamp > 0.0f) v = fminf(a.U_clamp, fmaxf(-a.U_clamp, v));
      su[r - r0] = v;
      const int u = r / a.H;
      if (r - u * a.H == 0 && a.u0) a.u0[(long)b * a.nu + u] = before ? old : v;
    }
    __syncthreads();
    for (int r = r0 + tid; r < r1; r += nt) {
      const int t = r % a.H;
      const float v = shift ? ((t < a.H - 1) ? su[r + 1 - r0] : a.shift_fill * su[r - r0]) : su[r - r0];
      U[r] = v;
      if (a.Umirror) a.Umirror[(long)b * rows + r] = v;
    }
    if (tid == 0) {
      if (blockIdx.x == 0 && b == 0 && a.seed_bump) atomicAdd(a.seed_bump, 1ull);  // noise kernel done: stream order
    }
    static_assert(!(GEN && LOCAL), "graph streams use the ticketed update");
    return;
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

constexpr bool kReduceLocal = true;

hipError_t launch_reduce(const SolveArgs& a, const NoiseGen* gen, hipStream_t stream) {
  const int rows = a.nu * a.H;
  // ~256 blocks of 8 waves in total (1 per CU), each wave streaming one row at a time with 4 16-B loads in flight
  // per lane (same-box sweep over rows x loads x block count on configs #4 and #5: 1 x 4 x 256 best by ~1 %)
  // Enough rows per block to amortise each block's softmin pass over the K costs.
  int target = 256;
  if (const char* e = std::getenv("MPPI_REDUCE_BLOCKS")) target = std::max(1, std::atoi(e));  // (A/B knob)
  int rpb = (rows * a.B + target - 1) / target;
  rpb = rpb < 1 ? 1 : rpb;
  // plain solves with enough solves x controls for one u-row per block to fill the chip: block-local update
  // (LOCAL; config #4: 16.9 -> 13.9 us).  Graph streams keep the ticketed form: their next-noise generation wants
  // the wider grid (LOCAL + GEN: step 117.8 -> 120.7 us, same box).
  const bool local = kReduceLocal && !gen && a.B * a.nu >= 128;
  if (local) rpb = a.H;
  const dim3 grid((rows + rpb - 1) / rpb, a.B);
  const size_t lds = (size_t)((a.Kp > a.nu * a.H ? a.Kp : a.nu * a.H) + 40 + (local ? rpb : 0)) * sizeof(float);
  const bool nt = (double)a.B * rows * a.Kp * 4.0 > 128.0 * 1024 * 1024;  // noise past what the caches keep
  auto kern = gen ? (nt ? reduce_kernel<true, false, true> : reduce_kernel<true, false>)
                  : (local ? (nt ? reduce_kernel<false, true, true> : reduce_kernel<false, true>)
                           : (nt ? reduce_kernel<false, false, true> : reduce_kernel<false, false>));
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds);
    if (e != hipSuccess) return e;
  }
  // 16 waves per block for LOCAL (fewer blocks: one per u-row) and for GEN (more waves for the VALU-bound
  // generation: config #5 step 53.0 -> 52.0 ms, config #4 -0.5 %, same box)
  hipLaunchKernelGGL(kern, grid, dim3(local || gen ? 1024 : 512), lds, stream, a, rpb,
                     gen ? *gen : NoiseGen{nullptr, 0, 0.0f, nullptr});
  return hipGetLastError();
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

}  // namespace mppi
