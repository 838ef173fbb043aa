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
template <bool GEN, bool LOCAL>
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
      for (int i = 0; i < kRR; ++i)
        // plain (cached) load: the rollout has just read this noise, so it is mostly still in L2 / MALL
        // (a nontemporal load here measured 2 us slower per solve on config #4)
        e[i][j] = *(reinterpret_cast<const f4*>(a.noise + ((long)b * rows + min(r + i, r1 - 1)) * a.Kp) + q);
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
  int rpb = (rows * a.B + 255) / 256;
  rpb = rpb < 1 ? 1 : rpb;
  // plain solves with enough solves x controls for one u-row per block to fill the chip: block-local update
  // (LOCAL; config #4: 16.9 -> 13.9 us).  Graph streams keep the ticketed form: their next-noise generation wants
  // the wider grid (LOCAL + GEN: step 117.8 -> 120.7 us, same box).
  const bool local = kReduceLocal && !gen && a.B * a.nu >= 128;
  if (local) rpb = a.H;
  const dim3 grid((rows + rpb - 1) / rpb, a.B);
  const size_t lds = (size_t)((a.Kp > a.nu * a.H ? a.Kp : a.nu * a.H) + 40 + (local ? rpb : 0)) * sizeof(float);
  auto kern = gen ? reduce_kernel<true, false> : (local ? reduce_kernel<false, true> : reduce_kernel<false, false>);
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
// a2-a6 for the analytic cartpole (models/cartpole.xml): one lane per sample, the H loop in
// registers, U[b] staged in LDS; writes costs[b][k]. Dynamics = oracle/mppi_ref.py::cartpole_step,
// which reproduces the recorded MuJoCo trajectory data/2025-04-21_011138 to 1.1e-16 (fp64).
// ------------------------------------------------------------------------------------------------
// The horizon is a dependent chain per sample (one lane each), so the kernel is latency-bound: the noise of the
// next 8 steps is loaded while the current 8 run (chunked register ring), the cost kind is a template parameter
// (no per-step switch) and the 2x2 solve uses the hardware reciprocal.
//
// FUSED (SolveArgs::part set: every solve but the env step).  A cartpole solve is a few thousand samples, so a
// separate reduce launch cost a third of the step (softmin prologue in every block, one noise row per block, ticket
// tail).  Each rollout block instead finishes its share of a7-a9 in the online-softmin form of
// src/cartpole_mppi.py:92-98, regrouped by block j of 256 samples:
//   m_j = min_k c_k,  S_j = sum_k exp(-(c_k - m_j)/lambda),  P_j[t] = sum_k exp(-(c_k - m_j)/lambda) eps[t][k]
// (the noise rows are L2-hot from the rollout: one 16-B load per lane per row), published with sc1 stores; the last
// block of the solve (sc1 ticket, as reduce_kernel) forms beta = min_j m_j, f_j = exp(-(m_j - beta)/lambda) and
// dU = sum_j f_j P_j / (sum_j f_j S_j + eps_norm) in block order (deterministic), the weights if requested, and
// applies the update + shift.  The non-finite flag is sticky (set by the kernel, cleared by the host that reads
// it).  GEN (graph streams): blocks past the rollout blocks generate the next solve's noise (noise_kernel's
// Philox counters) on CUs the Kp/256-block rollout leaves idle; the seed counter advances behind a global ticket.

// GEN blocks of a fused launch: the next solve's noise rows of solve b (counters (k/4, t, u = 0, b)), then the seed
// counter advances once every generator block of every solve has used the key.
__device__ void cartpole_generate(const SolveArgs& a, const NoiseGen& gen, int b, int gi, int ng, const KClock& kc) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  const uint64_t key = gen.seed + *a.seed_ctr;
  const uint32_t k0 = (uint32_t)key, k1 = (uint32_t)(key >> 32);
  const int nq = a.Kp >> 2;
  for (int i = gi * blockDim.x + threadIdx.x; i < a.H * nq; i += ng * blockDim.x) {
    const int t = i / nq, q = i - t * nq;
    float z[4];
    philox_normal4((uint32_t)q, (uint32_t)t, 0u, (uint32_t)b, k0, k1, z);
    __builtin_nontemporal_store(f4{gen.sigma * z[0], gen.sigma * z[1], gen.sigma * z[2], gen.sigma * z[3]},
                                reinterpret_cast<f4*>(gen.next + ((long)b * a.H + t) * a.Kp) + q);
  }
  __syncthreads();  // every thread of the block has used the key
  kclock_record(a, kc);
  if (threadIdx.x == 0 && __hip_atomic_fetch_add(gen.gticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                              (unsigned)(ng * gridDim.y) - 1) {
    __hip_atomic_store(gen.gticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    atomicAdd(a.seed_ctr, 1ull);
  }
}

// Fused a7-a9 of rollout block blockIdx.x of solve b (thread = sample k, cost cst, +inf if not finite).
// sc: LDS scratch, 16-B aligned, kFinishScratch(H) floats.
__host__ __device__ constexpr int kFinishScratch(int H) { return 256 + 16 + (H > 4096 ? H : 4096); }

__device__ void cartpole_finish(const SolveArgs& a, int b, int k, float cst, float* sc, int nblk, const KClock& kc) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int H = a.H, rl = 2 + H;  // partial record: m_j, S_j, P_j[H]
  float* sw = sc;         // [256] this block's weights; in the last block the combine factors / block sums
  float* red = sc + 256;  // [16]
  float* tr = sc + 272;   // [4 waves][16 rows][64 lanes] transpose tiles; in the last block the new U row
  const float inv_lam = 1.0f / a.lambda;
  // this wave's first pass of noise rows (L2-hot from the rollout) is issued before the softmin barriers, so its
  // latency hides behind them
  const int rq = a.Kp >> 2;
  const f4* e4 = reinterpret_cast<const f4*>(a.noise + (long)b * H * a.Kp) + min((int)blockIdx.x * 64 + lane, rq - 1);
  f4 e[16];
  auto load_rows = [&](int t0) {
#pragma unroll
    for (int i = 0; i < 16; ++i) e[i] = e4[(long)min(t0 + i, H - 1) * rq];
  };
  if (16 * wv < H) load_rows(16 * wv);
  const bool ok = k < a.K && cst < INFINITY;
  const float m = wave_min(ok ? cst : INFINITY);
  if (lane == 0) red[wv] = m;
  __syncthreads();
  const float mb = fminf(fminf(red[0], red[1]), fminf(red[2], red[3]));
  const float w = (ok && mb < INFINITY) ? __expf(-inv_lam * (cst - mb)) : 0.0f;
  sw[tid] = w;
  const float s = wave_sum(w);
  if (lane == 0) red[4 + wv] = s;
  __syncthreads();
  float* rec = a.part + ((long)b * nblk + blockIdx.x) * rl;
  // P_j[t]: lane l holds samples 4l..4l+3 of the block (lanes past Kp carry w = 0).  Each wave takes 16 rows per
  // pass (16 loads in flight per lane), then reduces them across its 64 lanes through an LDS transpose: lane l sums
  // quarter l&3 of row l>>2 (16 partials), two shuffles finish the row.
  const f4 w4 = reinterpret_cast<const f4*>(sw)[lane];
  float* trw = tr + wv * 1024;
  for (int t0 = 16 * wv; t0 < H; t0 += 64) {
    if (t0 != 16 * wv) load_rows(t0);  // the first pass is already in flight
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      float q = e[i].x * w4.x;
      q = fmaf(e[i].y, w4.y, q);
      q = fmaf(e[i].z, w4.z, q);
      q = fmaf(e[i].w, w4.w, q);
      trw[i * 64 + lane] = q;
    }
    const f4* rowq = reinterpret_cast<const f4*>(trw + (lane >> 2) * 64 + (lane & 3) * 16);
    const f4 x0 = rowq[0], x1 = rowq[1], x2 = rowq[2], x3 = rowq[3];
    float q = ((x0.x + x0.y) + (x0.z + x0.w)) + ((x1.x + x1.y) + (x1.z + x1.w)) + ((x2.x + x2.y) + (x2.z + x2.w)) +
              ((x3.x + x3.y) + (x3.z + x3.w));
    q += __shfl_xor(q, 1);
    q += __shfl_xor(q, 2);
    const int t = t0 + (lane >> 2);
    if ((lane & 3) == 0 && t < H) __hip_atomic_store(rec + 2 + t, q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (tid == 0) {
    __hip_atomic_store(rec, mb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(rec + 1, (red[4] + red[5]) + (red[6] + red[7]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // ticket (reduce_kernel's form): sc1 payload stores drained by every storing wave, barrier, one relaxed ticket
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  unsigned* last = reinterpret_cast<unsigned*>(red + 8);
  if (tid == 0)
    *last = __hip_atomic_fetch_add(a.tickets + b, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)nblk - 1
                ? 1u
                : 0u;
  __syncthreads();
  if (!*last) {
    kclock_record(a, kc);
    return;
  }
  // ---- the last block of solve b: combine the nblk records in block order (sc1 loads) and update U in place.
  // When they fit the scratch (config #2: 16 records of 52 floats), all records and the old U row come in ONE round
  // of loads into LDS (8 per thread in flight): the combine otherwise paid a memory round trip for the record
  // heads and another for the rows (3.4 us of the 14 us launch went to this block)
  auto ld = [](const float* q) { return __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
  const float* pb = a.part + (long)b * nblk * rl;
  float* fm = sw;        // [nblk <= 128] block minima, then the combine factors f_j
  float* fs = sw + 128;  // [nblk] block weight sums
  float* U = a.U + (long)b * H;
  if (tid == 0) __hip_atomic_store(a.tickets + b, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int nrec = nblk * rl, hp = (H + 3) & ~3;
  float* rs = tr + hp;  // LDS copy of the records (fast path)
  constexpr int kRecLd = 8;
  const bool fast = nrec <= 4096 - hp && nrec <= kRecLd * 256 && (int)blockDim.x == 256;
  const float old0 = U[min(tid, H - 1)];  // this thread's first U element (in flight with the records)
  float beta = INFINITY, S = 0.0f;
  if (fast) {
    float v[kRecLd];
#pragma unroll
    for (int i = 0; i < kRecLd; ++i) v[i] = ld(pb + min(tid + 256 * i, nrec - 1));  // unconditional: one round
#pragma unroll
    for (int i = 0; i < kRecLd; ++i)
      if (tid + 256 * i < nrec) rs[tid + 256 * i] = v[i];
    __syncthreads();
    // beta and S by every wave over the records by lane (fixed-order wave reductions: no serial LDS chain)
    float mloc = INFINITY;
    for (int j = lane; j < nblk; j += 64) mloc = fminf(mloc, rs[j * rl]);
    beta = wave_min(mloc);
    float sloc = 0.0f;
    for (int j = lane; j < nblk; j += 64) {
      const float mj = rs[j * rl];
      const float f = mj < INFINITY ? __expf(-inv_lam * (mj - beta)) : 0.0f;
      sloc = fmaf(f, rs[j * rl + 1], sloc);
      if (wv == 0) fm[j] = f;
    }
    S = wave_sum(sloc);
    __syncthreads();  // fm
  } else {
    for (int j = tid; j < nblk; j += blockDim.x) {
      fm[j] = ld(pb + (long)j * rl);
      fs[j] = ld(pb + (long)j * rl + 1);
    }
    __syncthreads();
    for (int j = 0; j < nblk; ++j) beta = fminf(beta, fm[j]);
    for (int j = 0; j < nblk; ++j) S = fmaf(fm[j] < INFINITY ? __expf(-inv_lam * (fm[j] - beta)) : 0.0f, fs[j], S);
    __syncthreads();  // every thread has read fm
    for (int j = tid; j < nblk; j += blockDim.x) fm[j] = fm[j] < INFINITY ? __expf(-inv_lam * (fm[j] - beta)) : 0.0f;
    __syncthreads();
  }
  const float inv_S = 1.0f / (S + a.norm_eps);
  // update (add / replace, clamp), u0 and shift, as update_solve (nu = 1), from the combined rows
  float* su = tr;  // [H]
  const bool before = (a.flags & MPPI_FLAG_U0_BEFORE) != 0;
  for (int t = tid; t < H; t += blockDim.x) {
    const float old = t == tid ? old0 : U[t];
    float acc = 0.0f;
    if (fast) {
      for (int j0 = 0; j0 < nblk; j0 += 16) {  // 16 LDS reads in flight, then the fmas in block order
        float f[16], v[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int j = min(j0 + i, nblk - 1);
          f[i] = fm[j];
          v[i] = rs[j * rl + 2 + t];
        }
#pragma unroll
        for (int i = 0; i < 16; ++i)
          if (j0 + i < nblk) acc = fmaf(f[i], v[i], acc);
      }
    } else {
      for (int j0 = 0; j0 < nblk; j0 += 16) {  // 16 loads in flight
        float v[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] = ld(pb + (long)min(j0 + i, nblk - 1) * rl + 2 + t);
#pragma unroll
        for (int i = 0; i < 16; ++i)
          if (j0 + i < nblk) acc = fmaf(fm[j0 + i], v[i], acc);
      }
    }
    const float d = acc * inv_S;
    a.dU[(long)b * H + t] = d;
    float nv = (a.update_mode == MPPI_UPDATE_REPLACE ? 0.0f : old) + d;
    if (a.U_clamp > 0.0f) nv = fminf(a.U_clamp, fmaxf(-a.U_clamp, nv));
    su[t] = nv;
    if (t == 0 && a.u0) a.u0[b] = before ? old : nv;
  }
  if (a.weights)  // costs were published with sc1 stores by every block
    for (int kk = tid; kk < a.Kp; kk += blockDim.x) {
      const float c = kk < a.K ? ld(a.costs + (long)b * a.Kp + kk) : INFINITY;
      a.weights[(long)b * a.Kp + kk] = (c < INFINITY && beta < INFINITY) ? __expf(-inv_lam * (c - beta)) * inv_S : 0.0f;
    }
  __syncthreads();
  const bool shift = (a.flags & MPPI_FLAG_SHIFT) != 0;
  for (int t = tid; t < H; t += blockDim.x) {
    const float v = shift ? (t < H - 1 ? su[t + 1] : a.shift_fill * su[t]) : su[t];
    U[t] = v;
    if (a.Umirror) a.Umirror[(long)b * H + t] = v;
  }
  if (a.kclock) {  // (uniform) the block's end: every thread's last store issued; the stamp reads the counter
    __syncthreads();   // before the seed bump below
    kclock_record(a, kc);
  }
  if (tid == 0) {
    if (b == 0 && a.seed_bump) atomicAdd(a.seed_bump, 1ull);  // plain solves: the next solve's noise key
    // sticky non-finite flag: set here, cleared by the host when it reads it (mppi_api.hip::read_status)
    if (!(beta < INFINITY)) atomicOr(a.status, 1u);
  }
}

template <int COST, bool FUSED>
__global__ __launch_bounds__(256) void cartpole_rollout_kernel(SolveArgs a, CartpoleParams p, NoiseGen gen, int nroll) {
  extern __shared__ __attribute__((aligned(16))) float sU[];  // [H, padded to 4]; FUSED: + kFinishScratch(H)
  const int b = blockIdx.y;
  const KClock kclk = kclock_begin(a);
  if constexpr (FUSED) {
    if ((int)blockIdx.x >= nroll) {  // generator block (GEN)
      cartpole_generate(a, gen, b, (int)blockIdx.x - nroll, (int)gridDim.x - nroll, kclk);
      return;
    }
  }
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (!FUSED && k == 0 && b == 0) *a.status = 0u;  // per-solve status word (OR-ed by the reduce)
  const int kc = k < a.Kp ? k : a.Kp - 1;  // FUSED: lanes past Kp run a clamped copy and reach every barrier
  const float* e = a.noise + (long)b * a.H * a.Kp + kc;
  constexpr int kC = 8;  // steps per chunk
  float en[kC], un[kC];  // the next chunk's noise (global) and U (LDS), loaded a chunk ahead
  auto load_noise = [&](int t0) {
#pragma unroll
    for (int j = 0; j < kC; ++j) en[j] = e[(long)min(t0 + j, a.H - 1) * a.Kp];
  };
  auto load_u = [&](int t0) {
#pragma unroll
    for (int j = 0; j < kC; ++j) un[j] = sU[min(t0 + j, a.H - 1)];
  };
  // the first chunk's noise and x0 are in flight while U is staged
  load_noise(0);
  const float* xb = a.x0 + (long)b * a.nx;
  float pos = xb[0], th = xb[1], xd = xb[2], thd = xb[3];
  for (int t = threadIdx.x; t < a.H; t += blockDim.x) sU[t] = a.U[(long)b * a.H + t];  // nu == 1
  __syncthreads();
  if (!FUSED && k >= a.Kp) return;
  load_u(0);
  const float dt = p.dt, D = p.damping, mp = p.m_pole, l = p.l;
  const float m11 = p.m_cart + mp + dt * D;
  const float m22 = mp * l * l + p.inertia + dt * D;
  const float mpl = mp * l;
  // the running cost as per-term sums (the cartpole costs take no per-solve context): x^2, the angle term, xd^2 +
  // thd^2 and u^2 accumulate separately and are weighted once after the horizon (6 VALU per step instead of 11;
  // src/cartpole_mppi.py:44-50 / src/cartpole_mppi_estimator.py:46-52 up to fp32 summation order)
  float sx = 0.0f, sc = 0.0f, sv = 0.0f, su = 0.0f;
  // sin/cos of the current angle, carried from step to step: the running cost of step t reads cos(theta_{t+1}),
  // which is also what step t+1's dynamics need (one sincos per step)
  float sn, cs;
  sincos_fast(th, &sn, &cs);
  const float cl = a.ctrl_clamp > 0.0f ? a.ctrl_clamp : INFINITY;  // clamp as one v_med3 (+-inf: none)
  auto step = [&](float u) {
    u = __builtin_amdgcn_fmed3f(u, -cl, cl);
    const float F = p.gear * __builtin_amdgcn_fmed3f(u, p.ctrl_lo, p.ctrl_hi);
    const float m12 = mpl * cs;
    const float f1 = F + mpl * sn * thd * thd - D * xd;
    const float f2 = mpl * p.g * sn - D * thd;
    const float inv_det = __builtin_amdgcn_rcpf(m11 * m22 - m12 * m12);
    const float a1 = (m22 * f1 - m12 * f2) * inv_det;
    const float a2 = (m11 * f2 - m12 * f1) * inv_det;
    xd = xd + dt * a1;
    thd = thd + dt * a2;
    pos = pos + dt * xd;
    th = th + dt * thd;
    sincos_fast(th, &sn, &cs);
    sx = fmaf(pos, pos, sx);
    const float c1 = cs - 1.0f;
    if constexpr (COST == MPPI_COST_CARTPOLE) {
      sc = fmaf(c1, c1, sc);
      su = fmaf(u, u, su);
    } else {
      sc += fabsf(c1);
    }
    sv = fmaf(xd, xd, sv);
    sv = fmaf(thd, thd, sv);
  };
  // whole chunks carry no per-step branch, and their U values come from LDS a chunk ahead like the noise: with a
  // break test per step, each step's U read and its lgkmcnt wait sat inside the dependent chain, and in-order
  // issue stalled the whole step on it.  The ragged tail chunk keeps the per-step test.
  int t0 = 0;
  for (; t0 + kC <= a.H; t0 += kC) {
    float uc[kC];
#pragma unroll
    for (int j = 0; j < kC; ++j) uc[j] = un[j] + en[j];
    if (t0 + kC < a.H) {
      load_noise(t0 + kC);
      load_u(t0 + kC);
    }
#pragma unroll
    for (int j = 0; j < kC; ++j) step(uc[j]);
  }
  if (t0 < a.H) {
#pragma unroll
    for (int j = 0; j < kC; ++j) {
      if (t0 + j >= a.H) break;
      step(un[j] + en[j]);
    }
  }
  float cost = COST == MPPI_COST_CARTPOLE ? sx + 20.0f * sc + 0.1f * sv + 0.01f * su : sx + 50.0f * sc + 0.1f * sv;
  if (a.terminal_weight != 0.0f) cost += a.terminal_weight * cartpole_cost_c<COST>(pos, cs, xd, thd, 0.0f);
  const float cst = isfinite(cost) ? cost : INFINITY;
  if (k < a.K) {
    if constexpr (FUSED)  // read back by the solve's last block, possibly on another XCD: write-through
      __hip_atomic_store(a.costs + (long)b * a.Kp + k, cst, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else
      a.costs[(long)b * a.Kp + k] = cst;
  }
  if (a.xout && k == 0) {
    float* xo = a.xout + (long)b * a.nx;
    xo[0] = pos;
    xo[1] = th;
    xo[2] = xd;
    xo[3] = thd;
  }
  if constexpr (FUSED) cartpole_finish(a, b, k, cst, sU + ((a.H + 3) & ~3), nroll, kclk);
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

hipError_t launch_cartpole_rollout(const SolveArgs& a, const CartpoleParams& p, const NoiseGen* gen, hipStream_t stream) {
  const bool fused = a.part != nullptr;
  const int nroll = (a.Kp + 255) / 256;
  // GEN: generator blocks beside the rollout blocks, about 4 noise quads per thread
  const int ngen = (fused && gen && gen->next) ? (a.H * (a.Kp / 4) + 1023) / 1024 : 0;
  const NoiseGen g = ngen ? *gen : NoiseGen{nullptr, 0, 0.0f, nullptr};
  const dim3 grid(nroll + ngen, a.B);
  const size_t lds = (size_t)(((a.H + 3) & ~3) + (fused ? kFinishScratch(a.H) : 0)) * sizeof(float);
  auto go = [&](auto kern) -> hipError_t {
    if (lds > 64 * 1024) {
      const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(kern, grid, dim3(256), lds, stream, a, p, g, nroll);
    return hipGetLastError();
  };
  switch (a.cost_kind) {
    case MPPI_COST_CARTPOLE:
      return fused ? go(cartpole_rollout_kernel<MPPI_COST_CARTPOLE, true>)
                   : go(cartpole_rollout_kernel<MPPI_COST_CARTPOLE, false>);
    case MPPI_COST_CARTPOLE_EST:
      return fused ? go(cartpole_rollout_kernel<MPPI_COST_CARTPOLE_EST, true>)
                   : go(cartpole_rollout_kernel<MPPI_COST_CARTPOLE_EST, false>);
    default: return hipErrorInvalidValue;  // the analytic cartpole carries a cartpole cost (mppi_set_cost checks)
  }
}

}  // namespace mppi
