// The analytic cartpole rollout with its fused a7-a9 epilogue (config #2), in its own translation unit so it takes
// its own codegen flags (build.py PER_FILE_FLAGS: the iterative-ILP machine scheduler interleaves the chunk's steps
// better on this dependent chain; the reduce and noise kernels keep the default).
#include <hip/hip_runtime.h>

#include "costs.h"
#include "mppi_internal.h"
#include "philox.h"
#include "wave_reduce.h"

namespace mppi {

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


hipError_t launch_cartpole_rollout(const SolveArgs& a, const CartpoleParams& p, const NoiseGen* gen, hipStream_t stream) {
  const bool fused = a.part != nullptr;
  const int nroll = (a.Kp + 255) / 256;
  // GEN: generator blocks beside the rollout blocks, about 4 noise quads per thread
  const int ngen = (fused && gen && gen->next) ? (a.H * (a.Kp / 4) + 1023) / 1024 : 0;
  const NoiseGen g = ngen ? *gen : NoiseGen{nullptr, 0, 0.0f, nullptr};
  const dim3 grid(nroll + ngen, a.B);
  note_kernel("cartpole_rollout_kernel");
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
