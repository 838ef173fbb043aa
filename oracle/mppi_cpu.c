/* oracle/mppi_cpu.c — TEST INFRASTRUCTURE / CPU BASELINE ONLY (never linked into the product).
 *
 * A plain-C, OpenMP restatement of the reference's MPPI solve (sample -> rollout -> cost -> softmin -> reduce ->
 * update), the compiled multi-core counterpart of the numpy oracle (oracle/mppi_ref.py, oracle/nets_ref.py).
 * It plays the part of the reference's threaded CPU path, Julia's `Threads.@threads for k in 1:K`
 * (src/Humanoid_mppi_v3.jl:131), so bench.py can time a fair multi-core CPU baseline on the GPU box's host cores
 * (CPU baseline (ii)).  The tests check it against the numpy oracle (tests/test_oracle_c.py).
 *
 * Two solves:
 *   mppi_cpu_cartpole_solve  fp64, the analytic mj_step of models/cartpole.xml (oracle/mppi_ref.py:cartpole_step)
 *                            with the running cost of src/cartpole_mppi.py:44-50 and the terminal cost of :52-53;
 *   mppi_cpu_fc_solve        fp32, x_{t+1} = x_t + net([x_t, u_t]) for an fc stack (Linear [+ LayerNorm] [+ ReLU]
 *                            per layer: learning/model.py:6-46 MLP, or the exactly folded CrossAttention net of
 *                            oracle/nets_ref.py:ca_fold) — the loop of src/cartpole_mppi_estimator.py:61-143 —
 *                            with the costs of src/Humanoid_mppi_v3.jl:27-105, src/mppi.jl:18-62,
 *                            src/quadruped_mppi_estimator.py:48-52, src/cartpole_mppi_estimator.py:46-52.
 * Softmin and update follow src/cartpole_mppi.py:92-98 (+1e-10 of src/mppi.jl:89 via norm_eps; clamps of
 * src/mppi.jl:73-74,93; replace-mode of src/cartpole_mppi_estimator.py:141-143).  No shift: the caller shifts.
 *
 * Samples are processed in blocks of 16 per thread with feature-major activations ([feature][16]) so the inner
 * loop of every Linear is two 8-wide vector FMAs (GNU vector extension, AVX2).  Build: oracle/cpu.py:build().
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

#define BLK 16
#define MAXL 8

enum { COST_CARTPOLE = 1, COST_CARTPOLE_EST = 2, COST_HUMANOID_V3 = 3, COST_QUAD_JL = 4, COST_QUAD_EST = 5 };

typedef struct {
  int nl;                /* layers */
  int dims[MAXL + 1];    /* dims[0] = nx + nu, dims[nl] >= nx (first nx outputs are the state delta) */
  const float* W[MAXL];  /* [dims[l+1]][dims[l]] row-major */
  const float* b[MAXL];  /* [dims[l+1]] */
  const float* lng[MAXL]; /* NULL or LayerNorm gamma [dims[l+1]] (eps 1e-5) */
  const float* lnb[MAXL]; /* LayerNorm beta */
  int relu[MAXL];
} mppi_cpu_net;

/* ------------------------------------------------------------------------------------------------ costs */

/* running cost of one sample: x = [qpos, qvel], u = the control used this step (NULL / usq = 0 for the terminal
 * term), ctx = per-solve context row (oracle/mppi_ref.py:humanoid_context) */
static float run_cost(int kind, const float* x, float u0, float usq, const float* ctx) {
  switch (kind) {
    case COST_CARTPOLE: { /* src/cartpole_mppi.py:44-50 */
      const float c = cosf(x[1]) - 1.0f;
      return x[0] * x[0] + 20.0f * c * c + 0.1f * x[2] * x[2] + 0.1f * x[3] * x[3] + 0.01f * u0 * u0;
    }
    case COST_CARTPOLE_EST: /* src/cartpole_mppi_estimator.py:46-52 */
      return x[0] * x[0] + 50.0f * fabsf(cosf(x[1]) - 1.0f) + 0.1f * x[2] * x[2] + 0.1f * x[3] * x[3];
    case COST_HUMANOID_V3: { /* src/Humanoid_mppi_v3.jl:27-105 */
      const float px = x[0], py = x[1], pz = x[2], q0 = x[3], q1 = x[4], q2 = x[5], q3 = x[6];
      const float roll = atan2f(2.0f * (q0 * q1 + q2 * q3), 1.0f - 2.0f * (q1 * q1 + q2 * q2));
      float sp = 2.0f * (q0 * q2 - q3 * q1);
      sp = sp > 1.0f ? 1.0f : (sp < -1.0f ? -1.0f : sp);
      const float pitch = asinf(sp);
      const float yaw = atan2f(2.0f * (q0 * q3 + q1 * q2), 1.0f - 2.0f * (q2 * q2 + q3 * q3));
      float c = 5.0f * (roll * roll + pitch * pitch) + 0.075f * yaw * yaw;
      c += 12.5f * hypotf(px - ctx[0], py - ctx[1]);
      c += 5.0f * fabsf(ctx[2] - pz);
      c += hypotf(x[28] - 0.3f, x[29]);
      const float ftx = px + 0.5f;
      c += 8.0f * fabsf(ctx[3] - ftx);
      c += 3.0f * (ctx[4] - ftx) * (ctx[4] - ftx) + ctx[5];
      return c + 0.01f * usq;
    }
    case COST_QUAD_JL: { /* src/mppi.jl:18-62 (nq = 19) */
      const int nq = 19;
      const float h = x[2] - 0.45f, vx = x[nq] - 0.6f;
      return 500.0f * h * h + 1000.0f * vx * vx + 500.0f * (x[6] * x[6] + x[7] * x[7]) +
             20.0f * (x[nq + 6] * x[nq + 6] + x[nq + 7] * x[nq + 7] + x[nq + 8] * x[nq + 8]) +
             1000.0f * (x[1] * x[1] + x[nq + 1] * x[nq + 1]) + 0.1f * usq;
    }
    case COST_QUAD_EST: { /* src/quadruped_mppi_estimator.py:48-52 */
      const float a = x[0] - ctx[0], b = x[1] - ctx[1], c = x[2] - ctx[2];
      return a * a + b * b + c * c + 0.1f * usq;
    }
    default:
      return NAN;
  }
}

/* ------------------------------------------------------------------------------------------------ softmin/update */

/* w = exp(-(c - min c)/lam) / (sum + eps), non-finite costs weight 0 (oracle/mppi_ref.py:softmin_weights);
 * dU[r] = sum_k w_k eps[r][k] over the nrow = nu*H rows; U = U + dU (or dU), clamped.  Returns 0, or -4 if no
 * cost is finite. */
static int softmin_update(int K, int nrow, const float* costs, const float* noise, float lam, float norm_eps,
                          int replace, float U_clamp, float* U, float* w_out, int nth) {
  double beta = INFINITY;
  for (int k = 0; k < K; ++k)
    if (isfinite(costs[k]) && costs[k] < beta) beta = costs[k];
  if (!isfinite(beta)) return -4;
  double* w = (double*)malloc(sizeof(double) * K);
  double S = 0.0;
  for (int k = 0; k < K; ++k) {
    w[k] = isfinite(costs[k]) ? exp(-(costs[k] - beta) / lam) : 0.0;
    S += w[k];
  }
  const double inv = 1.0 / (S + norm_eps);
  for (int k = 0; k < K; ++k) {
    w[k] *= inv;
    if (w_out) w_out[k] = (float)w[k];
  }
#pragma omp parallel for num_threads(nth) schedule(static)
  for (int r = 0; r < nrow; ++r) {
    const float* e = noise + (size_t)r * K;
    double acc = 0.0;
    for (int k = 0; k < K; ++k) acc += w[k] * e[k];
    float u = replace ? (float)acc : U[r] + (float)acc;
    if (U_clamp > 0.0f) u = u > U_clamp ? U_clamp : (u < -U_clamp ? -U_clamp : u);
    U[r] = u;
  }
  free(w);
  return 0;
}

/* ------------------------------------------------------------------------------------------------ fc rollout */

/* GNU vector extension: 8 fp32 lanes (one AVX2 register); a block of BLK = 16 samples is two of them */
typedef float v8f __attribute__((vector_size(32)));

/* h[o][:] = b[o] + sum_i W[o][i] a[i][:] for one 16-sample block, 4 outputs x 16 samples per pass (8 vector
 * accumulators, each loaded activation row used by 4 outputs) */
static void linear_block(const float* W, const float* b, int din, int dout, const float* a, float* h) {
  int o = 0;
  for (; o + 4 <= dout; o += 4) {
    v8f acc[4][2];
    for (int r = 0; r < 4; ++r) acc[r][0] = acc[r][1] = (v8f){0, 0, 0, 0, 0, 0, 0, 0} + b[o + r];
    const float* w0 = W + (size_t)o * din;
    for (int i = 0; i < din; ++i) {
      v8f x0, x1;
      memcpy(&x0, a + i * BLK, 32);
      memcpy(&x1, a + i * BLK + 8, 32);
      for (int r = 0; r < 4; ++r) {
        const float wv = w0[(size_t)r * din + i];
        acc[r][0] += wv * x0;
        acc[r][1] += wv * x1;
      }
    }
    for (int r = 0; r < 4; ++r) {
      memcpy(h + (o + r) * BLK, &acc[r][0], 32);
      memcpy(h + (o + r) * BLK + 8, &acc[r][1], 32);
    }
  }
  for (; o < dout; ++o) {
    v8f acc0 = (v8f){0, 0, 0, 0, 0, 0, 0, 0} + b[o], acc1 = acc0;
    const float* wr = W + (size_t)o * din;
    for (int i = 0; i < din; ++i) {
      v8f x0, x1;
      memcpy(&x0, a + i * BLK, 32);
      memcpy(&x1, a + i * BLK + 8, 32);
      acc0 += wr[i] * x0;
      acc1 += wr[i] * x1;
    }
    memcpy(h + o * BLK, &acc0, 32);
    memcpy(h + o * BLK + 8, &acc1, 32);
  }
}

/* one block of up to BLK samples through the horizon; act buffers are [feature][BLK] */
static void fc_block(const mppi_cpu_net* net, int nx, int nu, int K, int H, int k0, int nb, int cost_kind,
                     const float* ctx, const float* x0, const float* U, const float* noise, float ctrl_clamp,
                     float terminal_weight, float* costs, float* buf, int maxd) {
  float* a = buf;                 /* [maxd][BLK] */
  float* h = buf + maxd * BLK;    /* [maxd][BLK] */
  float* xs = h + maxd * BLK;     /* [nx][BLK] state */
  float xr[256];                  /* one sample's state (cost gather), nx <= 256 */
  float c[BLK];
  for (int j = 0; j < BLK; ++j) c[j] = 0.0f;
  for (int i = 0; i < nx; ++i)
    for (int j = 0; j < BLK; ++j) xs[i * BLK + j] = x0[i];
  for (int t = 0; t < H; ++t) {
    float usq[BLK], u0[BLK];
    for (int j = 0; j < BLK; ++j) usq[j] = 0.0f;
    for (int i = 0; i < nx; ++i) memcpy(a + i * BLK, xs + i * BLK, sizeof(float) * BLK);
    for (int q = 0; q < nu; ++q) {
      const float* e = noise + ((size_t)q * H + t) * K + k0;
      for (int j = 0; j < BLK; ++j) {
        float u = U[q * H + t] + (j < nb ? e[j] : 0.0f);
        if (ctrl_clamp > 0.0f) u = u > ctrl_clamp ? ctrl_clamp : (u < -ctrl_clamp ? -ctrl_clamp : u);
        a[(nx + q) * BLK + j] = u;
        usq[j] += u * u;
        if (q == 0) u0[j] = u;
      }
    }
    for (int l = 0; l < net->nl; ++l) {
      const int din = net->dims[l], dout = net->dims[l + 1];
      linear_block(net->W[l], net->b[l], din, dout, a, h);
      if (net->lng[l]) { /* LayerNorm over dout, per sample */
        float mu[BLK], var[BLK];
        for (int j = 0; j < BLK; ++j) mu[j] = var[j] = 0.0f;
        for (int o = 0; o < dout; ++o)
          for (int j = 0; j < BLK; ++j) mu[j] += h[o * BLK + j];
        for (int j = 0; j < BLK; ++j) mu[j] /= (float)dout;
        for (int o = 0; o < dout; ++o)
          for (int j = 0; j < BLK; ++j) {
            const float d = h[o * BLK + j] - mu[j];
            var[j] += d * d;
          }
        for (int j = 0; j < BLK; ++j) var[j] = 1.0f / sqrtf(var[j] / (float)dout + 1e-5f);
        for (int o = 0; o < dout; ++o) {
          const float g = net->lng[l][o], be = net->lnb[l][o];
          for (int j = 0; j < BLK; ++j) h[o * BLK + j] = (h[o * BLK + j] - mu[j]) * var[j] * g + be;
        }
      }
      if (net->relu[l])
        for (int o = 0; o < dout * BLK; ++o) h[o] = h[o] > 0.0f ? h[o] : 0.0f;
      float* tmp = a;
      a = h;
      h = tmp;
    }
    for (int i = 0; i < nx; ++i)
      for (int j = 0; j < BLK; ++j) xs[i * BLK + j] += a[i * BLK + j];
    for (int j = 0; j < nb; ++j) {
      for (int i = 0; i < nx; ++i) xr[i] = xs[i * BLK + j];
      c[j] += run_cost(cost_kind, xr, u0[j], usq[j], ctx);
    }
    if (a != buf) { /* keep a = buf, h = second buffer for the next step */
      float* tmp = a;
      a = h;
      h = tmp;
    }
  }
  for (int j = 0; j < nb; ++j) {
    if (terminal_weight != 0.0f) {
      for (int i = 0; i < nx; ++i) xr[i] = xs[i * BLK + j];
      c[j] += terminal_weight * run_cost(cost_kind, xr, 0.0f, 0.0f, ctx);
    }
    costs[k0 + j] = c[j];
  }
}

/* Solve one learned-dynamics MPPI step.  U [nu][H] in/out, noise [nu][H][K], costs_out / w_out NULL or [K]. */
int mppi_cpu_fc_solve(const mppi_cpu_net* net, int nx, int nu, int K, int H, int cost_kind, const float* ctx,
                      const float* x0, float* U, const float* noise, float lam, float ctrl_clamp, float U_clamp,
                      float norm_eps, float terminal_weight, int update_replace, float* costs_out, float* w_out,
                      int nthreads) {
  if (!net || net->nl < 1 || net->nl > MAXL || nx > 256 || net->dims[0] != nx + nu || K < 1 || H < 1) return -1;
  int maxd = 0;
  for (int l = 0; l <= net->nl; ++l) maxd = net->dims[l] > maxd ? net->dims[l] : maxd;
  const int nth = nthreads > 0 ? nthreads : 1;
  float* costs = costs_out ? costs_out : (float*)malloc(sizeof(float) * K);
  const int nblk = (K + BLK - 1) / BLK;
#pragma omp parallel num_threads(nth)
  {
    float* buf = (float*)malloc(sizeof(float) * (2 * maxd + nx) * BLK);
#pragma omp for schedule(dynamic, 1)
    for (int bi = 0; bi < nblk; ++bi) {
      const int k0 = bi * BLK, nb = K - k0 < BLK ? K - k0 : BLK;
      fc_block(net, nx, nu, K, H, k0, nb, cost_kind, ctx, x0, U, noise, ctrl_clamp, terminal_weight, costs, buf, maxd);
    }
    free(buf);
  }
  const int rc = softmin_update(K, nu * H, costs, noise, lam, norm_eps, update_replace, U_clamp, U, w_out, nth);
  if (!costs_out) free(costs);
  return rc;
}

/* ------------------------------------------------------------------------------------------------ cartpole */

/* models/cartpole.xml compiled the way MuJoCo does (oracle/mppi_ref.py:_cartpole_params) */
typedef struct {
  double mc, mp, l, I, D, gear, g, dt;
} cp_params;

static cp_params cartpole_params(void) {
  const double rho = 1000.0, r = 0.045, L = 0.6, pi = 3.14159265358979323846;
  const double mcyl = rho * pi * r * r * L, msph = rho * 4.0 / 3.0 * pi * r * r * r;
  cp_params p;
  p.mc = rho * 0.4 * 0.2 * 0.1;
  p.mp = mcyl + msph;
  p.l = L / 2.0;
  p.I = mcyl * (L * L / 12.0 + r * r / 4.0) + msph * (2.0 * r * r / 5.0 + L * L / 4.0 + 3.0 * L * r / 8.0);
  p.D = 0.05;
  p.gear = 50.0;
  p.g = 9.81;
  p.dt = 0.01;
  return p;
}

/* one mj_step (semi-implicit Euler, implicit joint damping), oracle/mppi_ref.py:cartpole_step */
static void cartpole_step(const cp_params* p, double* x, double u) {
  const double th = x[1], xd = x[2], thd = x[3];
  const double F = p->gear * (u > 1.0 ? 1.0 : (u < -1.0 ? -1.0 : u));
  const double s = sin(th), c = cos(th);
  const double m11 = p->mc + p->mp + p->dt * p->D, m12 = p->mp * p->l * c;
  const double m22 = p->mp * p->l * p->l + p->I + p->dt * p->D;
  const double f1 = F + p->mp * p->l * s * thd * thd - p->D * xd, f2 = p->mp * p->g * p->l * s - p->D * thd;
  const double det = m11 * m22 - m12 * m12;
  const double a1 = (m22 * f1 - m12 * f2) / det, a2 = (m11 * f2 - m12 * f1) / det;
  const double xdn = xd + p->dt * a1, thdn = thd + p->dt * a2;
  x[0] += p->dt * xdn;
  x[1] += p->dt * thdn;
  x[2] = xdn;
  x[3] = thdn;
}

static double cartpole_cost(const double* x, double u) { /* src/cartpole_mppi.py:44-50 */
  const double c = cos(x[1]) - 1.0;
  return x[0] * x[0] + 20.0 * c * c + 0.1 * x[2] * x[2] + 0.1 * x[3] * x[3] + 0.01 * u * u;
}

/* One cartpole MPPI step (src/cartpole_mppi.py:59-98), fp64.  U [H] in/out, noise [H][K]. */
int mppi_cpu_cartpole_solve(int K, int H, const double* x0, double* U, const double* noise, double lam,
                            double terminal_weight, int update_replace, double* costs_out, double* w_out,
                            int nthreads) {
  if (K < 1 || H < 1) return -1;
  const cp_params p = cartpole_params();
  const int nth = nthreads > 0 ? nthreads : 1;
  double* costs = costs_out ? costs_out : (double*)malloc(sizeof(double) * K);
#pragma omp parallel for num_threads(nth) schedule(static)
  for (int k = 0; k < K; ++k) {
    double x[4] = {x0[0], x0[1], x0[2], x0[3]}, c = 0.0;
    for (int t = 0; t < H; ++t) {
      const double u = U[t] + noise[(size_t)t * K + k];
      cartpole_step(&p, x, u);
      c += cartpole_cost(x, u); /* post-step state, raw ctrl (src/cartpole_mppi.py:78) */
    }
    if (terminal_weight != 0.0) c += terminal_weight * cartpole_cost(x, 0.0);
    costs[k] = c;
  }
  double beta = INFINITY, S = 0.0;
  for (int k = 0; k < K; ++k)
    if (isfinite(costs[k]) && costs[k] < beta) beta = costs[k];
  if (!isfinite(beta)) {
    if (!costs_out) free(costs);
    return -4;
  }
  double* w = (double*)malloc(sizeof(double) * K);
  for (int k = 0; k < K; ++k) {
    w[k] = isfinite(costs[k]) ? exp(-(costs[k] - beta) / lam) : 0.0;
    S += w[k];
  }
  for (int k = 0; k < K; ++k) {
    w[k] /= S;
    if (w_out) w_out[k] = w[k];
  }
#pragma omp parallel for num_threads(nth) schedule(static)
  for (int t = 0; t < H; ++t) {
    double acc = 0.0;
    for (int k = 0; k < K; ++k) acc += w[k] * noise[(size_t)t * K + k];
    U[t] = update_replace ? acc : U[t] + acc;
  }
  free(w);
  if (!costs_out) free(costs);
  return 0;
}
