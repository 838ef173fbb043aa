// C-ABI of the MPPI engine (include/mppi.h): handle lifecycle, device buffers, the solve pipeline
// (noise -> rollout -> reduce -> update) on one HIP stream, layout conversion at the boundary,
// per-kernel hipEvent timing, thread-local error strings. Never throws across the ABI.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "costs.h"
#include "fc_common.h"  // x3_l1_terms, kX3ProbeTol (the split CA's layer-1 probe)
#include "mppi_internal.h"

namespace mppi {
std::vector<unsigned char> build_fc_net(int kind, const void* blob, size_t nbytes, int precision, int nx, int nu,
                                        FcNet& net);
std::vector<unsigned char> build_fa_net(const void* blob, size_t nbytes, int precision, int nx, int nu, FaNet& net);
int fa_lds_bytes(int D, int precision, int nh, int L);
}

using namespace mppi;

static thread_local std::string g_err;

static int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIP_TRY(expr)                                                                                        \
  do {                                                                                                       \
    hipError_t e_ = (expr);                                                                                  \
    if (e_ != hipSuccess) return fail(MPPI_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));       \
  } while (0)

namespace {

enum KernelId { kNoise = 0, kRollout = 1, kReduce = 2, kUpdate = 3, kNumKernels = 4 };
const char* kKernelNames[kNumKernels] = {"noise", "rollout", "reduce", "update"};

struct PendingEvt {
  int id;
  hipEvent_t a, b;
};

}  // namespace

struct mppi_handle {
  mppi_config cfg{};
  int device = 0;
  int Kp = 0;
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  int dyn_kind = 0;
  int cost_kind = 0;
  float cost_params[MPPI_CTX_MAX] = {0};
  CartpoleParams cart{};
  FcNet net;
  FaNet fa;
  // device buffers (sized for cfg.max_batch)
  float *d_x0 = nullptr, *d_U = nullptr, *d_noise = nullptr, *d_costs = nullptr, *d_dU = nullptr;
  float *d_weights = nullptr, *d_u0 = nullptr, *d_ctx = nullptr;
  unsigned* d_status = nullptr;
  unsigned* d_tickets = nullptr;
  float* d_part = nullptr;        // analytic cartpole: per-block softmin partials of the fused epilogue
  unsigned long long* d_seed_ctr = nullptr;
  float *d_env_noise = nullptr, *d_env_costs = nullptr;  // env step (zero noise, cost scratch)
  unsigned* d_env_status = nullptr;
  // graph mode: noise double buffer (d_noise, d_noise2); solve i's reduce also generates solve i+1's noise
  // (reduce_kernel<GEN>).  One exec per start parity of the buffer pair.
  float* d_noise2 = nullptr;
  unsigned* d_gticket = nullptr;
  hipGraphExec_t graph_exec[2] = {nullptr, nullptr};
  int graph_B = 0, graph_n = 0, graph_parity = 0;
  bool prefetch_valid = false;  // d_noise / d_noise2 [graph_parity] holds the next launch's first noise
  int prefetch_B = 0;           // ... generated for this batch and seed (graph launches and chained solves)
  uint64_t prefetch_seed = 0;
  bool capturing = false;       // enqueue_solve is recording a graph (launches are counted at replay)
  uint64_t graph_seed = 0;
  std::vector<float> Uhost;  // column-major U staging between enqueue and finish
  // profiling
  bool prof = false;
  std::vector<PendingEvt> pending;
  std::vector<hipEvent_t> evt_pool;
  long prof_count[kNumKernels] = {0};
  double prof_ms[kNumKernels] = {0};
  std::vector<float> staging;
  // device launch clock of the rollouts (mppi_kernel_clock): [kClockSlots][2] {first block start, last block end}
  unsigned long long* d_kclock = nullptr;
  bool kclock = false;        // stamp rollouts enqueued (or captured) from now on
  bool graph_kclock = false;  // the captured graph stamps its rollouts
  long kclock_launches = 0;   // stamped rollout launches since the last reset
  // chained solves with the next solve's noise generated CONCURRENTLY with this solve's rollout (gen_overlap): a
  // low-priority generator stream running noise_kernel + the counter bump, ordered by events against the solve stream
  hipStream_t gstream = nullptr;
  hipEvent_t ev_gen = nullptr;  // the generator's last launch done (the noise the next rollout reads is written)
  hipEvent_t ev_red = nullptr;  // the solve stream's last reduce done (the buffer it read may be overwritten)
  hipEvent_t ev_switch = nullptr;  // mppi_set_stream: the old stream's tail, waited on by the new one
  bool gen_pending = false;     // ev_gen guards the prefetched noise: the solve stream must wait on it before use
  const char* rollout_kernel = "";  // the kernel the last solve's rollout was routed to (mppi_rollout_kernel)
};

static hipEvent_t take_event(mppi_handle* h) {
  if (!h->evt_pool.empty()) {
    hipEvent_t e = h->evt_pool.back();
    h->evt_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  (void)hipEventCreate(&e);
  return e;
}

static void harvest_events(mppi_handle* h) {
  for (auto& p : h->pending) {
    float ms = 0.0f;
    if (hipEventSynchronize(p.b) == hipSuccess && hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
      h->prof_count[p.id] += 1;
      h->prof_ms[p.id] += ms;
    }
    h->evt_pool.push_back(p.a);
    h->evt_pool.push_back(p.b);
  }
  h->pending.clear();
}

// Enqueue `launch` on the handle's stream, bracketed by events when profiling.
template <class F>
static hipError_t timed(mppi_handle* h, int id, F&& launch) {
  if (!h->prof) return launch();
  if (h->pending.size() > 4096) harvest_events(h);
  PendingEvt p{id, take_event(h), take_event(h)};
  (void)hipEventRecord(p.a, h->stream);
  hipError_t e = launch();
  (void)hipEventRecord(p.b, h->stream);
  h->pending.push_back(p);
  return e;
}

static CartpoleParams default_cartpole() {
  // models/cartpole.xml compiled as MuJoCo does (oracle/mppi_ref.py::_cartpole_params states the derivation).
  const double rho = 1000.0, r = 0.045, L = 0.6, pi = 3.14159265358979323846;
  const double m_cyl = rho * pi * r * r * L, m_sph = rho * 4.0 / 3.0 * pi * r * r * r;
  const double I = m_cyl * (L * L / 12.0 + r * r / 4.0) + m_sph * (2.0 * r * r / 5.0 + L * L / 4.0 + 3.0 * L * r / 8.0);
  CartpoleParams p;
  p.m_cart = (float)(rho * 0.4 * 0.2 * 0.1);
  p.m_pole = (float)(m_cyl + m_sph);
  p.l = (float)(L / 2.0);
  p.inertia = (float)I;
  p.damping = 0.05f;
  p.gear = 50.0f;
  p.ctrl_lo = -1.0f;
  p.ctrl_hi = 1.0f;
  p.g = 9.81f;
  p.dt = 0.01f;
  return p;
}

// --------------------------------------------------------------------------------------- presets

struct PresetRow {
  const char* name;
  int nx, nu, K, H;
  float lambda, sigma, ctrl_clamp, U_clamp, norm_eps, shift_fill, terminal_weight;
  int update_mode;
};

// SURVEY 8a variant table; constants cited from the reference scripts.
static const PresetRow kPresets[] = {
    {"cartpole_py", 4, 1, 30, 100, 1.0f, 1.0f, 0, 0, 0, 0.1f, 10.0f, MPPI_UPDATE_ADD},          // cartpole_mppi.py:12-15
    {"cartpole_jl", 4, 1, 30, 100, 1.0f, 1.0f, 0, 0, 0, 0.1f, 10.0f, MPPI_UPDATE_ADD},          // cartpole_mppi.jl:11-14
    {"cartpole_collect", 4, 1, 75, 100, 1.0f, 0.75f, 0, 0, 0, 0.1f, 10.0f, MPPI_UPDATE_ADD},    // cartpole_datacollection.py:13-16
    {"quad_mppi_jl", 37, 12, 50, 30, 0.2f, 0.3f, 10.0f, 10.0f, 1e-10f, 0.0f, 0.0f, MPPI_UPDATE_ADD},  // mppi.jl:10-13
    {"humanoid_v3", 55, 21, 30, 75, 1.0f, 0.75f, 0, 0, 0, 0.1f, 10.0f, MPPI_UPDATE_ADD},        // Humanoid_mppi_v3.jl:13-16
    {"humanoid_v1", 55, 21, 50, 100, 1.0f, 1.0f, 0, 0, 0, 0.1f, 10.0f, MPPI_UPDATE_ADD},        // Humanoid_mppi.jl:22-25
    {"humanoid_collect_v2", 55, 21, 50, 100, 1.0f, 0.5f, 0, 0, 0, 0.1f, 10.0f, MPPI_UPDATE_ADD},  // Humanoid_datacollection_v2.jl:46-49
    {"cartpole_est", 4, 1, 2048, 100, 10.0f, 0.5f, 0, 0, 0, 0.1f, 10.0f, MPPI_UPDATE_REPLACE},  // cartpole_mppi_estimator.py:37-40
    {"quad_est", 37, 12, 2048, 50, 10.0f, 0.4f, 0, 0, 0, 0.1f, 10.0f, MPPI_UPDATE_REPLACE},     // quadruped_mppi_estimator.py:38-41
};

extern "C" {

const char* mppi_last_error(void) { return g_err.c_str(); }
int mppi_abi_version(void) { return MPPI_ABI_VERSION; }
#ifndef MPPI_BUILD_ID
#define MPPI_BUILD_ID "unknown"
#endif
const char* mppi_build_id(void) { return MPPI_BUILD_ID; }  // build.py passes the source hash

int mppi_preset(const char* name, mppi_config* cfg) {
  if (!name || !cfg) return fail(MPPI_E_ARG, "mppi_preset: null argument");
  for (const PresetRow& p : kPresets) {
    if (std::strcmp(p.name, name) == 0) {
      std::memset(cfg, 0, sizeof(*cfg));
      cfg->nx = p.nx;
      cfg->nu = p.nu;
      cfg->K = p.K;
      cfg->H = p.H;
      cfg->max_batch = 1;
      cfg->lambda = p.lambda;
      cfg->sigma = p.sigma;
      cfg->ctrl_clamp = p.ctrl_clamp;
      cfg->U_clamp = p.U_clamp;
      cfg->norm_eps = p.norm_eps;
      cfg->shift_fill = p.shift_fill;
      cfg->terminal_weight = p.terminal_weight;
      cfg->update_mode = p.update_mode;
      cfg->precision = MPPI_PREC_BF16;
      return MPPI_OK;
    }
  }
  return fail(MPPI_E_ARG, std::string("mppi_preset: unknown preset ") + name);
}

void mppi_destroy(mppi_handle* h) {
  if (!h) return;
  (void)hipSetDevice(h->device);
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  harvest_events(h);
  for (hipEvent_t e : h->evt_pool) (void)hipEventDestroy(e);
  void* bufs[] = {h->d_x0, h->d_U, h->d_noise, h->d_costs, h->d_dU, h->d_weights, h->d_u0, h->d_ctx, h->d_status,
                  h->d_tickets, h->net.d_img, h->fa.d_img, h->fa.d_ws, h->d_seed_ctr, h->d_env_noise, h->d_env_costs,
                  h->d_env_status, h->d_noise2, h->d_gticket, h->d_part, h->d_kclock};
  for (hipGraphExec_t& g : h->graph_exec)
    if (g) (void)hipGraphExecDestroy(g);
  if (h->gstream) (void)hipStreamSynchronize(h->gstream);
  for (void* p : bufs)
    if (p) (void)hipFree(p);
  if (h->ev_gen) (void)hipEventDestroy(h->ev_gen);
  if (h->ev_red) (void)hipEventDestroy(h->ev_red);
  if (h->ev_switch) (void)hipEventDestroy(h->ev_switch);
  if (h->gstream) (void)hipStreamDestroy(h->gstream);
  if (h->own_stream) (void)hipStreamDestroy(h->own_stream);
  delete h;
}

int mppi_create(const mppi_config* cfg, int device, mppi_handle** out) {
  if (!cfg || !out) return fail(MPPI_E_ARG, "mppi_create: null argument");
  *out = nullptr;
  const mppi_config& c = *cfg;
  if (c.nx < 1 || c.nx > 4096 || c.nu < 1 || c.nu > 4096 || c.H < 1 || c.K < 1 || c.K > kMaxK || c.max_batch < 1)
    return fail(MPPI_E_ARG, "mppi_create: bad dimensions (need nx,nu,H,K,max_batch >= 1, K <= 32768)");
  if (!(c.lambda > 0.0f)) return fail(MPPI_E_ARG, "mppi_create: lambda must be > 0");
  if (c.update_mode != MPPI_UPDATE_ADD && c.update_mode != MPPI_UPDATE_REPLACE)
    return fail(MPPI_E_ARG, "mppi_create: bad update_mode");
  if (c.precision != MPPI_PREC_FP32 && c.precision != MPPI_PREC_BF16 && c.precision != MPPI_PREC_BF16X3)
    return fail(MPPI_E_ARG, "mppi_create: bad precision");
  if ((size_t)c.nu * c.H * sizeof(float) > 64 * 1024) return fail(MPPI_E_ARG, "mppi_create: nu*H too large (> 16384)");
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return fail(MPPI_E_ARG, "mppi_create: no such device");
  HIP_TRY(hipSetDevice(device));
  mppi_handle* h = new (std::nothrow) mppi_handle();
  if (!h) return fail(MPPI_E_ARG, "mppi_create: out of host memory");
  h->cfg = c;
  h->device = device;
  h->Kp = (c.K + kKpAlign - 1) / kKpAlign * kKpAlign;
  h->cart = default_cartpole();
  const size_t B = (size_t)c.max_batch;
  auto alloc = [&](void** p, size_t bytes) -> hipError_t {
    hipError_t e = hipMalloc(p, bytes < 16 ? 16 : bytes);
    if (e == hipSuccess) e = hipMemset(*p, 0, bytes < 16 ? 16 : bytes);
    return e;
  };
  hipError_t e = hipStreamCreateWithFlags(&h->own_stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = alloc((void**)&h->d_x0, B * c.nx * 4);
  if (e == hipSuccess) e = alloc((void**)&h->d_U, B * c.nu * c.H * 4);
  if (e == hipSuccess) e = alloc((void**)&h->d_noise, B * c.nu * c.H * (size_t)h->Kp * 4);
  if (e == hipSuccess) e = alloc((void**)&h->d_costs, B * h->Kp * 4);
  if (e == hipSuccess) e = alloc((void**)&h->d_dU, B * c.nu * c.H * 4);
  if (e == hipSuccess) e = alloc((void**)&h->d_weights, B * h->Kp * 4);
  if (e == hipSuccess) e = alloc((void**)&h->d_u0, B * c.nu * 4);
  if (e == hipSuccess) e = alloc((void**)&h->d_ctx, B * MPPI_CTX_MAX * 4);
  if (e == hipSuccess) e = alloc((void**)&h->d_status, 16);
  if (e == hipSuccess) e = alloc((void**)&h->d_tickets, B * 4);
  if (e == hipSuccess) e = alloc((void**)&h->d_seed_ctr, 8);
  if (e == hipSuccess) e = alloc((void**)&h->d_env_noise, B * c.nu * kKpAlign * 4);
  if (e == hipSuccess) e = alloc((void**)&h->d_env_costs, B * kKpAlign * 4);
  if (e == hipSuccess) e = alloc((void**)&h->d_env_status, 16);
  if (e != hipSuccess) {
    mppi_destroy(h);
    return fail(MPPI_E_HIP, std::string("mppi_create: ") + hipGetErrorString(e));
  }
  h->stream = h->own_stream;
  *out = h;
  return MPPI_OK;
}

int mppi_load_dynamics(mppi_handle* h, int kind, const void* blob, size_t nbytes) {
  if (!h) return fail(MPPI_E_ARG, "mppi_load_dynamics: null handle");
  HIP_TRY(hipSetDevice(h->device));
  if (kind == MPPI_DYN_CARTPOLE) {
    if (h->cfg.nx != 4 || h->cfg.nu != 1) return fail(MPPI_E_ARG, "cartpole dynamics need nx=4, nu=1");
    h->cart = default_cartpole();
    if (!h->d_part) {  // [max_batch][Kp/256][2 + H] partial records (fixed by the config: allocated once)
      const size_t n = (size_t)h->cfg.max_batch * ((h->Kp + 255) / 256) * (2 + h->cfg.H) * sizeof(float);
      HIP_TRY(hipMalloc(&h->d_part, n));
      HIP_TRY(hipMemset(h->d_part, 0, n));
    }
    if (blob) {
      if (nbytes != 10 * sizeof(float)) return fail(MPPI_E_ARG, "cartpole params: expected 10 floats");
      std::memcpy(&h->cart, blob, sizeof(CartpoleParams));
    }
    h->dyn_kind = kind;
    return MPPI_OK;
  }
  if (kind == MPPI_DYN_MLP || kind == MPPI_DYN_CROSS_ATTN) {
    if (!blob || nbytes == 0) return fail(MPPI_E_ARG, "mppi_load_dynamics: weight blob required");
    std::vector<unsigned char> img;
    FcNet net;
    try {
      img = build_fc_net(kind, blob, nbytes, h->cfg.precision, h->cfg.nx, h->cfg.nu, net);
    } catch (const std::exception& ex) {
      return fail(MPPI_E_UNSUPPORTED, std::string("mppi_load_dynamics: ") + ex.what());
    }
    if (h->cfg.precision == MPPI_PREC_BF16 && net.lds_bytes > 128 * 1024)
      return fail(MPPI_E_UNSUPPORTED, "mppi_load_dynamics: LDS part of the packed bf16 image exceeds 128 KiB");
    HIP_TRY(hipStreamSynchronize(h->stream));
    void* d = nullptr;
    HIP_TRY(hipMalloc(&d, img.size()));
    if (const hipError_t e = hipMemcpy(d, img.data(), img.size(), hipMemcpyHostToDevice); e != hipSuccess) {
      (void)hipFree(d);
      return fail(MPPI_E_HIP, std::string("mppi_load_dynamics: image upload: ") + hipGetErrorString(e));
    }
    if (h->net.d_img) (void)hipFree(h->net.d_img);
    net.d_img = d;
    net.x3_l1 = 0;  // a new net: the split layer-1 probe runs again at the next solve (x3_probe)
    h->net = net;
    h->dyn_kind = kind;
    return MPPI_OK;
  }
  if (kind == MPPI_DYN_FEATURE_ATTN) {
    if (!blob || nbytes == 0) return fail(MPPI_E_ARG, "mppi_load_dynamics: weight blob required");
    if (h->cfg.precision == MPPI_PREC_BF16X3)
      return fail(MPPI_E_UNSUPPORTED, "mppi_load_dynamics: MPPI_PREC_BF16X3 is built for the fc nets (MLP, CA) only");
    std::vector<unsigned char> img;
    FaNet net;
    try {
      img = build_fa_net(blob, nbytes, h->cfg.precision, h->cfg.nx, h->cfg.nu, net);
    } catch (const std::exception& ex) {
      return fail(MPPI_E_UNSUPPORTED, std::string("mppi_load_dynamics: ") + ex.what());
    }
    const int lds = fa_lds_bytes(net.D, net.precision, net.nh, net.L);
    if (lds <= 0 || lds > 160 * 1024)
      return fail(MPPI_E_UNSUPPORTED, "mppi_load_dynamics: feature-attention shape does not fit the kernel's LDS");
    HIP_TRY(hipStreamSynchronize(h->stream));
    // the new image first: the loaded net stays in place (and usable) if anything below fails
    void* d = nullptr;
    HIP_TRY(hipMalloc(&d, img.size()));
    if (const hipError_t e = hipMemcpy(d, img.data(), img.size(), hipMemcpyHostToDevice); e != hipSuccess) {
      (void)hipFree(d);
      return fail(MPPI_E_HIP, std::string("mppi_load_dynamics: image upload: ") + hipGetErrorString(e));
    }
    net.d_img = d;
    const char* lay_env = getenv("MPPI_FA_LAYERED");
    if (net.lay && lay_env && atoi(lay_env) == 1) {  // the layer-by-layer hidden-512 path's activations (~10 KB per
                                                      // token row; skipped above 32 GiB), only when it is selected
      const long rows = (long)h->cfg.max_batch * h->cfg.K * net.L;
      const size_t ws = fa_layered_ws_bytes(rows);
      // an optional workspace: if it cannot be had, the fused kernel runs (net.d_ws stays null), no error
      if (ws <= ((size_t)32 << 30) && hipMalloc(&net.d_ws, ws) == hipSuccess) {
        if (hipMemset(net.d_ws, 0, ws) == hipSuccess) {
          net.ws_rows = rows;
        } else {
          (void)hipFree(net.d_ws);
          net.d_ws = nullptr;
        }
      }
      (void)hipGetLastError();  // a failed optional allocation leaves no sticky error behind
    }
    if (h->fa.d_img) (void)hipFree(h->fa.d_img);
    if (h->fa.d_ws) (void)hipFree(h->fa.d_ws);
    h->fa = net;
    h->dyn_kind = kind;
    return MPPI_OK;
  }
  return fail(MPPI_E_UNSUPPORTED, "mppi_load_dynamics: unknown dynamics kind");
}

int mppi_set_cost(mppi_handle* h, int kind, const float* params, int nparams) {
  if (!h) return fail(MPPI_E_ARG, "mppi_set_cost: null handle");
  if (kind < MPPI_COST_CARTPOLE || kind > MPPI_COST_HUMANOID_V1) return fail(MPPI_E_UNSUPPORTED, "unknown cost kind");
  const CostIdx ci = cost_idx(kind);
  for (int i = 0; i < ci.n; ++i)
    if (ci.idx[i] >= h->cfg.nx) return fail(MPPI_E_ARG, "mppi_set_cost: cost reads state entries beyond nx");
  if (nparams < 0 || nparams > MPPI_CTX_MAX || (nparams > 0 && !params))
    return fail(MPPI_E_ARG, "mppi_set_cost: params must be <= 8 floats");
  float def[MPPI_CTX_MAX] = {0};
  if (kind == MPPI_COST_HUMANOID_V3 || kind == MPPI_COST_HUMANOID_V1) {
    // src/Humanoid_mppi_v3.jl:12 target (v1: the constants of src/Humanoid_mppi.jl:36,56); no real-env terms by default
    def[0] = 2.0f;
    def[1] = 0.0f;
    def[2] = 1.28f;
  } else if (kind == MPPI_COST_QUAD_EST) {  // src/quadruped_mppi_estimator.py:45
    def[0] = 2.0f;
    def[1] = 0.0f;
    def[2] = 0.35f;
  }
  for (int i = 0; i < nparams; ++i) def[i] = params[i];
  std::memcpy(h->cost_params, def, sizeof(def));
  h->cost_kind = kind;
  return MPPI_OK;
}

int mppi_set_stream(mppi_handle* h, void* s) {
  if (!h) return fail(MPPI_E_ARG, "mppi_set_stream: null handle");
  const hipStream_t ns = s ? (hipStream_t)s : h->own_stream;
  if (ns != h->stream && (h->gen_pending || h->prefetch_valid)) {
    // chained-solve state spans the switch: the next chained solve reads the noise the previous one prefetched, and
    // (MPPI_GEN_OVERLAP) the generator stream orders itself behind ev_red recorded on the CURRENT stream as "the
    // previous reduce".  Order the new stream behind everything already on the old one, so that both hold across it.
    HIP_TRY(hipSetDevice(h->device));
    if (!h->ev_switch) HIP_TRY(hipEventCreateWithFlags(&h->ev_switch, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(h->ev_switch, h->stream));
    HIP_TRY(hipStreamWaitEvent(ns, h->ev_switch, 0));
  }
  h->stream = ns;
  return MPPI_OK;
}

int mppi_sync(mppi_handle* h) {
  if (!h) return fail(MPPI_E_ARG, "mppi_sync: null handle");
  HIP_TRY(hipSetDevice(h->device));
  HIP_TRY(hipStreamSynchronize(h->stream));
  return MPPI_OK;
}

int mppi_profile(mppi_handle* h, int enable) {
  if (!h) return fail(MPPI_E_ARG, "mppi_profile: null handle");
  if (enable && !h->prof) {
    harvest_events(h);
    for (int i = 0; i < kNumKernels; ++i) {
      h->prof_count[i] = 0;
      h->prof_ms[i] = 0.0;
    }
  }
  h->prof = enable != 0;
  return MPPI_OK;
}

int mppi_kernel_time(mppi_handle* h, const char* kernel, int* count, double* total_ms) {
  if (!h || !kernel) return fail(MPPI_E_ARG, "mppi_kernel_time: null argument");
  harvest_events(h);
  for (int i = 0; i < kNumKernels; ++i) {
    if (std::strcmp(kernel, kKernelNames[i]) == 0) {
      if (count) *count = (int)h->prof_count[i];
      if (total_ms) *total_ms = h->prof_ms[i];
      return MPPI_OK;
    }
  }
  return fail(MPPI_E_ARG, std::string("mppi_kernel_time: unknown kernel ") + kernel);
}

int mppi_kernel_clock(mppi_handle* h, int enable) {
  if (!h) return fail(MPPI_E_ARG, "mppi_kernel_clock: null handle");
  HIP_TRY(hipSetDevice(h->device));
  if (enable) {
    // [kClockSlots][2] stamps, then the launch counter and the block-arrival ticket (mppi_internal.h::KClock)
    const size_t n = 2 * (size_t)kClockSlots + 2;
    if (!h->d_kclock) HIP_TRY(hipMalloc(&h->d_kclock, n * sizeof(unsigned long long)));
    std::vector<unsigned long long> init(n, 0ull);
    for (size_t i = 0; i < 2 * (size_t)kClockSlots; i += 2) init[i] = ~0ull;  // start = min, end = max over blocks
    HIP_TRY(hipMemcpyAsync(h->d_kclock, init.data(), n * sizeof(unsigned long long), hipMemcpyHostToDevice, h->stream));
    HIP_TRY(hipStreamSynchronize(h->stream));
    h->kclock_launches = 0;
  }
  h->kclock = enable != 0;
  return MPPI_OK;
}

int mppi_kernel_clock_read(mppi_handle* h, int* launches, double* total_us, double* max_us) {
  if (!h || !launches || !total_us) return fail(MPPI_E_ARG, "mppi_kernel_clock_read: null argument");
  *launches = 0;
  *total_us = 0.0;
  if (max_us) *max_us = 0.0;
  if (!h->d_kclock) return fail(MPPI_E_STATE, "mppi_kernel_clock_read: call mppi_kernel_clock(h, 1) first");
  if (h->kclock_launches > kClockSlots)
    return fail(MPPI_E_UNSUPPORTED, "mppi_kernel_clock_read: more stamped launches than clock slots since the reset");
  HIP_TRY(hipSetDevice(h->device));
  int rate_khz = 0;  // s_memrealtime frequency
  HIP_TRY(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, h->device));
  if (rate_khz <= 0) return fail(MPPI_E_HIP, "mppi_kernel_clock_read: no device wall-clock rate");
  std::vector<unsigned long long> v(2 * (size_t)kClockSlots + 1);  // the slots, then the device launch counter
  HIP_TRY(hipStreamSynchronize(h->stream));
  HIP_TRY(hipMemcpy(v.data(), h->d_kclock, v.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  const unsigned long long dev_launches = v.back();
  v.pop_back();
  // kclock_record's invariant (one stamping leader per block of every stamped launch): the device counter has
  // advanced once per launch the host issued; a kernel that broke it would fold later launches into one slot
  if (dev_launches != (unsigned long long)h->kclock_launches)
    return fail(MPPI_E_STATE, "mppi_kernel_clock_read: device launch counter (" + std::to_string(dev_launches) +
                                  ") != stamped launches (" + std::to_string(h->kclock_launches) +
                                  "): a stamped kernel broke kclock_record's one-leader-per-block invariant");
  for (size_t i = 0; i < v.size(); i += 2) {
    if (v[i + 1] == 0ull || v[i] == ~0ull || v[i + 1] < v[i]) continue;
    const double us = (double)(v[i + 1] - v[i]) * 1e3 / rate_khz;
    *launches += 1;
    *total_us += us;
    if (max_us && us > *max_us) *max_us = us;
  }
  if (*launches != h->kclock_launches)
    return fail(MPPI_E_STATE, "mppi_kernel_clock_read: stamped slots (" + std::to_string(*launches) +
                                  ") != stamped launches (" + std::to_string(h->kclock_launches) + ")");
  return MPPI_OK;
}

int mppi_device_buffers(mppi_handle* h, void** dU, void** du0, void** dcosts) {
  if (!h) return fail(MPPI_E_ARG, "mppi_device_buffers: null handle");
  if (dU) *dU = h->d_U;
  if (du0) *du0 = h->d_u0;
  if (dcosts) *dcosts = h->d_costs;
  return MPPI_OK;
}

int mppi_get_U(mppi_handle* h, int B, float* U) {
  if (!h || !U || B < 1 || B > h->cfg.max_batch) return fail(MPPI_E_ARG, "mppi_get_U: bad argument");
  HIP_TRY(hipSetDevice(h->device));
  HIP_TRY(hipMemcpyAsync(U, h->d_U, (size_t)B * h->cfg.nu * h->cfg.H * 4, hipMemcpyDeviceToHost, h->stream));
  HIP_TRY(hipStreamSynchronize(h->stream));
  return MPPI_OK;
}

int mppi_set_U(mppi_handle* h, int B, const float* U) {
  if (!h || !U || B < 1 || B > h->cfg.max_batch) return fail(MPPI_E_ARG, "mppi_set_U: bad argument");
  HIP_TRY(hipSetDevice(h->device));
  HIP_TRY(hipMemcpyAsync(h->d_U, U, (size_t)B * h->cfg.nu * h->cfg.H * 4, hipMemcpyHostToDevice, h->stream));
  HIP_TRY(hipStreamSynchronize(h->stream));
  return MPPI_OK;
}

}  // extern "C"

// Validate one solve request against the handle.
static int check_solve(mppi_handle* h, int B, const mppi_io* io, int flags) {
  if (!h || !io) return fail(MPPI_E_ARG, "mppi_solve: null argument");
  const mppi_config& c = h->cfg;
  if (B < 1 || B > c.max_batch) return fail(MPPI_E_ARG, "mppi_solve: B out of range [1, max_batch]");
  if (h->dyn_kind == 0) return fail(MPPI_E_STATE, "mppi_solve: call mppi_load_dynamics first");
  if (h->cost_kind == 0) return fail(MPPI_E_STATE, "mppi_solve: call mppi_set_cost first");
  const bool dev = (flags & MPPI_FLAG_DEVICE) != 0;
  if (!io->x0) return fail(MPPI_E_ARG, "mppi_solve: x0 is required");
  if (!io->U && !(flags & MPPI_FLAG_RESIDENT_U)) return fail(MPPI_E_ARG, "mppi_solve: U is required unless MPPI_FLAG_RESIDENT_U");
  if (dev && (flags & MPPI_FLAG_COLMAJOR)) return fail(MPPI_E_ARG, "mppi_solve: MPPI_FLAG_COLMAJOR applies to host arrays only");
  if ((flags & MPPI_FLAG_ENV_STEP) && !dev) return fail(MPPI_E_ARG, "mppi_solve: MPPI_FLAG_ENV_STEP needs MPPI_FLAG_DEVICE");
  if (h->dyn_kind == MPPI_DYN_CARTPOLE && h->cost_kind != MPPI_COST_CARTPOLE && h->cost_kind != MPPI_COST_CARTPOLE_EST)
    return fail(MPPI_E_UNSUPPORTED, "cartpole dynamics take a cartpole cost (cartpole or cartpole_est)");
  if (h->dyn_kind == MPPI_DYN_CARTPOLE && (c.nx != 4 || c.nu != 1))
    return fail(MPPI_E_UNSUPPORTED, "cartpole dynamics need nx=4, nu=1");
  if ((h->dyn_kind == MPPI_DYN_MLP || h->dyn_kind == MPPI_DYN_CROSS_ATTN) && h->net.arch != kArchGeneric &&
      (c.nx > kMaxNx || c.nu > kMaxNu))
    return fail(MPPI_E_UNSUPPORTED, "learned dynamics: nx <= 64, nu <= 32");
  return MPPI_OK;
}

static hipError_t launch_rollout(mppi_handle* h, const SolveArgs& a, hipStream_t s) {
  if (h->dyn_kind == MPPI_DYN_CARTPOLE) return launch_cartpole_rollout(a, h->cart, nullptr, s);
  if (h->dyn_kind == MPPI_DYN_FEATURE_ATTN) return launch_fa_rollout(a, h->fa, s);
  return launch_fc_rollout(a, h->net, s);
}

// A graph launch leaves the next launch's first noise prefetched, generated with one counter value ahead.  When
// that noise will not be used (a plain solve comes next, or a re-capture for another batch/seed), the counter is
// stepped back so the next consumer draws exactly the key the prefetch took: the key sequence of any interleaving
// of plain solves and graph launches equals a loop of plain solves.
static hipError_t drop_prefetch(mppi_handle* h) {
  if (h->gen_pending) {  // the overlapped generator's launch (and its counter bump) precede anything on the stream
    const hipError_t e = hipStreamWaitEvent(h->stream, h->ev_gen, 0);
    if (e != hipSuccess) return e;
    h->gen_pending = false;
  }
  if (!h->prefetch_valid) return hipSuccess;
  h->prefetch_valid = false;
  return launch_seed_bump(h->d_seed_ctr, -1, h->stream);
}

// Graph mode (captured streams of solves): this solve's noise is already in `cur` (generated by the previous
// solve's reduce, or primed by mppi_graph_launch); this solve's reduce writes the next solve's into `next`.
struct NoiseStep {
  float* cur;
  float* next;
};

// Enqueue one solve on the handle's stream: inputs, noise, rollout, reduce (+ update, shift), env step, outputs.
// Synchronises only for host-side column-major staging. Capturable into a hipGraph in device mode.
static int enqueue_solve(mppi_handle* h, int B, const mppi_io* io, uint64_t seed, int flags, float* rec_x = nullptr,
                         float* rec_u = nullptr, const NoiseStep* ns = nullptr) {
  const mppi_config& c = h->cfg;
  const bool dev = (flags & MPPI_FLAG_DEVICE) != 0;
  const bool resident = (flags & MPPI_FLAG_RESIDENT_U) != 0;
  const bool colmajor = (flags & MPPI_FLAG_COLMAJOR) != 0;
  hipStream_t s = h->stream;
  const int nx = c.nx, nu = c.nu, H = c.H, K = c.K, Kp = h->Kp;
  const size_t rowsU = (size_t)B * nu * H;

  SolveArgs a;
  std::memset(&a, 0, sizeof(a));
  a.B = B;
  a.nx = nx;
  a.nu = nu;
  a.H = H;
  a.K = K;
  a.Kp = Kp;
  a.lambda = c.lambda;
  a.ctrl_clamp = c.ctrl_clamp;
  a.U_clamp = c.U_clamp;
  a.norm_eps = c.norm_eps;
  a.shift_fill = c.shift_fill;
  a.terminal_weight = c.terminal_weight;
  a.update_mode = c.update_mode;
  a.flags = flags;
  a.cost_kind = h->cost_kind;
  std::memcpy(a.ctx_default, h->cost_params, sizeof(a.ctx_default));
  a.noise = ns ? ns->cur : h->d_noise;
  a.costs = h->d_costs;
  a.dU = h->d_dU;
  a.weights = io->weights ? h->d_weights : nullptr;
  a.u0 = (dev && io->u0) ? io->u0 : h->d_u0;  // device mode: kernels write u0 straight to the caller
  a.status = h->d_status;
  a.tickets = h->d_tickets;
  a.seed_ctr = (flags & MPPI_FLAG_SEED_COUNTER) ? h->d_seed_ctr : nullptr;
  a.seed_bump = ns ? nullptr : a.seed_ctr;  // graph mode: reduce_kernel<GEN> advances the counter instead
  a.xout = nullptr;
  // launch clock: only solves that use the seed counter are stamped (bench.py's timed paths)
  a.kclock = (h->kclock && a.seed_ctr) ? h->d_kclock : nullptr;
  a.kclock_ctr = h->d_kclock ? h->d_kclock + 2 * (size_t)kClockSlots : nullptr;
  a.kclock_ticket = h->d_kclock ? reinterpret_cast<unsigned*>(h->d_kclock + 2 * (size_t)kClockSlots + 1) : nullptr;
  if (a.kclock && !h->capturing) h->kclock_launches += 1;  // graph replays count graph_n each (mppi_graph_launch)

  // ---- inputs
  if (dev) {
    a.x0 = io->x0;
    a.ctx = io->ctx;
    a.U = resident ? h->d_U : io->U;
    a.Umirror = (resident && io->U) ? io->U : nullptr;  // written by the update kernels themselves
  } else {
    HIP_TRY(hipMemcpyAsync(h->d_x0, io->x0, (size_t)B * nx * 4, hipMemcpyHostToDevice, s));
    a.x0 = h->d_x0;
    if (io->ctx) HIP_TRY(hipMemcpyAsync(h->d_ctx, io->ctx, (size_t)B * MPPI_CTX_MAX * 4, hipMemcpyHostToDevice, s));
    a.ctx = io->ctx ? h->d_ctx : nullptr;
    a.U = h->d_U;
    if (!resident) {
      const float* src = io->U;
      if (colmajor) {  // Julia U (nu,H) column-major -> [nu][H]
        h->staging.resize(rowsU);
        for (int b = 0; b < B; ++b)
          for (int u = 0; u < nu; ++u)
            for (int t = 0; t < H; ++t)
              h->staging[((size_t)b * nu + u) * H + t] = io->U[((size_t)b * H + t) * nu + u];
        src = h->staging.data();
      }
      HIP_TRY(hipMemcpyAsync(h->d_U, src, rowsU * 4, hipMemcpyHostToDevice, s));
      if (colmajor) HIP_TRY(hipStreamSynchronize(s));  // staging reused below
    }
  }

  // ---- a1: noise
  if (io->noise) {
    const float* src = io->noise;
    std::vector<float> tmp;
    if (colmajor) {  // Julia noise (nu,H,K) column-major -> [nu][H][K]
      tmp.resize(rowsU * K);
      for (int b = 0; b < B; ++b)
        for (int k = 0; k < K; ++k)
          for (int t = 0; t < H; ++t)
            for (int u = 0; u < nu; ++u)
              tmp[(((size_t)b * nu + u) * H + t) * K + k] = io->noise[(((size_t)b * K + k) * H + t) * nu + u];
      src = tmp.data();
    }
    if (K != Kp) HIP_TRY(hipMemsetAsync(h->d_noise, 0, rowsU * Kp * 4, s));
    HIP_TRY(hipMemcpy2DAsync(h->d_noise, (size_t)Kp * 4, src, (size_t)K * 4, (size_t)K * 4, rowsU,
                             dev ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, s));
    if (!tmp.empty()) HIP_TRY(hipStreamSynchronize(s));
  } else if (!ns) {
    HIP_TRY(timed(h, kNoise, [&] { return launch_noise(a.noise, B, nu, H, Kp, seed, a.seed_ctr, c.sigma, s); }));
  }

  // ---- a2-a6: rollout + cost; a7-a9: softmin + weighted-noise reduce + update + shift
  const NoiseGen gen{ns ? ns->next : nullptr, seed, c.sigma, h->d_gticket};
  const NoiseGen* pg = ns && ns->next ? &gen : nullptr;
  if (h->dyn_kind == MPPI_DYN_CARTPOLE) {  // one launch: the rollout blocks finish the solve (fused epilogue)
    a.part = h->d_part;
    HIP_TRY(timed(h, kRollout, [&] { return launch_cartpole_rollout(a, h->cart, pg, s); }));
    h->rollout_kernel = g_rollout_kernel;
  } else {
    HIP_TRY(timed(h, kRollout, [&] { return launch_rollout(h, a, s); }));
    h->rollout_kernel = g_rollout_kernel;
    HIP_TRY(timed(h, kReduce, [&] { return launch_reduce(a, pg, s); }));
  }

  // ---- env step: x0 <- f(x0, u0), the rollout kernel over one sample, one step, zero noise, U = u0, final
  // state written straight back to x0.  Kp = 16 makes it ONE 16-sample group (fc: one block; FA: one block;
  // cartpole: only wave 0 works), so every read of x0 precedes the single writer's store in program order or
  // behind the kernel's own barriers.
  if (flags & MPPI_FLAG_ENV_STEP) {
    SolveArgs e = a;
    e.K = 1;
    e.Kp = 16;
    e.H = 1;
    e.U = a.u0;  // [B][nu] == [B][nu][1]
    e.noise = h->d_env_noise;
    e.costs = h->d_env_costs;
    e.weights = nullptr;
    e.status = h->d_env_status;
    e.seed_ctr = nullptr;
    e.seed_bump = nullptr;
    e.part = nullptr;  // plain rollout (no fused epilogue)
    e.kclock = nullptr;
    e.terminal_weight = 0.0f;
    e.xout = const_cast<float*>(io->x0);
    if (rec_x) HIP_TRY(launch_record(io->x0, a.u0, rec_x, rec_u, B * nx, B * nu, s));
    HIP_TRY(launch_rollout(h, e, s));
  }

  // ---- outputs
  const hipMemcpyKind d2x = dev ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
  if (io->costs)
    HIP_TRY(hipMemcpy2DAsync(io->costs, (size_t)K * 4, h->d_costs, (size_t)Kp * 4, (size_t)K * 4, B, d2x, s));
  if (io->weights)
    HIP_TRY(hipMemcpy2DAsync(io->weights, (size_t)K * 4, h->d_weights, (size_t)Kp * 4, (size_t)K * 4, B, d2x, s));
  if (io->u0 && !dev) HIP_TRY(hipMemcpyAsync(io->u0, h->d_u0, (size_t)B * nu * 4, d2x, s));
  h->Uhost.clear();
  if (!dev && (!resident || io->U)) {  // (RESIDENT_U with a host io.U: a copy of the resident U)
    if (colmajor) {
      h->Uhost.resize(rowsU);
      HIP_TRY(hipMemcpyAsync(h->Uhost.data(), h->d_U, rowsU * 4, hipMemcpyDeviceToHost, s));
    } else {
      HIP_TRY(hipMemcpyAsync(io->U, h->d_U, rowsU * 4, hipMemcpyDeviceToHost, s));
    }
  }
  return MPPI_OK;
}

// The device status word (bit 0: some solve had no finite cost).  The fc/FA rollouts reset it per launch; the fused
// cartpole epilogue only sets it, so it is cleared here once read (sticky between reads).
static int read_status(mppi_handle* h, unsigned* st) {
  HIP_TRY(hipMemcpy(st, h->d_status, 4, hipMemcpyDeviceToHost));
  if (*st) HIP_TRY(hipMemset(h->d_status, 0, 4));
  return MPPI_OK;
}

// Wait for the stream, finish host-side layout conversion, report non-finite solves.
static int finish_solve(mppi_handle* h, int B, const mppi_io* io) {
  HIP_TRY(hipStreamSynchronize(h->stream));
  const int nu = h->cfg.nu, H = h->cfg.H;
  if (!h->Uhost.empty())
    for (int b = 0; b < B; ++b)
      for (int u = 0; u < nu; ++u)
        for (int t = 0; t < H; ++t) io->U[((size_t)b * H + t) * nu + u] = h->Uhost[((size_t)b * nu + u) * H + t];
  h->Uhost.clear();
  unsigned st = 0;
  if (const int rc = read_status(h, &st); rc != MPPI_OK) return rc;
  if (st & 1u) return fail(MPPI_E_NONFINITE, "mppi_solve: every sample of some solve had a non-finite cost");
  return MPPI_OK;
}

// The graph-stream noise double buffer (d_noise, d_noise2) and the generators' ticket, allocated on first use.
static int ensure_stream_buffers(mppi_handle* h) {
  const mppi_config& c = h->cfg;
  if (!h->d_noise2) {
    HIP_TRY(hipMalloc(&h->d_noise2, (size_t)c.max_batch * c.nu * c.H * (size_t)h->Kp * 4));
    HIP_TRY(hipMemset(h->d_noise2, 0, (size_t)c.max_batch * c.nu * c.H * (size_t)h->Kp * 4));  // K..Kp pads stay 0
  }
  if (!h->d_gticket) {
    HIP_TRY(hipMalloc(&h->d_gticket, 16));
    HIP_TRY(hipMemset(h->d_gticket, 0, 16));
  }
  return MPPI_OK;
}

// Make d_noise / d_noise2 [graph_parity] hold the noise of the next solve of batch B with key seed + counter: keep a
// matching prefetch, otherwise generate it now (one noise launch, counter bumped behind it).
static int prime_prefetch(mppi_handle* h, int B, uint64_t seed) {
  if (h->prefetch_valid && (h->prefetch_B != B || h->prefetch_seed != seed)) HIP_TRY(drop_prefetch(h));
  if (h->prefetch_valid) return MPPI_OK;
  const mppi_config& c = h->cfg;
  HIP_TRY(launch_noise(h->graph_parity ? h->d_noise2 : h->d_noise, B, c.nu, c.H, h->Kp, seed, h->d_seed_ctr, c.sigma,
                       h->stream));
  HIP_TRY(launch_seed_bump(h->d_seed_ctr, 1, h->stream));
  h->prefetch_valid = true;
  h->prefetch_B = B;
  h->prefetch_seed = seed;
  return MPPI_OK;
}

// MPPI_GEN_OVERLAP=1 (read per call; default 0, an A/B arm): chained solves generate the next solve's noise on a
// second, low-priority stream concurrently with this solve's rollout (noise_kernel + counter bump, the plain solves'
// exact keys), and reduce with the read-only reduce_kernel; default: the next noise comes out of reduce_kernel<GEN>
// after the rollout.  Same-box A/B (profiles/r04_ab_gen_overlap.log): config #4 at 64 solves 0.4795 / 0.4833 ->
// 0.4835 / 0.4732 ms per step (the rollout 360 -> 397 us: the generator's Philox VALU lands in the issue-bound
// rollout, where reduce_kernel<GEN> hides it under its HBM stream), 8 solves 0.1017 -> 0.1037, config #3 0.0530 ->
// 0.0611, config #2 0.0159 -> 0.0322 (the cross-stream event waits of a short step)
static bool gen_overlap() {
  const char* e = std::getenv("MPPI_GEN_OVERLAP");
  return e && e[0] == '1';
}

static int ensure_gen_stream(mppi_handle* h) {
  if (h->gstream) return MPPI_OK;
  int lo = 0, hi = 0;
  HIP_TRY(hipDeviceGetStreamPriorityRange(&lo, &hi));  // lo: the numerically greatest = lowest priority
  HIP_TRY(hipStreamCreateWithPriority(&h->gstream, hipStreamNonBlocking, lo));
  HIP_TRY(hipEventCreateWithFlags(&h->ev_gen, hipEventDisableTiming));
  HIP_TRY(hipEventCreateWithFlags(&h->ev_red, hipEventDisableTiming));
  return MPPI_OK;
}

// MPPI_FLAG_CHAIN: one solve of a graph stream, launched on the stream (rollout -> reduce_kernel<GEN>, or with
// gen_overlap the generator stream's noise launch beside the rollout, then the read-only reduce).  A graph launch pays
// a fixed gap at its boundary (~8.5 us on the box, rocprof trace) that back-to-back stream launches do not, so
// one-solve-per-step loops chain on the stream and multi-solve streams replay graphs.
static int chain_solve(mppi_handle* h, int B, const mppi_io* io, uint64_t seed, int flags) {
  if (!(flags & MPPI_FLAG_DEVICE)) return fail(MPPI_E_ARG, "mppi_solve: MPPI_FLAG_CHAIN needs MPPI_FLAG_DEVICE");
  if (io->noise) return fail(MPPI_E_ARG, "mppi_solve: MPPI_FLAG_CHAIN draws device noise (no injected noise)");
  flags |= MPPI_FLAG_SEED_COUNTER;
  if (const int rc = ensure_stream_buffers(h); rc != MPPI_OK) return rc;
  const bool overlap = gen_overlap() && !h->capturing;
  if (!overlap && h->gen_pending) {  // leaving overlap mode: order the solve stream behind the last generator launch
    HIP_TRY(hipStreamWaitEvent(h->stream, h->ev_gen, 0));
    h->gen_pending = false;
  }
  if (const int rc = prime_prefetch(h, B, seed); rc != MPPI_OK) return rc;
  float* buf[2] = {h->d_noise, h->d_noise2};
  if (!overlap) {
    const NoiseStep ns{buf[h->graph_parity], buf[h->graph_parity ^ 1]};
    const int rc = enqueue_solve(h, B, io, seed, flags, nullptr, nullptr, &ns);
    if (rc != MPPI_OK) return rc;
    h->graph_parity ^= 1;  // this solve's reduce prefetched the next one's noise (still key-valid for B, seed)
    if (flags & MPPI_FLAG_ASYNC) return MPPI_OK;
    return finish_solve(h, B, io);
  }
  if (const int rc = ensure_gen_stream(h); rc != MPPI_OK) return rc;
  const mppi_config& c = h->cfg;
  // this solve's noise (buf[p]) was written by the previous call's generator launch (or primed on the stream)
  if (h->gen_pending) HIP_TRY(hipStreamWaitEvent(h->stream, h->ev_gen, 0));
  // the next solve's noise into buf[p ^ 1], once the previous solve's reduce (which read buf[p ^ 1]) is done; the
  // generator stream alone reads and bumps the key counter from here on, in launch order
  HIP_TRY(hipEventRecord(h->ev_red, h->stream));  // = the previous reduce (everything enqueued so far)
  HIP_TRY(hipStreamWaitEvent(h->gstream, h->ev_red, 0));
  HIP_TRY(launch_noise(buf[h->graph_parity ^ 1], B, c.nu, c.H, h->Kp, seed, h->d_seed_ctr, c.sigma, h->gstream));
  HIP_TRY(launch_seed_bump(h->d_seed_ctr, 1, h->gstream));
  HIP_TRY(hipEventRecord(h->ev_gen, h->gstream));
  h->gen_pending = true;
  const NoiseStep ns{buf[h->graph_parity], nullptr};  // read-only reduce, no counter bump (the generator owns it)
  const int rc = enqueue_solve(h, B, io, seed, flags, nullptr, nullptr, &ns);
  if (rc != MPPI_OK) return rc;
  h->graph_parity ^= 1;  // the generator prefetched the next one's noise (key-valid for B, seed)
  if (flags & MPPI_FLAG_ASYNC) return MPPI_OK;
  return finish_solve(h, B, io);
}

// The split CA's two-product layer 1 (fc_common.h x3_l1_terms) as a CHECKED property of the loaded weights.  Before
// the first split-mode solve of a CrossAttention net the engine rolls the first solve's own states and U (up to
// kProbeB solves, kProbeK samples each, seeded device noise of the configured sigma, the configured horizon, cost and
// context) through the same routed kernel twice, with two and with three products on layer 1, and keeps the two-product
// form only if the costs agree within kX3ProbeTol (relative, every finite cost; a non-finite mismatch fails it).  Three
// products are within ~1.5e-6 of the fp32 oracle (profiles/r05_x3_error_budget.txt), so the difference measures the
// two-product form's own error on this net, these states and this horizon.  Runs once per loaded net, on the handle's
// stream, with its own buffers (no effect on the noise counter, the prefetched noise or U), before any graph capture.
// Horizons beyond kX3TwoTermMaxH keep three products without a probe (the error grows ~H^2); MPPI_X3_L1_TERMS forces.
// The same run decides the fp16 form (fc_common.h x3_f16_on): one more rollout of the same inputs through each kernel
// that runs the form -- fc_wave32_x3p_kernel (the large batches) and fc_rollout_kernel_x3h (the few-tiles shards),
// x3_route, whatever the probe's batch -- kept only if both are within kX3ProbeTol of the three-product costs
// (FcNet::x3_f16 = 1, x3_f16_err = the larger error), else not (-1).  The probe covers up to kProbeB of the first batch's solves at kProbeK samples
// each: the CA surrogate's dynamics do not depend on the controls (its action encoder never reaches the output), so
// the form's error is one number per state -- more states, not more samples, find the worst.
static int x3_probe(mppi_handle* h, int B, const mppi_io* io, int flags) {
  if (h->dyn_kind != MPPI_DYN_CROSS_ATTN || h->cfg.precision != MPPI_PREC_BF16X3 || h->net.arch != kArchCA ||
      h->net.x3_l1 != 0)
    return MPPI_OK;
  const mppi_config& c = h->cfg;
  if (x3_l1_env() || c.H > kX3TwoTermMaxH) {
    h->net.x3_l1 = c.H > kX3TwoTermMaxH ? 3 : x3_l1_env();
    h->net.x3_l1_err = -1.0f;
    h->net.x3_f16 = -1;  // (MPPI_X3_F16=1 still forces it: x3_f16_on)
    h->net.x3_f16_err = -1.0f;
    return MPPI_OK;
  }
  const bool f16 = h->net.w32f16_off >= 0;
  constexpr int kProbeB = 64, kProbeK = 64;
  const int Bp = B < kProbeB ? B : kProbeB, Kpr = h->Kp < kProbeK ? h->Kp : kProbeK;
  const bool dev = (flags & MPPI_FLAG_DEVICE) != 0, colmajor = (flags & MPPI_FLAG_COLMAJOR) != 0;
  const size_t nU = (size_t)Bp * c.nu * c.H, nN = nU * Kpr, nC = (size_t)Bp * Kpr;
  char* buf = nullptr;
  const size_t bytes = (nN + nU + 4 * nC + (size_t)Bp * c.nx + (size_t)Bp * MPPI_CTX_MAX + 16) * 4;
  HIP_TRY(hipMalloc(&buf, bytes));
  float* p_noise = reinterpret_cast<float*>(buf);
  float* p_U = p_noise + nN;
  float* p_c2 = p_U + nU;
  float* p_c3 = p_c2 + nC;
  float* p_c1 = p_c3 + nC;
  float* p_ch = p_c1 + nC;  // the fp16 form on fc_rollout_kernel_x3h
  float* p_x0 = p_ch + nC;
  float* p_ctx = p_x0 + (size_t)Bp * c.nx;
  unsigned* p_st = reinterpret_cast<unsigned*>(p_ctx + (size_t)Bp * MPPI_CTX_MAX);
  hipStream_t s = h->stream;
  std::vector<float> hc1(nC), hc2(nC), hc3(nC), hch(nC), stage;
  FcArgs fh{};  // (only fc_x3h_wanted's fields: the shards' kernel can run this net's fp16 form)
  fh.w_off[1] = h->net.w_off[1];
  fh.ln_n = h->net.ln_n;
  fh.wmf16_0_off = h->net.wmf16_0_off;
  fh.wmf16_0b_off = h->net.wmf16_0b_off;
  fh.wmf16_off = h->net.wmf16_off;
  fh.x3_f16 = 1;
  bool x3h = false;
  auto run = [&]() -> hipError_t {
    const hipMemcpyKind k = dev ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
    hipError_t e = hipMemcpyAsync(p_x0, io->x0, (size_t)Bp * c.nx * 4, k, s);
    const float* U = io->U;
    hipMemcpyKind ku = k;
    if (flags & MPPI_FLAG_RESIDENT_U) {  // the handle's resident U is the input
      U = h->d_U;
      ku = hipMemcpyDeviceToDevice;
    } else if (colmajor) {  // Julia U (nu,H) column-major -> [nu][H]
      stage.resize(nU);
      for (int b = 0; b < Bp; ++b)
        for (int u = 0; u < c.nu; ++u)
          for (int t = 0; t < c.H; ++t)
            stage[((size_t)b * c.nu + u) * c.H + t] = io->U[((size_t)b * c.H + t) * c.nu + u];
      U = stage.data();
    }
    if (e == hipSuccess) e = hipMemcpyAsync(p_U, U, nU * 4, ku, s);
    if (e == hipSuccess && io->ctx) e = hipMemcpyAsync(p_ctx, io->ctx, (size_t)Bp * MPPI_CTX_MAX * 4, k, s);
    if (e == hipSuccess) e = launch_noise(p_noise, Bp, c.nu, c.H, Kpr, 0x5EEDC0DEull, nullptr, c.sigma, s);
    SolveArgs a;
    std::memset(&a, 0, sizeof(a));
    a.B = Bp;
    a.nx = c.nx;
    a.nu = c.nu;
    a.H = c.H;
    a.K = Kpr < c.K ? Kpr : c.K;
    a.Kp = Kpr;
    a.lambda = c.lambda;
    a.ctrl_clamp = c.ctrl_clamp;
    a.terminal_weight = c.terminal_weight;
    a.cost_kind = h->cost_kind;
    std::memcpy(a.ctx_default, h->cost_params, sizeof(a.ctx_default));
    a.x0 = p_x0;
    a.U = p_U;
    a.noise = p_noise;
    a.ctx = io->ctx ? p_ctx : nullptr;
    a.status = p_st;
    FcNet n = h->net;
    n.x3_f16 = -1;
    for (int terms : {2, 3}) {
      n.x3_l1 = terms;
      a.costs = terms == 2 ? p_c2 : p_c3;
      if (e == hipSuccess) e = launch_fc_rollout(a, n, s);
    }
    if (f16) {  // the fp16 form on fc_wave32_x3p_kernel
      n.x3_route = 1;
      n.x3_f16 = 1;
      a.costs = p_c1;
      if (e == hipSuccess) e = launch_fc_rollout(a, n, s);
      if (e == hipSuccess) e = hipMemcpyAsync(hc1.data(), p_c1, nC * 4, hipMemcpyDeviceToHost, s);
      a.costs = p_ch;
      x3h = fc_x3h_wanted(a, fh);
      if (x3h) {  // ... and on fc_rollout_kernel_x3h
        n.x3_route = 2;
        if (e == hipSuccess) e = launch_fc_rollout(a, n, s);
        if (e == hipSuccess) e = hipMemcpyAsync(hch.data(), p_ch, nC * 4, hipMemcpyDeviceToHost, s);
      }
    }
    if (e == hipSuccess) e = hipMemcpyAsync(hc2.data(), p_c2, nC * 4, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipMemcpyAsync(hc3.data(), p_c3, nC * 4, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    return e;
  };
  const hipError_t e = run();
  (void)hipFree(buf);
  if (e != hipSuccess) return fail(MPPI_E_HIP, std::string("x3 layer-1 probe: ") + hipGetErrorString(e));
  const int Kv = Kpr < c.K ? Kpr : c.K;
  auto diff = [&](const std::vector<float>& hc) {  // max relative difference to three products (inf: a finiteness mismatch)
    double worst = 0.0;
    for (int b = 0; b < Bp; ++b)
      for (int k = 0; k < Kv; ++k) {
        const float v = hc[(size_t)b * Kpr + k], v3 = hc3[(size_t)b * Kpr + k];
        if (!std::isfinite(v3) && !std::isfinite(v)) continue;
        if (!std::isfinite(v) || !std::isfinite(v3)) return (double)INFINITY;
        const double d = std::fabs((double)v - v3) / std::fmax(std::fabs((double)v3), 1e-30);
        worst = d > worst ? d : worst;
      }
    return worst;
  };
  const double w2 = diff(hc2);
  h->net.x3_l1 = w2 <= kX3ProbeTol ? 2 : 3;
  h->net.x3_l1_err = (float)w2;
  const double w1 = f16 ? std::fmax(diff(hc1), x3h ? diff(hch) : 0.0) : (double)INFINITY;
  h->net.x3_f16 = w1 <= kX3ProbeTol ? 1 : -1;
  h->net.x3_f16_err = f16 ? (float)w1 : -1.0f;
  return MPPI_OK;
}

extern "C" {

int mppi_x3_layer1(mppi_handle* h, int* products, float* probe_rel_err) {
  if (!h) return fail(MPPI_E_ARG, "mppi_x3_layer1: null handle");
  const bool split_ca = h->dyn_kind == MPPI_DYN_CROSS_ATTN && h->cfg.precision == MPPI_PREC_BF16X3 &&
                        h->net.arch == kArchCA;
  if (products) *products = split_ca && h->net.x3_l1 ? x3_l1_terms(h->cfg.H, h->net.x3_l1) : 0;
  if (probe_rel_err) *probe_rel_err = split_ca ? h->net.x3_l1_err : -1.0f;
  return MPPI_OK;
}

int mppi_x3_f16(mppi_handle* h, int* on, float* probe_rel_err) {
  if (!h) return fail(MPPI_E_ARG, "mppi_x3_f16: null handle");
  const bool split_ca = h->dyn_kind == MPPI_DYN_CROSS_ATTN && h->cfg.precision == MPPI_PREC_BF16X3 &&
                        h->net.arch == kArchCA;
  if (on)
    *on = split_ca && x3_f16_on(h->cfg.H, h->net.x3_f16, h->net.w32f16_off)
              ? (x3_f16_l2x1(h->net.x3_f16) ? 2 : 1)
              : 0;
  if (probe_rel_err) *probe_rel_err = split_ca ? h->net.x3_f16_err : -1.0f;
  return MPPI_OK;
}

const char* mppi_rollout_kernel(mppi_handle* h) { return h ? h->rollout_kernel : ""; }

int mppi_solve_ex(mppi_handle* h, int B, const mppi_io* io, uint64_t seed, int flags) {
  int rc = check_solve(h, B, io, flags);
  if (rc != MPPI_OK) return rc;
  HIP_TRY(hipSetDevice(h->device));
  if ((rc = x3_probe(h, B, io, flags)) != MPPI_OK) return rc;
  if (flags & MPPI_FLAG_CHAIN) return chain_solve(h, B, io, seed, flags);
  HIP_TRY(drop_prefetch(h));  // a plain solve generates its own noise into d_noise
  rc = enqueue_solve(h, B, io, seed, flags);
  if (rc != MPPI_OK) return rc;
  if ((flags & MPPI_FLAG_DEVICE) && (flags & MPPI_FLAG_ASYNC)) return MPPI_OK;
  return finish_solve(h, B, io);
}

int mppi_graph_capture(mppi_handle* h, int B, const mppi_io* io, uint64_t seed, int flags, int n_solves) {
  return mppi_graph_capture_traj(h, B, io, seed, flags, n_solves, nullptr, nullptr);
}

int mppi_graph_capture_traj(mppi_handle* h, int B, const mppi_io* io, uint64_t seed, int flags, int n_solves,
                            float* traj_x, float* traj_u) {
  if (n_solves < 1) return fail(MPPI_E_ARG, "mppi_graph_capture: n_solves must be >= 1");
  if ((traj_x != nullptr) != (traj_u != nullptr)) return fail(MPPI_E_ARG, "mppi_graph_capture: traj_x and traj_u go together");
  if (traj_x && !(flags & MPPI_FLAG_ENV_STEP))
    return fail(MPPI_E_ARG, "mppi_graph_capture: trajectory logging needs MPPI_FLAG_ENV_STEP");
  if (!(flags & MPPI_FLAG_DEVICE)) return fail(MPPI_E_ARG, "mppi_graph_capture: device pointers (MPPI_FLAG_DEVICE) required");
  if (io && io->noise) return fail(MPPI_E_ARG, "mppi_graph_capture: injected noise is not replayable; use device noise");
  flags = (flags | MPPI_FLAG_SEED_COUNTER | MPPI_FLAG_ASYNC) & ~MPPI_FLAG_COLMAJOR;
  int rc = check_solve(h, B, io, flags);
  if (rc != MPPI_OK) return rc;
  HIP_TRY(hipSetDevice(h->device));
  if ((rc = x3_probe(h, B, io, flags)) != MPPI_OK) return rc;  // before the capture: it synchronises the stream
  for (hipGraphExec_t& g : h->graph_exec)
    if (g) {
      HIP_TRY(hipGraphExecDestroy(g));
      g = nullptr;
    }
  // a prefetched noise stays valid for a graph of the same batch and seed (checked again at launch)
  if (h->prefetch_valid && (B != h->prefetch_B || seed != h->prefetch_seed)) HIP_TRY(drop_prefetch(h));
  const mppi_config& c = h->cfg;
  if (const int e = ensure_stream_buffers(h); e != MPPI_OK) return e;
  float* buf[2] = {h->d_noise, h->d_noise2};
  const bool prof = h->prof;
  h->prof = false;  // no event nodes inside the graph
  h->capturing = true;
  // exec p starts from noise buffer p (an odd stream flips the parity every launch; a re-capture keeps the parity
  // of a valid prefetch)
  for (int p = 0; p < 2 && rc == MPPI_OK; ++p) {
    HIP_TRY(hipStreamBeginCapture(h->stream, hipStreamCaptureModeRelaxed));
    for (int i = 0; i < n_solves && rc == MPPI_OK; ++i) {
      const NoiseStep ns{buf[(p + i) % 2], buf[(p + i + 1) % 2]};
      rc = enqueue_solve(h, B, io, seed, flags, traj_x ? traj_x + (size_t)i * B * c.nx : nullptr,
                         traj_u ? traj_u + (size_t)i * B * c.nu : nullptr, &ns);
    }
    hipGraph_t g = nullptr;
    const hipError_t ec = hipStreamEndCapture(h->stream, &g);
    if (rc != MPPI_OK || ec != hipSuccess) {
      if (g) (void)hipGraphDestroy(g);
      h->prof = prof;
      h->capturing = false;
      if (rc != MPPI_OK) return rc;
      return fail(MPPI_E_HIP, std::string("mppi_graph_capture: ") + hipGetErrorString(ec));
    }
    const hipError_t ei = hipGraphInstantiate(&h->graph_exec[p], g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    if (ei != hipSuccess) {
      h->graph_exec[p] = nullptr;
      h->prof = prof;
      h->capturing = false;
      return fail(MPPI_E_HIP, std::string("mppi_graph_capture: instantiate: ") + hipGetErrorString(ei));
    }
  }
  h->prof = prof;
  h->capturing = false;
  h->graph_kclock = h->kclock;
  h->graph_B = B;
  h->graph_n = n_solves;
  h->graph_seed = seed;
  return MPPI_OK;
}

int mppi_graph_launch(mppi_handle* h, int sync) {
  if (!h) return fail(MPPI_E_ARG, "mppi_graph_launch: null handle");
  if (!h->graph_exec[0] || !h->graph_exec[1])
    return fail(MPPI_E_STATE, "mppi_graph_launch: call mppi_graph_capture first");
  HIP_TRY(hipSetDevice(h->device));
  if (h->gen_pending) {  // chained solves with the overlapped generator came before: its noise and bump first
    HIP_TRY(hipStreamWaitEvent(h->stream, h->ev_gen, 0));
    h->gen_pending = false;
  }
  // first launch (or after plain solves / a counter reset / chained solves of another batch): generate the noise
  if (const int rc = prime_prefetch(h, h->graph_B, h->graph_seed); rc != MPPI_OK) return rc;
  HIP_TRY(hipGraphLaunch(h->graph_exec[h->graph_parity], h->stream));
  if (h->graph_kclock) h->kclock_launches += h->graph_n;
  h->graph_parity = (h->graph_parity + h->graph_n) % 2;  // the launch prefetched the next one's first noise
  if (!sync) return MPPI_OK;
  HIP_TRY(hipStreamSynchronize(h->stream));
  unsigned st = 0;
  if (const int rc = read_status(h, &st); rc != MPPI_OK) return rc;
  if (st & 1u) return fail(MPPI_E_NONFINITE, "mppi_graph_launch: every sample of some solve had a non-finite cost");
  return MPPI_OK;
}

int mppi_set_seed_counter(mppi_handle* h, uint64_t value) {
  if (!h) return fail(MPPI_E_ARG, "mppi_set_seed_counter: null handle");
  HIP_TRY(hipSetDevice(h->device));
  if (h->gen_pending) {  // the generator's last bump lands before the new value
    HIP_TRY(hipStreamWaitEvent(h->stream, h->ev_gen, 0));
    h->gen_pending = false;
  }
  HIP_TRY(hipMemcpyAsync(h->d_seed_ctr, &value, 8, hipMemcpyHostToDevice, h->stream));
  HIP_TRY(hipStreamSynchronize(h->stream));
  h->prefetch_valid = false;  // a prefetched noise used the old counter
  return MPPI_OK;
}

int mppi_get_seed_counter(mppi_handle* h, uint64_t* value) {
  if (!h || !value) return fail(MPPI_E_ARG, "mppi_get_seed_counter: null argument");
  HIP_TRY(hipSetDevice(h->device));
  if (h->gen_pending) {  // the overlapped generator's bump is part of the counter's value
    HIP_TRY(hipStreamWaitEvent(h->stream, h->ev_gen, 0));
    h->gen_pending = false;
  }
  uint64_t v = 0;
  HIP_TRY(hipMemcpyAsync(&v, h->d_seed_ctr, 8, hipMemcpyDeviceToHost, h->stream));
  HIP_TRY(hipStreamSynchronize(h->stream));
  // the LOGICAL counter: the key the next solve draws.  After chained solves or a graph launch the next solve's noise
  // is already prefetched and the device counter already advanced past its key (drop_prefetch steps it back for the
  // same reason), so mppi_set_seed_counter(value) -- which drops any prefetch -- resumes the stream exactly
  *value = h->prefetch_valid ? v - 1 : v;
  return MPPI_OK;
}

int mppi_solve(mppi_handle* h, int B, const float* x0, float* U, const float* noise, uint64_t seed, float* costs_out,
               float* u0_out, int flags) {
  mppi_io io;
  std::memset(&io, 0, sizeof(io));
  io.x0 = x0;
  io.U = U;
  io.noise = noise;
  io.costs = costs_out;
  io.u0 = u0_out;
  return mppi_solve_ex(h, B, &io, seed, flags);
}

}  // extern "C"
