/*
 * mppi.h — C-ABI of the MI355X-native MPPI solve engine (libmppi_hip.so).
 *
 * One call = one MPPI solve (reference "mppi_step"): sample -> rollout -> cost ->
 * softmin weight -> weighted-noise reduce -> U update [-> receding-horizon shift],
 * batched over B independent solves (different initial states / contexts).
 *
 * Every entry point replaces a reference function on the hot path (paths relative to
 * the reference repository SheffieldWang616/Humanoid_MPPI-RL):
 *
 *   mppi_solve / mppi_solve_ex
 *       src/cartpole_mppi.py:88-98        mppi_step(model, data)         (numpy, additive update)
 *       src/cartpole_mppi.py:59-85        rollout(model, data, U, noise) (costs_out)
 *       src/cartpole_mppi.py:101-106      mppi_controller (flag MPPI_FLAG_SHIFT, u0_out)
 *       src/mppi.jl:64-99                 rollout / mppi_update!          (clamp, +1e-10, zero fill)
 *       src/Humanoid_mppi_v3.jl:128-179   rollout / mppi_step! / mppi_controller!
 *       src/cartpole_mppi_estimator.py:61-151, src/quadruped_mppi_estimator.py:58-102
 *                                         learned-dynamics rollouts, replace-mode update
 *   mppi_load_dynamics
 *       mujoco.mj_step on models/cartpole.xml  (analytic cartpole, MPPI_DYN_CARTPOLE)
 *       learning/model.py:6-46  MLPStatePredictor              (MPPI_DYN_MLP)
 *       learning/model.py:157-202 CrossAttentionStatePredictor (MPPI_DYN_CROSS_ATTN)
 *       learning/model.py:48-153 FeatureAttentionStatePredictor (MPPI_DYN_FEATURE_ATTN), the net of
 *                                src/cartpole_mppi_estimator.py:28-33, src/quadruped_mppi_estimator.py:24-35
 *   mppi_set_cost
 *       src/cartpole_mppi.py:44-53, src/cartpole_mppi_estimator.py:46-55,
 *       src/Humanoid_mppi_v3.jl:27-121, src/mppi.jl:18-62, src/quadruped_mppi_estimator.py:48-55
 *   mppi_get_U / mppi_set_U
 *       the module-global U_global (src/cartpole_mppi.py:56, src/Humanoid_mppi_v3.jl:124)
 *
 * Layout (default = numpy C order, k fastest = state-major on device):
 *   x0     [B][nx]            U      [B][nu][H]        noise [B][nu][H][K]
 *   costs  [B][K]             weights[B][K]            u0    [B][nu]
 *   ctx    [B][MPPI_CTX_MAX]  per-solve cost context (humanoid real-env terms)
 * MPPI_FLAG_COLMAJOR selects Julia Array layouts instead: U (nu,H) column-major = [B][H][nu],
 * noise (nu,H,K) column-major = [B][K][H][nu].
 *
 * Ownership: host buffers are borrowed for the duration of the call. The library owns all
 * device buffers, weights and RNG state. A handle is bound to one device and one stream and
 * is NOT thread-safe: use one handle per host thread.
 *
 * Errors: 0 = OK, negative = error (see MPPI_E_*). Never throws or aborts across the ABI.
 * mppi_last_error() returns a thread-local message for the last failing call.
 */
#ifndef MPPI_H_
#define MPPI_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI history:
 *   1  round 1 (first boundary)
 *   2  MPPI_FLAG_CHAIN; mppi_kernel_clock / mppi_kernel_clock_read; MPPI_COST_HUMANOID_V1; preset "quad_collect_py"
 *      removed.  BEHAVIOUR CHANGE: with MPPI_FLAG_RESIDENT_U a non-NULL io.U now RECEIVES the updated U on every
 *      solve (device mode: written by the update kernel itself); version 1 ignored io.U in device mode.
 *   3  mppi_x3_layer1 (the split CA's layer-1 probe), mppi_rollout_kernel.  BEHAVIOUR CHANGE: mppi_get_seed_counter
 *      returns the LOGICAL counter (the key the next solve draws) also after chained solves and graph launches,
 *      whose prefetched noise had already advanced the device counter by one.
 *   4  mppi_x3_f16.  BEHAVIOUR CHANGE: MPPI_PREC_BF16X3 CrossAttention solves run the fp16 form when the engine's
 *      probe of the loaded weights allows it (below). */
#define MPPI_ABI_VERSION 4

/* ---- status codes ---- */
#define MPPI_OK 0
#define MPPI_E_ARG (-1)         /* bad argument / shape                          */
#define MPPI_E_HIP (-2)         /* HIP runtime error                             */
#define MPPI_E_UNSUPPORTED (-3) /* dynamics/cost/shape combination not built     */
#define MPPI_E_NONFINITE (-4)   /* every sample of some solve had a non-finite cost */
#define MPPI_E_STATE (-5)       /* call order (e.g. solve before load_dynamics)  */

/* ---- dynamics kinds (mppi_load_dynamics) ---- */
#define MPPI_DYN_CARTPOLE 1   /* analytic restatement of mj_step on models/cartpole.xml   */
#define MPPI_DYN_MLP 2        /* learning/model.py:6-46, x+ = x + net([x,u])             */
#define MPPI_DYN_CROSS_ATTN 3 /* learning/model.py:157-202, x+ = x + net([x,u])          */
#define MPPI_DYN_FEATURE_ATTN 4 /* learning/model.py:48-153, x+ = x + net([x,u]); 4 or 8 heads, hidden 64/128/512,
                                  up to 8 layers and 80 tokens                                              */

/* ---- cost kinds (mppi_set_cost) ---- */
#define MPPI_COST_CARTPOLE 1     /* src/cartpole_mppi.py:44-53                          */
#define MPPI_COST_CARTPOLE_EST 2 /* src/cartpole_mppi_estimator.py:46-55                */
#define MPPI_COST_HUMANOID_V3 3  /* src/Humanoid_mppi_v3.jl:27-121 (+ per-solve ctx)    */
#define MPPI_COST_QUAD_JL 4      /* src/mppi.jl:18-62                                   */
#define MPPI_COST_QUAD_EST 5     /* src/quadruped_mppi_estimator.py:48-55               */
#define MPPI_COST_HUMANOID_V1 6  /* src/Humanoid_mppi.jl:31-121 (+ per-solve ctx; the swing foot follows the
                                    rollout step t, :76-87)                             */

/* ---- update modes ---- */
#define MPPI_UPDATE_ADD 0     /* U += sum_k w_k eps_k   (cartpole_mppi.py:96-98)                   */
#define MPPI_UPDATE_REPLACE 1 /* U  = sum_k w_k eps_k   (cartpole_mppi_estimator.py:141-143)       */

/* ---- precision of learned-dynamics rollouts ---- */
#define MPPI_PREC_FP32 0 /* exact-f32 MFMA (v_mfma_f32_16x16x4_f32); fc nets: every wave's fp32 weight fragments
                            held in registers for the whole horizon (one wave per SIMD); FA nets: streamed from L2 */
#define MPPI_PREC_BF16 1 /* bf16 MFMA (v_mfma_f32_16x16x32_bf16 or v_mfma_f32_32x32x16_bf16 by kernel), weights in
                            registers or LDS, fp32 state / accumulate / cost / reduce                           */
#define MPPI_PREC_BF16X3 2 /* fp32-accurate split bf16 (MLP and CrossAttention nets of the register-resident shapes):
                              every weight and activation as a bf16 hi + lo pair, W a = W_hi a_hi + W_hi a_lo +
                              W_lo a_hi on bf16 MFMAs (16x16x32 or 32x32x16 by kernel; fp32 accumulate), ~2^-16
                              relative per product.  EXCEPTION, the CrossAttention net's layer 1 (256 -> 128): two
                              products (W_hi a_hi + W_lo a_hi, the W_hi a_lo term dropped) when the engine's probe of
                              the loaded weights allows it -- before the first solve it rolls the first solve's
                              states through both forms and keeps two products only if every cost agrees within
                              7.5e-5 relative (3/4 of the fp32-accurate bar) and H <= 64; mppi_x3_layer1 reports the
                              decision.  Env MPPI_X3_L1_TERMS=3 (=2) forces three (two) products without a probe.
                              SECOND EXCEPTION, the fp16 form: layer 1 as ONE fp16 product (fp16 W1 and
                              activations), layer 0 and the LayerNorm statistic as two (fp16 W hi + lo against one
                              fp16 operand) and the last layer as two too, fp32 accumulate, when the same probe finds
                              it within 7.5e-5 of three products (H <= 64); mppi_x3_f16 reports it.  Env
                              MPPI_X3_F16=0 (=1) forces the form off (on) without a probe; MPPI_X3_F16_L2=1 opts into
                              a one-product last layer (faster, NOT fp32-accurate on every state). */

/* ---- solve flags ---- */
#define MPPI_FLAG_SHIFT 0x1        /* controller step: u0_out = U[:,0], shift U left, fill last  */
#define MPPI_FLAG_COLMAJOR 0x2     /* host arrays in Julia column-major layout                   */
#define MPPI_FLAG_DEVICE 0x4       /* all pointers in mppi_io are device pointers; no H2D/D2H    */
#define MPPI_FLAG_ASYNC 0x8        /* with MPPI_FLAG_DEVICE: return without synchronising stream */
#define MPPI_FLAG_U0_BEFORE 0x10   /* u0_out = U[:,0] BEFORE the update (quadruped_datacollection.py:170) */
#define MPPI_FLAG_RESIDENT_U 0x20  /* use/keep the handle-resident U (warm start); io.U may be NULL, else it receives
                                      a copy of the updated U (device mode: written by the update kernel itself, so a
                                      per-step snapshot for a gather costs no copy launch) */
#define MPPI_FLAG_ENV_STEP 0x40    /* with MPPI_FLAG_DEVICE: after the update, advance io.x0 IN PLACE by one step of
                                      the loaded dynamics with u0 (x0 <- f(x0, u0)): the on-device stand-in for the
                                      control loop's mujoco.mj_step (src/cartpole_mppi_estimator.py:158-162) */
#define MPPI_FLAG_SEED_COUNTER 0x80 /* noise key = seed + a per-handle device counter that every solve advances,
                                       so replays of a captured graph draw fresh noise */
#define MPPI_FLAG_CHAIN 0x100       /* with MPPI_FLAG_DEVICE (MPPI_FLAG_SEED_COUNTER implied): a chained solve, the
                                       stream-launched form of a graph stream -- it uses the noise the previous
                                       chained solve (or graph launch) prefetched and prefetches the next solve's
                                       inside its reduce (env MPPI_GEN_OVERLAP=1, an A/B arm: on a second,
                                       low-priority stream concurrently with this solve's rollout); bitwise equal to
                                       plain counter solves either way.  Injected noise and MPPI_FLAG_COLMAJOR are
                                       not allowed */

#define MPPI_CTX_MAX 8 /* floats of per-solve cost context */

typedef struct mppi_config {
  int32_t nx;            /* state dim (qpos+qvel)                                       */
  int32_t nu;            /* control dim                                                 */
  int32_t H;             /* horizon (reference T / H)                                   */
  int32_t K;             /* samples (any K >= 1; padded internally, pad lanes masked)   */
  int32_t max_batch;     /* max independent solves B per call                           */
  float lambda;          /* softmin temperature                                         */
  float sigma;           /* noise std (device Philox noise only)                        */
  float ctrl_clamp;      /* >0: clamp U+eps to +-ctrl_clamp before dynamics AND cost (mppi.jl:74) */
  float U_clamp;         /* >0: clamp U after the update (mppi.jl:93)                   */
  float norm_eps;        /* added to sum(w) (mppi.jl:89: 1e-10)                         */
  float shift_fill;      /* last column after shift = shift_fill * previous last (0.1 or 0) */
  float terminal_weight; /* terminal = terminal_weight * running(x_H, u=0); 0 disables  */
  int32_t update_mode;   /* MPPI_UPDATE_ADD / MPPI_UPDATE_REPLACE                       */
  int32_t precision;     /* MPPI_PREC_*  (learned dynamics only)                        */
  int32_t reserved[4];
} mppi_config;

typedef struct mppi_io {
  const float* x0;    /* [B][nx]                                  */
  float* U;           /* [B][nu][H] in/out; with RESIDENT_U: NULL or out only (a copy of the resident U) */
  const float* noise; /* NULL => device Philox N(0, sigma^2); else [B][nu][H][K] (already scaled) */
  float* costs;       /* NULL or [B][K] out                        */
  float* weights;     /* NULL or [B][K] out (normalised softmin)   */
  float* u0;          /* NULL or [B][nu] out                       */
  const float* ctx;   /* NULL or [B][MPPI_CTX_MAX] per-solve cost context */
} mppi_io;

typedef struct mppi_handle mppi_handle;

/* Fill *cfg with the reference constants of a named preset:
 * "cartpole_py", "cartpole_jl", "cartpole_collect", "quad_mppi_jl", "humanoid_v3", "humanoid_v1",
 * "humanoid_collect_v2", "cartpole_est", "quad_est".  (src/quadruped_datacollection.py has no preset: its cost
 * reads the rollout's simulation time and weighs each actuator differently, and it clips to the Go1's per-actuator
 * ctrlrange; DESIGN.md §7.  Its apply-before-update convention is MPPI_FLAG_U0_BEFORE.) */
int mppi_preset(const char* name, mppi_config* cfg);

int mppi_create(const mppi_config* cfg, int device, mppi_handle** out);
void mppi_destroy(mppi_handle* h);

/* Binary blob format for learned dynamics: see DESIGN.md "weight blob". For
 * MPPI_DYN_CARTPOLE blob may be NULL (models/cartpole.xml constants) or 10 floats. */
int mppi_load_dynamics(mppi_handle* h, int kind, const void* blob, size_t nbytes);

/* params: cost-kind specific floats (may be NULL => reference defaults). */
int mppi_set_cost(mppi_handle* h, int kind, const float* params, int nparams);

/* Survey 8(b) signature: plain pointers, host memory unless MPPI_FLAG_DEVICE. */
int mppi_solve(mppi_handle* h, int B, const float* x0, float* U, const float* noise, uint64_t seed,
               float* costs_out, float* u0_out, int flags);

/* Extended form: every optional output + per-solve context. */
int mppi_solve_ex(mppi_handle* h, int B, const mppi_io* io, uint64_t seed, int flags);

/* Receding-horizon stream: record n_solves chained solves (device pointers, MPPI_FLAG_DEVICE
 * required; MPPI_FLAG_SEED_COUNTER implied) into a hipGraph on the handle's stream, then replay the whole chain
 * with one launch. With MPPI_FLAG_SHIFT | MPPI_FLAG_ENV_STEP each solve warm-starts from the shifted U and the
 * state advanced by the previous one: the reference's controller loop without host round trips.
 * mppi_graph_launch(h, sync): sync != 0 waits and reports MPPI_E_NONFINITE like mppi_solve. */
int mppi_graph_capture(mppi_handle* h, int B, const mppi_io* io, uint64_t seed, int flags, int n_solves);
int mppi_graph_launch(mppi_handle* h, int sync);
/* As mppi_graph_capture, with trajectory logging (needs MPPI_FLAG_ENV_STEP): solve i's env step records the
 * state it starts from and the control it applies, traj_x[i][B][nx] and traj_u[i][B][nu] (device memory) --
 * the (state, action) rows of src/Humanoid_datacollection_v2.jl:70-81 log_data! (mppi_hip.trajectory writes
 * them in the reference's CSV layout for learning/data_loader.py). */
int mppi_graph_capture_traj(mppi_handle* h, int B, const mppi_io* io, uint64_t seed, int flags, int n_solves,
                            float* traj_x, float* traj_u);
/* Device noise-key counter (MPPI_FLAG_SEED_COUNTER), e.g. to replay a stream from its start; get waits for the
 * handle's stream and returns the key the NEXT solve will draw (every enqueued solve has advanced it; a noise already
 * prefetched by chained solves or a graph launch is accounted for), so saving it with mppi_get_U and restoring both
 * (set drops any prefetch) continues a plain, chained or graph stream with the noise it would have drawn. */
int mppi_set_seed_counter(mppi_handle* h, uint64_t value);
int mppi_get_seed_counter(mppi_handle* h, uint64_t* value);

/* MPPI_PREC_BF16X3 with a CrossAttention net: *products = the products layer 1 runs with (2 or 3; 0 = not a split CA
 * handle, or no solve yet), *probe_rel_err = the probe's max relative cost difference between the two forms (-1: no
 * probe ran: forced by env, or H > 64).  Either pointer may be NULL. */
int mppi_x3_layer1(mppi_handle* h, int* products, float* probe_rel_err);
/* The rollout kernel the handle's last solve was routed to (e.g. "fc_wave32_x3p_kernel<l1=2>"); "" before the first
 * solve.  Valid until the next solve on the handle. */
const char* mppi_rollout_kernel(mppi_handle* h);
/* MPPI_PREC_BF16X3 with a CrossAttention net: *on = 1 if the rollouts run the fp16 form (MPPI_PREC_BF16X3 above) for
 * this handle's horizon, 2 with the opt-in one-product last layer (MPPI_X3_F16_L2=1), 0 if not (also before the first
 * solve); *probe_rel_err = the probe's max relative cost difference between the fp16 form on fc_wave32_x3p_kernel and
 * three products (-1: no probe ran).  Either pointer may be NULL. */
int mppi_x3_f16(mppi_handle* h, int* on, float* probe_rel_err);

/* Warm start: handle-resident nominal sequence, [B][nu][H] host memory. */
int mppi_get_U(mppi_handle* h, int B, float* U);
int mppi_set_U(mppi_handle* h, int B, const float* U);

/* Bind the handle to an existing hipStream_t (e.g. torch.cuda.current_stream().cuda_stream).
 * NULL restores the handle's own stream.  Between chained solves (MPPI_FLAG_CHAIN) the new stream is ordered behind
 * the work already enqueued on the old one. */
int mppi_set_stream(mppi_handle* h, void* hip_stream);
int mppi_sync(mppi_handle* h);

/* Per-kernel timing with hipEvents recorded on the handle's stream around each launch.
 * enable != 0 starts accumulating; mppi_kernel_times returns {count, total_ms} per kernel
 * name. names: "noise", "rollout", "reduce", "update". */
int mppi_profile(mppi_handle* h, int enable);
int mppi_kernel_time(mppi_handle* h, const char* kernel, int* count, double* total_ms);

/* Device launch clock of the rollout kernels, for timing INSIDE a timed region (graph replays included, no event
 * in the stream): every block folds its start / end device wall-clock stamps (s_memrealtime) into its launch's
 * slot with atomic min / max.  enable != 0 resets the slots and stamps every rollout enqueued or captured from
 * then on that uses the seed counter (MPPI_FLAG_SEED_COUNTER; graph streams always do); enable = 0 stops new
 * stamping.  A graph captured while enabled stamps on every replay.  mppi_kernel_clock_read waits for the stream
 * and returns the stamped launches since the reset with their summed (and largest) first-block-start to
 * last-block-end durations in microseconds; MPPI_E_UNSUPPORTED past 65536 launches per reset (kClockSlots). */
int mppi_kernel_clock(mppi_handle* h, int enable);
int mppi_kernel_clock_read(mppi_handle* h, int* launches, double* total_us, double* max_us);

/* Device pointers of the handle-resident buffers (for RCCL gathers without copies). */
int mppi_device_buffers(mppi_handle* h, void** dU, void** du0, void** dcosts);

const char* mppi_last_error(void);
int mppi_abi_version(void);
/* Provenance: the SHA-256 (hex) of the sources this library was built from (humanoid_mppi-rl_amd/build.py
 * source_hash: csrc/ and include/), so a caller can check that the binary it loaded matches its checkout. */
const char* mppi_build_id(void);

#ifdef __cplusplus
}
#endif
#endif /* MPPI_H_ */
