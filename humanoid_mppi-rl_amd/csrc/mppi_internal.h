// Internal structures shared by the C-ABI host code (mppi_api.hip) and the kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mppi.h"

namespace mppi {

constexpr int kWave = 64;
constexpr int kKpAlign = 64;       // device pitch of the K axis (noise rows, costs)
constexpr int kMaxK = 32768;       // softmin weights are staged in LDS (<= 128 KiB)
constexpr int kMaxNx = 64;         // fc-stack state slots (4 m-tiles of 16)
constexpr int kMaxNu = 32;         // fc-stack control slots (2 m-tiles of 16)

// Everything a solve's kernels need, passed by value (kernel arguments live in SGPRs / constant
// cache; no per-call device allocation, so a solve can be captured into a hipGraph).
struct SolveArgs {
  int B, nx, nu, H, K, Kp;
  float lambda, ctrl_clamp, U_clamp, norm_eps, shift_fill, terminal_weight;
  int update_mode, flags, cost_kind;
  float ctx_default[MPPI_CTX_MAX];
  const float* x0;      // [B][nx]
  float* U;             // [B][nu][H]   (read by rollout, updated in place by the update kernel)
  float* noise;         // [B][nu][H][Kp]
  float* costs;         // [B][Kp]
  float* dU;            // [B][nu][H]   weighted-noise sums (normalised)
  float* weights;       // [B][Kp] or nullptr
  float* u0;            // [B][nu] or nullptr
  const float* ctx;     // [B][MPPI_CTX_MAX] or nullptr (-> ctx_default)
  unsigned* status;     // [1] bit0: some solve had no finite cost
  unsigned* tickets;    // [B] reduce-block arrival counters (zero between solves)
  float* xout;          // [B][nx] or nullptr: rollouts write the final state of sample k = 0 (env step)
  float* Umirror;       // [B][nu][H] or nullptr: the update also writes the new U here (RESIDENT_U + io.U, device)
  unsigned long long* seed_ctr;   // or nullptr: noise key = seed + *seed_ctr
  unsigned long long* seed_bump;  // or nullptr: the reduce advances this counter after the solve (plain solves)
  // analytic cartpole: per-block softmin partials [B][Kp/256][2 + H] (block min, block weight sum, weighted noise
  // rows); non-null = the rollout finishes the solve itself (fused epilogue, no reduce launch)
  float* part;
  // or nullptr: device wall-clock stamps of this rollout launch (mppi_kernel_clock), [kClockSlots][2] =
  // {earliest block start, latest block end}; slot = *kclock_ctr at the block's start
  unsigned long long* kclock;
  unsigned long long* kclock_ctr;  // stamped launches since the reset (advanced by the launch's last block)
  unsigned* kclock_ticket;         // block arrivals of the current stamped launch (zero between launches)
};

// Rollout launch clock (mppi_kernel_clock): every block's leader folds its start / end stamps (s_memrealtime,
// the constant-rate device wall clock) into the launch's slot with global atomic min / max, so the launch duration
// (first block start -> last block end) is measured inside a timed region, graph replays included, with no event
// in the stream.  The slot is the clock's own launch counter, read at the block's start; the launch's LAST
// arriving block (a ticket over the whole grid) advances it, so no block of the launch can see it move whatever
// the order in which the hardware dispatches the blocks.  Three vector atomics per block: nothing measurable
// against a rollout of >= 10 us.
constexpr int kClockSlots = 65536;
struct KClock {
  unsigned long long t0;
  unsigned slot;
};
__device__ __forceinline__ KClock kclock_begin(const SolveArgs& a) {
  if (!a.kclock) return KClock{0ull, 0u};
  return KClock{(unsigned long long)wall_clock64(), (unsigned)(*a.kclock_ctr & (kClockSlots - 1))};
}
// leader: the ONE thread per block that stamps (the block's thread 0 after the block's last barrier by default).
// INVARIANT: every block of a stamped launch calls kclock_record exactly once with exactly one leader, after all of
// its work (no early exit past it, no second leader): the launch counter advances only when the ticket counts every
// block of the grid, and a launch that broke this would leave it behind, folding all later launches into one slot.
// mppi_kernel_clock_read checks the device counter against the host's count of stamped launches and fails loudly.
__device__ __forceinline__ void kclock_record(const SolveArgs& a, const KClock& c, bool leader = threadIdx.x == 0) {
  if (a.kclock && leader) {
    unsigned long long* s = a.kclock + 2 * c.slot;
    atomicMin(s, c.t0);
    atomicMax(s + 1, (unsigned long long)wall_clock64());
    const unsigned nblk = gridDim.x * gridDim.y * gridDim.z;
    if (__hip_atomic_fetch_add(a.kclock_ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nblk - 1) {
      __hip_atomic_store(a.kclock_ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      atomicAdd(a.kclock_ctr, 1ull);
    }
  }
}

// Analytic cartpole constants (models/cartpole.xml; derivation in oracle/mppi_ref.py::_cartpole_params).
struct CartpoleParams {
  float m_cart, m_pole, l, inertia, damping, gear, ctrl_lo, ctrl_hi, g, dt;
};

// Learned-dynamics (fc stack) network description after folding + packing (mppi_nets.cpp).
enum FcArch : int { kArchNone = 0, kArchCA = 1, kArchMLP = 2, kArchGeneric = 3 };
// bf16 fc rollouts: layers (bit l = layer l) whose per-wave A fragments live in VGPRs for the whole horizon; the
// packer puts the others first, as the LDS-staged image prefix.  All layers: no weight traffic in the loop.
constexpr int kCaRegMask = 0x7;   // folded CA: 3 layers
// Folded CA, bf16 image: layer 0's bias also sits in the (zero) pad state slots 28 and 29 as a bf16 hi / lo pair, so
// a kernel whose layer-0 operand holds 1.0 in those slots gets h = W0 x + b0 from the MFMA alone (fc_pipe_kernel);
// kernels that keep the slots at 0 add the fp32 bias as before.
constexpr int kCaBiasSlotHi = 28, kCaBiasSlotLo = 29;
// ... and beta' of the folded LayerNorm as a bf16 hi / lo pair in the pad columns 30 (hi), 31 (lo) and 59 (hi again):
// an operand holding (s_hi, s_hi, s_lo) there adds beta' s (to ~2^-18) for the per-wave kernel's s = sqrt(var + eps)
constexpr int kCaBetaSlotHi0 = 30, kCaBetaSlotLo = 31, kCaBetaSlotHi1 = 59;
// ... and fc_wave32_kernel's block-diagonal layer 0 (w32_bd): the qvel-fed rows' b0 pair in pad slots 60, 61 (1.0 in
// the state) and their beta' pair in 62, 63 (against s_hi); row 30 of its Gram factor is the row mean of layer 0
constexpr int kCaBdBiasSlotHi = 60, kCaBdBiasSlotLo = 61, kCaBdBetaSlotHi = 62, kCaBdBetaSlotLo = 63;
constexpr int kCaBdMeanRow = 30;
// ... and the split per-wave image's layer 0 (L0x): a column of 1.0 in pad slots 29 (qpos rows) and 61 (qvel rows),
// against which fc_wave32_x3p_kernel's operand carries -mu (hi / lo), so the row mean leaves through the MFMA
constexpr int kCaX3MeanSlot = 29, kCaX3BdMeanSlot = 61;
// ... and, for its fp16 form (one fp16 operand, fc_common.h x3_f16_on), -mu's lo part against a second column of 1.0
constexpr int kCaX3MeanLoSlot = 31, kCaX3BdMeanLoSlot = 63;
// ... and the fp16-form M-split kernel fc_rollout_kernel_x3h: layer 0's bias in this pad column (against a state slot
// held at 1.0), so h = W0 x + b0 leaves the MFMA chain with no bias read (needs qpos <= 31)
constexpr int kCaX3hBiasSlot = 31;
#ifndef MPPI_X3_F16_L0  // the fp16 form's layer 0 and statistic: fp16 W hi + lo against one fp16 operand (1), or the
                        // bf16 three products (0); the packer (mppi_nets.cpp) and the per-wave kernels agree on it
#define MPPI_X3_F16_L0 1
#endif
constexpr int kMlpRegMask = 0xF;  // MLP(hidden 128, 2 hidden layers): 4 layers
// MLP, bf16 image: layer 0's bias as a bf16 hi / lo pair in the pad state columns 62, 63 (when nx <= 62), for the
// per-wave kernel whose state holds 1.0 there; the M-split kernel keeps those slots at 0 and adds the fp32 bias
constexpr int kMlpBiasSlotHi = 62, kMlpBiasSlotLo = 63;

// Generic fc stack (kernels_fc_generic.hip): any MLPStatePredictor (hidden width, depth, eval-mode BatchNorm folded)
// and any CrossAttentionStatePredictor (qpos / qvel / hidden; folded) that the shape-specialised kernel does not take.
// Layer 0 reads [x (nx) ; u (nu) ; 0] padded to kin[0]; layer l writes mt[l] 16-row tiles; the last layer's rows are
// the state deltas.  Fragments packed by mppi_nets.cpp::pack_frags (16x32, [mt][kb][lane]).
constexpr int kGenMaxLayers = 16;
constexpr int kGenMaxWidth = 1024;  // widest layer (padded); fp32 parity mode: 512
struct FcGenNet {
  int nl = 0;
  int kin[kGenMaxLayers] = {0};    // padded input width of layer l (multiple of 32)
  int mt[kGenMaxLayers] = {0};     // output 16-row tiles of layer l
  int w_off[kGenMaxLayers] = {0};  // packed fragments of layer l
  int b_off[kGenMaxLayers] = {0};  // fp32 bias of layer l (16 mt[l] floats)
  int relu_mask = 0;               // bit l: ReLU after layer l
  int lnb_off = -1;                // >= 0: layer 0 is followed by the folded LayerNorm (CA): beta' (16 mt[0] floats)
  int ln_n = 0;                    // true LayerNorm width
  int maxw = 0;                    // widest activation row (padded to 32)
};

struct FcNet {
  int arch = kArchNone;
  FcGenNet gen;                    // arch == kArchGeneric
  int precision = MPPI_PREC_BF16;
  // Byte offsets inside the packed image (identical layout for LDS copy and global reads).
  int w_off[4] = {0, 0, 0, 0};     // per-layer packed weight fragments
  int b_off[4] = {0, 0, 0, 0};     // per-layer fp32 bias (padded rows)
  int lnb_off = 0;                 // beta' of the LayerNorm after layer 0, folded (fp32; gamma lives in layer 1)
  int ln_n = 0;                    // true LayerNorm width (pads excluded)
  int img_bytes = 0;
  int lds_bytes = 0;               // bf16: prefix of the image staged in LDS (the other layers live in VGPRs)
  int reg_mask = 0;                // layers packed after the LDS prefix (kCaRegMask / kMlpRegMask)
  // state slots: x[0, qp) -> slots [0, qp); x[qp, qp+qv) -> slots [32, 32+qv) (CA: qpos | qvel).
  int qp = 0, qv = 0;
  // folded humanoid CA, bf16: the per-wave rollout (kernels_fc_wave.hip) also needs the layer-0 Gram matrix of the
  // bf16 columns as hi / lo bf16 fragments (G_hi at g_off, G_lo at g_off + 8 KiB) and beta' as bf16 hi / lo in the pad
  // state columns kCaBetaSlotHi0/Lo/Hi1 of layer 0; -1: not built (other shapes or fp32)
  int g_off = -1;
  int w32_off = -1;                // ... and the CA layers + Gram factor as 32x32x16 A fragments (fc_wave32_kernel)
  int w32_bd = 0;                  // ... with layer 0 block-diagonal, uncentred (the mean from the Gram factor's row 30):
                                   // 1 = 112 MFMAs per wave-step, 2 = 108 (qpos rows' bias via the accumulators); 0 = dense
  int w0bd_off = -1, gbd_off = -1;  // form 2 for fc_wave_kernel (16x16): its layer 0 and Gram factor as 16x32 fragments
  int w32x3_off = -1, w32x3_l1lo_off = -1;  // split bf16 per-wave image (fc_wave32_x3_kernel): LDS part, W1 lo part
  int wmx3_off = -1, wmx3_lo_off = -1;      // split bf16 per-wave MLP image (fc_wave_mlp_x3_kernel): LDS part, W1|W2 lo
  int wm32x3_off = -1, wm32x3_lo_off = -1;  // ... 32 samples per wave (fc_wave32_mlp_x3_kernel): LDS part, W1|W2 lo
  int wave = 0;                    // the image carries what the per-wave kernel needs (CA: g_off, beta'; MLP: the b0 pair)
  // split bf16 (MPPI_PREC_BF16X3) CA only: products on layer 1 as decided for THIS net by the engine's probe
  // (mppi_api.hip x3_probe: the two- and three-product rollouts of the first solve's own states against each other);
  // 0 = not probed yet (three products), 2 = the probe stayed within kX3ProbeTol, 3 = it did not
  int x3_l1 = 0;
  float x3_l1_err = -1.0f;         // the probe's max relative cost difference (-1: no probe ran)
  // ... and the fp16 form (fc_common.h x3_f16_on): its images (fc_wave32_x3p_kernel's: the w32x3 LDS image in fp16;
  // the M-split kernel's below), the probe's decision (0 = not probed, 1 = within kX3ProbeTol, -1 = not; 2 = the
  // opt-in one-product last layer, x3_f16_l2x1) and difference; x3_route = 1 / 2 only in the probe's own copy
  // (fc_wave32_x3p_kernel whatever the batch)
  int w32f16_off = -1;
  int wmf16_off = -1, wmf16_x_off = -1;  // ... the M-split kernels' (fc_rollout_kernel_x3d<F16>): W1, the last layer,
  int wmf16_0_off = -1;                  //     layer 0 (fp16 hi / lo)
  int wmf16_0b_off = -1;                 //     ... with b0 in the pad column kCaX3hBiasSlot (fc_rollout_kernel_x3h)
  int x3_f16 = 0;
  float x3_f16_err = -1.0f;
  int x3_route = 0;
  void* d_img = nullptr;           // device copy of the packed image
};

// CU count of the CURRENT device (the launchers size persistent grids by it), cached per device id: a process that
// drives several GPUs gets each one's own count.  Thread-safe (relaxed atomics; a race only repeats the query).
int current_device_cus();

// The rollout kernel the last fc / FA / cartpole launch on this host thread routed to (mppi_rollout_kernel): set by
// every launcher, read by the ABI right after the launch (a handle is used from one thread).
extern thread_local const char* g_rollout_kernel;
inline void note_kernel(const char* name) { g_rollout_kernel = name; }

// FeatureAttentionStatePredictor (learning/model.py:48-153) rollout. Blocking shared by the host packer and the
// kernel: 4 heads; attention is processed in chunks of fa_cw(D) columns (whole heads), the FFN hidden layer in
// chunks of fa_fc(D) rows; a workgroup has fa_nw(D) waves and kFaRows token rows.
// Up to 5 token n-tiles (80 rows: the full humanoid state + action, 76 tokens, learning/model.py:215), up to 8
// attention layers (learning/train.py:72 trains 7), 4 or 8 heads (num_heads, learning/train.py:72: 8).
constexpr int kFaRows = 80;
constexpr int kFaMaxLayers = 8;
constexpr int kFaHeads = 4;  // the small-net kernel: one head per wave
__host__ __device__ constexpr int fa_nt_min(int L) { return L <= 16 ? 1 : (L <= 32 ? 2 : (L <= 64 ? 4 : 5)); }
// attention chunk width (whole heads of width D / NH): 5 token tiles, and hidden 128 with 8 heads (8 probability
// tiles per chunk otherwise), take 64-wide chunks to fit the LDS
__host__ __device__ constexpr bool fa_narrow(int D, int NH, int NT) { return NT > 4 || (D == 128 && NH == 8); }
__host__ __device__ constexpr int fa_cw(int D, int NH = 4, int NT = 4) {
  return fa_narrow(D, NH, NT) ? (D / NH > 64 ? D / NH : 64) : (D / NH >= 128 ? D / NH : (D < 128 ? D : 128));
}
// waves per workgroup: 8 for wide nets; hidden 128 with 64-wide chunks takes 4 (its Q|K|V tiles split evenly)
__host__ __device__ constexpr int fa_nw(int D, int NT = 4, int NH = 4) {
  return D >= 128 && !(D == 128 && fa_narrow(D, NH, NT)) ? 8 : 4;
}
__host__ __device__ constexpr int fa_fc(int D) { return D >= 512 ? 256 : (4 * D < 512 ? 4 * D : 512); }

struct FaNet {
  int D = 0, L = 0, nlayers = 0, nh = 4, precision = MPPI_PREC_BF16;
  // fp32 vectors (byte offsets into the image)
  int we = 0, be = 0, ge = 0, bte = 0, pos = 0, wout = 0;
  int ln1g[kFaMaxLayers], ln1b[kFaMaxLayers], bqkv[kFaMaxLayers], bo[kFaMaxLayers];
  int ln2g[kFaMaxLayers], ln2b[kFaMaxLayers], b1[kFaMaxLayers], b2[kFaMaxLayers];
  // packed A-operand fragments (chunked, see mppi_nets.cpp::build_fa_net)
  int wqkv[kFaMaxLayers], wo[kFaMaxLayers], w1[kFaMaxLayers], w2[kFaMaxLayers];
  // small-net kernel (bf16, D = 64, L <= 16: kernels_fa.hip::fa_small_kernel): per-head Q|K|V and the FFN matrices
  // with the register-operand k order; small = 0: not built
  int small = 0;
  int s_wqkv[kFaMaxLayers], s_w1[kFaMaxLayers], s_w2[kFaMaxLayers];
  int s_c1 = 0, s_c2 = 0;  // encoding: (w - mean w) gamma, (b - mean b) gamma (fp32 vectors)
  int s_bqkv[kFaMaxLayers], s_b1[kFaMaxLayers];  // biases of the LayerNorm-folded Q|K|V and FFN1 (fp32 vectors)
  // closed-form LayerNorm statistics of the scalar feature encoding h = w v + b (population moments over D)
  float enc_mw = 0, enc_mb = 0, enc_vw = 0, enc_cwb = 0, enc_vb = 0, b_out = 0;
  // hidden 512, bf16: the layer-by-layer path (kernels_fa_layered.hip) reads every matrix as plain row-major bf16
  // [out][in] (Q rows pre-scaled by 1/sqrt(head dim)) and the Q|K|V bias in natural order; lay = 0: not built
  int lay = 0;
  int lwqkv[kFaMaxLayers], lwo[kFaMaxLayers], lw1[kFaMaxLayers], lw2[kFaMaxLayers], lbqkv[kFaMaxLayers];
  int img_bytes = 0;
  void* d_img = nullptr;
  // ... and its activation workspace (fa_layered_ws_bytes), allocated by mppi_load_dynamics for max_batch * K * L
  // token rows; nullptr: the fused fa_rollout_kernel runs
  void* d_ws = nullptr;
  long ws_rows = 0;
};

// Launchers (return hipSuccess or the launch error). All enqueue on `stream` only.
// device noise into noise[B][nu][H][Kp]; seed_ctr (or nullptr): device key offset
hipError_t launch_noise(float* noise, int B, int nu, int H, int Kp, uint64_t seed, const unsigned long long* seed_ctr,
                        float sigma, hipStream_t stream);
hipError_t launch_seed_bump(unsigned long long* seed_ctr, long long delta, hipStream_t stream);  // += delta
hipError_t launch_fc_rollout(const SolveArgs& a, const FcNet& net, hipStream_t stream);
hipError_t launch_fc_generic(const SolveArgs& a, const FcNet& net, hipStream_t stream);  // kernels_fc_generic.hip

// LDS layout (bytes) of one block of the generic fc-stack kernel: activation rows A0 | A1 ([16][maxw] of E-byte
// elements, +16 B per row), the LayerNorm layer's fp32 raw rows, the fp32 state [16][nx], the fp32 controls of two
// steps [2][16][nu], the per-wave LayerNorm partial sums [4][16].
struct GenLay {
  int A0, A1, SCR, XS, UF, ST, total;
  __host__ __device__ GenLay(const FcGenNet& g, int E, int nx, int nu) {
    const int act_s = g.maxw * E + 16;
    A0 = 0;
    A1 = A0 + 16 * act_s;
    SCR = A1 + 16 * act_s;
    XS = SCR + (g.lnb_off >= 0 ? 16 * g.maxw * 4 : 0);
    UF = XS + 16 * nx * 4;
    ST = UF + 2 * 16 * (nu > 0 ? nu : 1) * 4;
    total = (ST + 4 * 16 * 4 + 15) / 16 * 16;
  }
};
inline int fc_generic_lds_bytes(const FcGenNet& g, int precision, int nx, int nu) {
  return GenLay(g, precision == MPPI_PREC_BF16 ? 2 : 4, nx, nu).total;
}
hipError_t launch_fa_rollout(const SolveArgs& a, const FaNet& net, hipStream_t stream);
// kernels_fa_layered.hip: the layer-by-layer hidden-512 rollout and its workspace size for `rows` token rows
hipError_t launch_fa_layered(const SolveArgs& a, const FaNet& net, hipStream_t stream);
size_t fa_layered_ws_bytes(long rows);
// reduce_kernel<GEN>: also writes the next solve's noise (graph streams)
struct NoiseGen {
  float* next;
  uint64_t seed;
  float sigma;
  unsigned* gticket;  // [1], zero between solves
};
hipError_t launch_reduce(const SolveArgs& a, const NoiseGen* gen, hipStream_t stream);  // softmin + reduce + update + shift
// analytic cartpole rollout; with a.part set it also runs a7-a9 (fused epilogue) and, given gen, writes the next
// solve's noise (graph streams)
hipError_t launch_cartpole_rollout(const SolveArgs& a, const CartpoleParams& p, const NoiseGen* gen, hipStream_t stream);
hipError_t launch_record(const float* x, const float* u, float* rx, float* ru, int nxB, int nuB, hipStream_t stream);

}  // namespace mppi
