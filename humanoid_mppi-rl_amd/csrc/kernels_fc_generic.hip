// Learned-dynamics MPPI rollout for ANY fc-stack shape the shape-specialised kernel (fc_rollout.h) does not take:
// MLPStatePredictor of any hidden width / depth (learning/model.py:6-46; eval-mode BatchNorm folded on the host) and
// CrossAttentionStatePredictor of any qpos / qvel / hidden width (learning/model.py:157-202, folded as
// oracle/nets_ref.py::ca_fold + ln_fold), e.g. checkpoints_cartpole/model_final.pth (qpos 2, qvel 2, hidden 144) or
// the MLP of learning/train.py:70 (hidden 512, 6 hidden layers, BatchNorm).  x_{t+1} = x_t + net([x_t, u_t]).
//
// Mapping: a block = one group of 16 samples of one solve, 4 waves.  Activations live in LDS as [sample][feature]
// rows (bf16, or fp32 in the exact-fp32 mode), the MFMA B operand; every layer is out^T = W act^T with W the A operand,
// pre-packed 16x32 fragments (frag_traits.h) read from L2, output m-tiles dealt round-robin to the 4 waves.  The
// folded LayerNorm after layer 0 (CA) takes a second pass: raw rows to an fp32 scratch and per-wave sum h^2, one
// barrier, then y = relu(h rstd + beta').  The state is an fp32 [sample][nx] master copy; wave 0's lanes 0..15 evaluate
// the running cost of their sample every step (fa_cost, as the FeatureAttention kernels).  Correctness-first: the
// shipped headline shapes (folded humanoid CA, MLP(128 x 2)) run the register-resident kernel of fc_rollout.h.
#include <hip/hip_runtime.h>

#include "fa_common.h"
#include "frag_traits.h"

namespace mppi {

struct GenArgs {
  const char* img;
  FcGenNet g;
  int nx, nu;
  int act_s;  // bytes per activation row (maxw * E + 16)
};

template <int PREC>
__global__ __launch_bounds__(256) void fc_generic_kernel(SolveArgs a, GenArgs ga) {
  using F = FP<PREC>;
  constexpr int E = F::E;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const KClock kc = kclock_begin(a);
  const FcGenNet& g = ga.g;
  const GenLay Y(g, E, ga.nx, ga.nu);
  const int tid = threadIdx.x, lane = tid & 63, lg = lane >> 4, n = lane & 15;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nx = ga.nx, nu = ga.nu, H = a.H, act_s = ga.act_s;
  const int gps = a.Kp >> 4;  // groups per solve
  const int b = blockIdx.x / gps;
  const int k0 = (blockIdx.x - b * gps) * 16;
  if (blockIdx.x == 0 && tid == 0) *a.status = 0u;

  char* A0 = lds + Y.A0;
  char* A1 = lds + Y.A1;
  float* SCR = reinterpret_cast<float*>(lds + Y.SCR);
  float* XS = reinterpret_cast<float*>(lds + Y.XS);
  float* UF = reinterpret_cast<float*>(lds + Y.UF);
  float* ST = reinterpret_cast<float*>(lds + Y.ST);
  // zero the activation rows once: the padded input columns of every layer stay 0
  for (int i = tid; i < (Y.A1 + 16 * act_s) / 16; i += 256) reinterpret_cast<int4*>(lds)[i] = make_int4(0, 0, 0, 0);
  const float* x0 = a.x0 + (long)b * nx;
  for (int i = tid; i < 16 * nx; i += 256) XS[i] = x0[i % nx];

  float cx[MPPI_CTX_MAX];
#pragma unroll
  for (int i = 0; i < MPPI_CTX_MAX; ++i) cx[i] = a.ctx ? a.ctx[(long)b * MPPI_CTX_MAX + i] : a.ctx_default[i];
  const float cl = a.ctrl_clamp > 0.0f ? a.ctrl_clamp : INFINITY;
  const bool cown = w == 0 && lg == 0;  // lanes 0..15 of wave 0: the running cost of sample n
  float cost = 0.0f;
  const float* Ub = a.U + (long)b * nu * H;
  const float* Eb = a.noise + (long)b * nu * H * a.Kp;
  auto wr_act = [&](char* row, int col, float v) {
    if constexpr (E == 2)
      *reinterpret_cast<__bf16*>(row + col * 2) = (__bf16)v;
    else
      *reinterpret_cast<float*>(row + col * 4) = v;
  };
  __syncthreads();

  for (int t = 0; t < H; ++t) {
    // ---- layer-0 input [x ; u_t] (u = U + eps, clamped), the fp32 controls of this step for the cost
    float* uf = UF + (t & 1) * 16 * nu;
    for (int i = tid; i < 16 * nx; i += 256) {
      const int s = i / nx, j = i - s * nx;
      wr_act(A0 + s * act_s, j, XS[i]);
    }
    const int pad = g.kin[0] - nx - nu;  // layer 1 writes its output over A0: re-zero layer 0's padding columns
    for (int i = tid; i < 16 * pad; i += 256) {
      const int s = i / pad;
      wr_act(A0 + s * act_s, nx + nu + (i - s * pad), 0.0f);
    }
    for (int i = tid; i < 16 * nu; i += 256) {
      const int s = i / nu, j = i - s * nu;
      const int k = min(k0 + s, a.Kp - 1);
      const float u = __builtin_amdgcn_fmed3f(Ub[j * H + t] + Eb[((long)j * H + t) * a.Kp + k], -cl, cl);
      uf[s * nu + j] = u;
      wr_act(A0 + s * act_s, nx + j, u);
    }
    __syncthreads();
    char* in = A0;
    char* out = A1;
    for (int l = 0; l < g.nl; ++l) {
      const int KB = g.kin[l] / 32, MT = g.mt[l];
      const char* W = ga.img + g.w_off[l];
      const float* bias = reinterpret_cast<const float*>(ga.img + g.b_off[l]);
      const bool last = l + 1 == g.nl, ln = l == 0 && g.lnb_off >= 0, relu = (g.relu_mask >> l) & 1;
      float q = 0.0f;  // LayerNorm: this lane's part of sum h^2 of sample n
      for (int mt = w; mt < MT; mt += 4) {
        const int row = 16 * mt + 4 * lg;
        f32x4 acc = *reinterpret_cast<const f32x4*>(bias + row);
        const char* Wt = W + (long)mt * KB * F::FRAG;
        const char* bin = in + n * act_s;
        int kb = 0;
        for (; kb + 4 <= KB; kb += 4) {  // 4 k-blocks of loads in flight, then their MFMAs
          typename F::Frag af[4], bf[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            af[j] = F::ldA(Wt + (kb + j) * F::FRAG, lane);
            bf[j] = F::ldB(bin, kb + j, lg);
          }
#pragma unroll
          for (int j = 0; j < 4; ++j) acc = F::mma(af[j], bf[j], acc);
        }
        for (; kb < KB; ++kb) acc = F::mma(F::ldA(Wt + kb * F::FRAG, lane), F::ldB(bin, kb, lg), acc);
        if (last) {  // x += dx (state rows < nx)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (row + r < nx) XS[n * nx + row + r] += acc[r];
        } else if (ln) {
          *reinterpret_cast<f32x4*>(SCR + n * g.maxw + row) = acc;
          q += (acc[0] * acc[0] + acc[1] * acc[1]) + (acc[2] * acc[2] + acc[3] * acc[3]);
        } else if (relu) {
          F::st4_relu(out + n * act_s + row * E, acc);
        } else {
          F::st4(out + n * act_s + row * E, acc);
        }
      }
      if (ln) {  // folded LayerNorm: rows centred on the host, so var = mean(h^2); y = relu(h rstd + beta')
        q = fa_group_sum(q);
        if (lg == 0) ST[w * 16 + n] = q;
        __syncthreads();
        const float tot = (ST[n] + ST[16 + n]) + (ST[32 + n] + ST[48 + n]);
        const float rstd = __builtin_amdgcn_rsqf(tot / (float)g.ln_n + 1e-5f);
        const float* bp = reinterpret_cast<const float*>(ga.img + g.lnb_off);
        for (int mt = w; mt < MT; mt += 4) {
          const int row = 16 * mt + 4 * lg;
          const f32x4 h = *reinterpret_cast<const f32x4*>(SCR + n * g.maxw + row);
          const f32x4 be = *reinterpret_cast<const f32x4*>(bp + row);
          f32x4 y;
#pragma unroll
          for (int r = 0; r < 4; ++r) y[r] = fmaf(h[r], rstd, be[r]);
          F::st4_relu(out + n * act_s + row * E, y);
        }
      }
      __syncthreads();
      char* tmp = in;
      in = out;
      out = tmp;
    }
    // ---- running cost of step t on x_{t+1} with u_t (src/cartpole_mppi.py:78 order)
    if (cown) {
      const float* ur = uf + n * nu;
      float usq = 0.0f;
      for (int j = 0; j < nu; ++j) usq = fmaf(ur[j], ur[j], usq);
      cost += fa_cost(a.cost_kind, XS + n * nx, nu > 0 ? ur[0] : 0.0f, usq, cx, t + 1);
    }
  }
  kclock_record(a, kc);  // after the horizon's last barrier
  if (cown) {
    if (a.terminal_weight != 0.0f) cost += a.terminal_weight * fa_cost(a.cost_kind, XS + n * nx, 0.0f, 0.0f, cx, H);
    const int k = k0 + n;
    if (k < a.K) a.costs[(long)b * a.Kp + k] = isfinite(cost) ? cost : INFINITY;
  }
  if (a.xout && k0 == 0 && tid < nx) a.xout[(long)b * nx + tid] = XS[tid];  // env step: sample 0's final state
}

hipError_t launch_fc_generic(const SolveArgs& a, const FcNet& net, hipStream_t stream) {
  GenArgs ga;
  ga.img = reinterpret_cast<const char*>(net.d_img);
  ga.g = net.gen;
  ga.nx = a.nx;
  ga.nu = a.nu;
  const int E = net.precision == MPPI_PREC_BF16 ? 2 : 4;
  ga.act_s = net.gen.maxw * E + 16;
  const int lds = fc_generic_lds_bytes(net.gen, net.precision, a.nx, a.nu);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  const int grid = a.B * (a.Kp >> 4);
  note_kernel("fc_generic_kernel");
  auto kern = net.precision == MPPI_PREC_BF16 ? fc_generic_kernel<MPPI_PREC_BF16> : fc_generic_kernel<MPPI_PREC_FP32>;
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(kern, dim3(grid), dim3(256), lds, stream, a, ga);
  return hipGetLastError();
}

}  // namespace mppi
