// Host-side preparation of learned dynamics: parse the weight blob, fold the cross-attention net,
// map state/control features to kernel slots and pack MFMA A-operand fragments (bf16 or fp32).
//
// Weight blob (little endian), written by mppi_hip.nets.pack_blob():
//   "MPPW" | u32 version=1 | u32 kind | i32 dims[8] | u32 n_tensors |
//   n_tensors x { u32 name_len | name | u32 ndim | u32 shape[ndim] | f32 data[prod(shape)] }
// Tensor names are the torch state_dict keys of learning/model.py modules.
//   kind MPPI_DYN_MLP:        dims = {state_dim, action_dim, hidden_dim, hidden_layers}
//   kind MPPI_DYN_CROSS_ATTN: dims = {qpos_dim, qvel_dim, action_dim, hidden_dim, num_heads}
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

#include "mppi_internal.h"

namespace mppi {

struct Tensor {
  std::vector<int> shape;
  std::vector<double> v;
};

using TensorMap = std::map<std::string, Tensor>;

static void parse_blob(const void* blob, size_t n, int* kind, int dims[8], TensorMap& out) {
  const unsigned char* p = static_cast<const unsigned char*>(blob);
  const unsigned char* end = p + n;
  auto need = [&](size_t k) {
    if ((size_t)(end - p) < k) throw std::runtime_error("weight blob truncated");
  };
  auto rd_u32 = [&]() {
    need(4);
    uint32_t v;
    std::memcpy(&v, p, 4);
    p += 4;
    return v;
  };
  need(4);
  if (std::memcmp(p, "MPPW", 4) != 0) throw std::runtime_error("weight blob: bad magic (expected MPPW)");
  p += 4;
  if (rd_u32() != 1) throw std::runtime_error("weight blob: unsupported version");
  *kind = (int)rd_u32();
  for (int i = 0; i < 8; ++i) dims[i] = (int)rd_u32();
  const uint32_t nt = rd_u32();
  for (uint32_t t = 0; t < nt; ++t) {
    const uint32_t ln = rd_u32();
    need(ln);
    std::string name(reinterpret_cast<const char*>(p), ln);
    p += ln;
    const uint32_t nd = rd_u32();
    if (nd > 8) throw std::runtime_error("weight blob: tensor rank > 8");
    Tensor T;
    size_t cnt = 1;
    const size_t left = (size_t)(end - p) / 4;  // floats the rest of the blob can hold (bounds every product below)
    for (uint32_t d = 0; d < nd; ++d) {
      const uint32_t dim = rd_u32();
      if (dim > (1u << 30) || (dim > 0 && cnt > left / dim)) throw std::runtime_error("weight blob truncated");
      T.shape.push_back((int)dim);
      cnt *= dim;
    }
    need(cnt * 4);
    T.v.resize(cnt);
    for (size_t i = 0; i < cnt; ++i) {
      float f;
      std::memcpy(&f, p + 4 * i, 4);
      T.v[i] = f;
    }
    p += cnt * 4;
    out[name] = std::move(T);
  }
}

static const Tensor& get(const TensorMap& m, const std::string& k, std::vector<int> shape) {
  auto it = m.find(k);
  if (it == m.end()) throw std::runtime_error("weight blob: missing tensor " + k);
  if (it->second.shape != shape) throw std::runtime_error("weight blob: bad shape for " + k);
  return it->second;
}

// Dense matrix helpers (row-major, double).
struct Mat {
  int r = 0, c = 0;
  std::vector<double> a;
  Mat() = default;
  Mat(int r_, int c_) : r(r_), c(c_), a((size_t)r_ * c_, 0.0) {}
  double& operator()(int i, int j) { return a[(size_t)i * c + j]; }
  double operator()(int i, int j) const { return a[(size_t)i * c + j]; }
};

static Mat from(const Tensor& t, int row0 = 0, int rows = -1) {
  const int C = t.shape.size() == 2 ? t.shape[1] : 1;
  const int R = rows < 0 ? t.shape[0] : rows;
  Mat m(R, C);
  for (int i = 0; i < R; ++i)
    for (int j = 0; j < C; ++j) m(i, j) = t.v[(size_t)(row0 + i) * C + j];
  return m;
}
static Mat matmul(const Mat& A, const Mat& B) {
  Mat C(A.r, B.c);
  for (int i = 0; i < A.r; ++i)
    for (int k = 0; k < A.c; ++k) {
      const double a = A(i, k);
      for (int j = 0; j < B.c; ++j) C(i, j) += a * B(k, j);
    }
  return C;
}
static std::vector<double> matvec(const Mat& A, const std::vector<double>& x) {
  std::vector<double> y(A.r, 0.0);
  for (int i = 0; i < A.r; ++i)
    for (int j = 0; j < A.c; ++j) y[i] += A(i, j) * x[j];
  return y;
}
static std::vector<double> vec(const Tensor& t, int off = 0, int n = -1) {
  n = n < 0 ? (int)t.v.size() : n;
  return std::vector<double>(t.v.begin() + off, t.v.begin() + off + n);
}

// One layer in SLOT coordinates (rows = 16*MTO padded outputs, cols = 16*MTI padded inputs).
// blocks > 1: block-diagonal (row block i reads only column block i); only the diagonal blocks are packed.
struct SlotLayer {
  int mto, mti;
  Mat W;                  // [16*mto][16*mti]
  std::vector<double> b;  // [16*mto]
  int blocks = 1;
};

static uint16_t f32_to_bf16_rne(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7F800000u) == 0x7F800000u && (u & 0x7FFFFFu)) return (uint16_t)((u >> 16) | 0x40);  // quiet NaN
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
// IEEE binary16, round to nearest even, subnormals kept (what v_cvt_pk_f16_f32 does), overflow to infinity
static uint16_t f32_to_f16_rne(float f) {
  const uint16_t sgn = std::signbit(f) ? 0x8000 : 0;
  const double a = std::fabs((double)f);
  if (std::isnan(f)) return 0x7E00;
  if (a >= 65520.0) return sgn | 0x7C00;
  if (a == 0.0) return sgn;
  int e;
  std::frexp(a, &e);
  const int E = std::max(e - 1, -14);                       // binade [2^E, 2^(E+1)); subnormals share 2^-14's spacing
  const double r = std::nearbyint(std::ldexp(a, 10 - E));  // in units of the spacing 2^(E - 10), ties to even
  if (E == -14 && r < 1024.0) return sgn | (uint16_t)r;    // subnormal (or zero)
  const int Er = r >= 2048.0 ? E + 1 : E;                  // rounded up into the next binade
  const uint32_t m = (uint32_t)(r >= 2048.0 ? r / 2 : r) - 1024u;
  return Er > 15 ? (uint16_t)(sgn | 0x7C00) : (uint16_t)(sgn | (uint32_t)(Er + 15) << 10 | m);
}
static double f16_to_f64(uint16_t b) {
  const int e = (b >> 10) & 31, m = b & 1023;
  const double v = e == 31 ? (m ? NAN : INFINITY) : (e ? std::ldexp(1024.0 + m, e - 25) : std::ldexp((double)m, -24));
  return (b & 0x8000) ? -v : v;
}

// Pack the layer stack + LN into one image; fills offsets in `net`.  Image order: the weight fragments of the
// layers NOT in `reg_mask` (bit l: layer l) -- the prefix [0, net.lds_bytes) the bf16 kernel stages in LDS --, then
// the fragments of the `reg_mask` layers (loaded into VGPRs once per launch), then every layer's fp32 bias and the
// folded LayerNorm's beta'.
static std::vector<unsigned char> pack_image(const std::vector<SlotLayer>& L, const std::vector<double>* ln_b,
                                             int precision, int reg_mask,
                                             FcNet& net, const std::vector<SlotLayer>* gram = nullptr,
                                             const SlotLayer* l0_32 = nullptr,
                                             const std::vector<SlotLayer>* gram32 = nullptr,
                                             const SlotLayer* l0_x3 = nullptr, const SlotLayer* r_x3 = nullptr,
                                             bool mlp_x3 = false) {
  std::vector<unsigned char> img;
  auto align16 = [&]() {
    while (img.size() % 16) img.push_back(0);
  };
  auto put_f32 = [&](float f) {
    unsigned char b[4];
    std::memcpy(b, &f, 4);
    img.insert(img.end(), b, b + 4);
  };
  auto put_frags = [&](const SlotLayer& S) {
    // fragment (mt, kk) of k-step ks = blk(mt) * KSB + kk, at index (mt * KSB + kk) * 64 + lane
    // (kernels_fc.hip::mfma_rows). bf16 k-step = 32 features, fp32 k-step = 4 features.  Split bf16 (BF16X3): per lane
    // the bf16 fragment of W (hi, 16 B) then that of W - hi (lo, 16 B): 32 B per lane (fc_common.h P<BF16X3>::Wt)
    const bool bf = precision == MPPI_PREC_BF16 || precision == MPPI_PREC_BF16X3;
    const int KS = bf ? S.mti / 2 : S.mti * 4;
    const int KSB = KS / S.blocks, RPB = S.mto / S.blocks;
    for (int mt = 0; mt < S.mto; ++mt)
      for (int kk = 0; kk < KSB; ++kk) {
        const int ks = (S.blocks == 1 ? 0 : (mt / RPB) * KSB) + kk;
        for (int lane = 0; lane < 64; ++lane) {
          const int row = 16 * mt + (lane & 15);
          if (bf) {
            for (int part = 0; part < (precision == MPPI_PREC_BF16X3 ? 2 : 1); ++part)
              for (int j = 0; j < 8; ++j) {
                const int col = 32 * ks + 16 * (j >> 2) + 4 * (lane >> 4) + (j & 3);
                const float w = (float)S.W(row, col);
                uint16_t h = f32_to_bf16_rne(w);
                if (part == 1) {  // the residual W - hi, itself rounded to bf16
                  const uint32_t hu = (uint32_t)h << 16;
                  float hf;
                  std::memcpy(&hf, &hu, 4);
                  h = f32_to_bf16_rne((float)(S.W(row, col) - (double)hf));
                }
                img.push_back((unsigned char)(h & 0xFF));
                img.push_back((unsigned char)(h >> 8));
              }
          } else {
            put_f32((float)S.W(row, 16 * (ks >> 2) + 4 * (lane >> 4) + (ks & 3)));
          }
        }
      }
  };
  auto put_frags16 = [&](const SlotLayer& S, int parts) {
    // put_frags' bf16 lane layout and (m-tile, k-step) order in fp16: one part (W rounded) or two (hi, then lo = W - hi
    // itself rounded, 32 B per lane like BX3) -- fc_rollout_kernel_x3d's fp16 form (fc_common.h x3_f16_on)
    const int KS = S.mti / 2, KSB = KS / S.blocks, RPB = S.mto / S.blocks;
    for (int mt = 0; mt < S.mto; ++mt)
      for (int kk = 0; kk < KSB; ++kk) {
        const int ks = (S.blocks == 1 ? 0 : (mt / RPB) * KSB) + kk;
        for (int lane = 0; lane < 64; ++lane) {
          const int row = 16 * mt + (lane & 15);
          for (int part = 0; part < parts; ++part)
            for (int j = 0; j < 8; ++j) {
              const double w = S.W(row, 32 * ks + 16 * (j >> 2) + 4 * (lane >> 4) + (j & 3));
              uint16_t h = f32_to_f16_rne((float)w);
              if (part == 1) h = f32_to_f16_rne((float)(w - f16_to_f64(h)));
              img.push_back((unsigned char)(h & 0xFF));
              img.push_back((unsigned char)(h >> 8));
            }
        }
      }
  };
  auto put_layer = [&](size_t l) {
    align16();
    net.w_off[l] = (int)img.size();
    put_frags(L[l]);
  };
  for (size_t l = 0; l < L.size(); ++l)
    if (!(reg_mask >> l & 1)) put_layer(l);
  align16();
  net.lds_bytes = (int)img.size();
  for (size_t l = 0; l < L.size(); ++l)
    if (reg_mask >> l & 1) put_layer(l);
  for (size_t l = 0; l < L.size(); ++l) {
    align16();
    net.b_off[l] = (int)img.size();
    for (double v : L[l].b) put_f32((float)v);
  }
  if (ln_b) {
    align16();
    net.lnb_off = (int)img.size();
    for (double v : *ln_b) put_f32((float)v);
  }
  if (gram) {  // the per-wave CA kernel's Gram matrix: G_hi, then G_lo (8 KiB each)
    align16();
    net.g_off = (int)img.size();
    for (const SlotLayer& S : *gram) put_frags(S);
    // ... and every layer + the Gram factor again as v_mfma_f32_32x32x16_bf16 A fragments (kernels_fc_wave.hip,
    // fc_wave32_kernel): fragment (D-tile T of 32 rows, k-step ks of 16) at index T * KS16 + ks, lane l holds row
    // 32 T + (l & 31) at the k slots 8 (l >> 5) + j, which carry input feature
    //   32 (ks / 2) + 8 (2 (ks % 2) + (j >> 2)) + 4 (l >> 5) + (j & 3)
    // -- the row a lane of the previous layer's 32x32 accumulator tile holds there (value v = 4 i + r of lane l is row
    // 8 i + 4 (l >> 5) + r), so that accumulator packed to bf16 (values 8 (ks % 2) .. + 7) is this layer's B operand.
    align16();
    net.w32_off = (int)img.size();
    auto put32 = [&](const SlotLayer& S) {
      const int MT32 = S.mto / 2, KS16 = S.mti;  // 32-row D-tiles; 16-wide k-steps over 16 mti inputs
      for (int T = 0; T < MT32; ++T)
        for (int ks = 0; ks < KS16; ++ks)
          for (int lane = 0; lane < 64; ++lane) {
            const int row = 32 * T + (lane & 31), h = lane >> 5;
            for (int j = 0; j < 8; ++j) {
              const int col = 32 * (ks / 2) + 8 * (2 * (ks % 2) + (j >> 2)) + 4 * h + (j & 3);
              const uint16_t b = f32_to_bf16_rne((float)S.W(row, col));
              img.push_back((unsigned char)(b & 0xFF));
              img.push_back((unsigned char)(b >> 8));
            }
          }
    };
    // (fc_wave32_kernel's own layer 0 and Gram factor when given: the block-diagonal form, net.w32_bd)
    for (size_t l = 0; l < L.size(); ++l) put32(l == 0 && l0_32 ? *l0_32 : L[l]);
    for (const SlotLayer& S : gram32 ? *gram32 : *gram) put32(S);
    if (l0_32 && gram32 && net.w32_bd == 2) {  // ... and for fc_wave_kernel (16x32 fragments, put_frags order)
      align16();
      net.w0bd_off = (int)img.size();
      put_frags(*l0_32);
      align16();
      net.gbd_off = (int)img.size();
      for (const SlotLayer& S : *gram32) put_frags(S);
    }
  }
  if (l0_x3 && r_x3) {
    // fc_wave32_x3_kernel (split bf16, kernels_fc_x3.hip): 32x32x16 A fragments (put32's lane layout) as bf16
    // hi and lo parts (lo = W - hi, itself rounded).  LDS image, in the kernel's order: hi of layer 0's 16 used
    // fragments (D-tiles 0..3 k-steps 0, 1; 4..7 k-steps 2, 3), W1 (T 16 + ks), WX (T 8 + ks), R (T 4 + ks); lo of
    // layer 0's 16, WX's 16, R's 8; then, read from global memory per step, lo of W1's 64.
    auto frag32 = [&](const SlotLayer& S, int T, int ks, int part, bool f16 = false) {
      for (int lane = 0; lane < 64; ++lane) {
        const int row = 32 * T + (lane & 31), h = lane >> 5;
        for (int j = 0; j < 8; ++j) {
          const int col = 32 * (ks / 2) + 8 * (2 * (ks % 2) + (j >> 2)) + 4 * h + (j & 3);
          const double w = S.W(row, col);
          uint16_t b = f16 ? f32_to_f16_rne((float)w) : f32_to_bf16_rne((float)w);
          if (f16 && part == 1) {
            b = f32_to_f16_rne((float)(w - f16_to_f64(b)));
          } else if (part == 1) {
            const uint32_t hu = (uint32_t)b << 16;
            float hf;
            std::memcpy(&hf, &hu, 4);
            b = f32_to_bf16_rne((float)(w - (double)hf));
          }
          img.push_back((unsigned char)(b & 0xFF));
          img.push_back((unsigned char)(b >> 8));
        }
      }
    };
    auto l0 = [&](int part) {
      for (int T = 0; T < 8; ++T)
        for (int ks = T < 4 ? 0 : 2; ks < (T < 4 ? 2 : 4); ++ks) frag32(*l0_x3, T, ks, part);
    };
    auto layer = [&](const SlotLayer& S, int part, bool f16 = false) {
      for (int T = 0; T < S.mto / 2; ++T)
        for (int ks = 0; ks < S.mti; ++ks) frag32(S, T, ks, part, f16);
    };
    align16();
    net.w32x3_off = (int)img.size();
    l0(0);
    layer(L[1], 0);
    layer(L[2], 0);
    layer(*r_x3, 0);
    l0(1);
    layer(L[2], 1);
    layer(*r_x3, 1);
    align16();
    net.w32x3_l1lo_off = (int)img.size();
    layer(L[1], 1);
    // ... and fc_wave32_x3p_kernel's fp16 form (fc_common.h x3_f16_on): the same LDS image with W1 as ONE fp16
    // fragment per (T, ks) in W1's hi place and the last layer's hi / lo as fp16 (lo = W - hi, itself rounded to fp16,
    // subnormals kept); layer 0 and the statistic factor as fp16 hi / lo too (MPPI_X3_F16_L0: against one fp16
    // operand), else unchanged
    auto l0f = [&](int part) {
      for (int T = 0; T < 8; ++T)
        for (int ks = T < 4 ? 0 : 2; ks < (T < 4 ? 2 : 4); ++ks) frag32(*l0_x3, T, ks, part, MPPI_X3_F16_L0 != 0);
    };
    align16();
    net.w32f16_off = (int)img.size();
    l0f(0);
    layer(L[1], 0, true);
    layer(L[2], 0, true);
    layer(*r_x3, 0, MPPI_X3_F16_L0 != 0);
    l0f(1);
    layer(L[2], 1, true);
    layer(*r_x3, 1, MPPI_X3_F16_L0 != 0);
    // ... and the M-split kernels' fp16 form (fc_rollout_kernel_x3d<F16>): layer 1 as one fp16 16x32 fragment per
    // (m-tile, k-step), the last layer and (MPPI_X3_F16_L0) the dense layer 0 as fp16 hi / lo (put_frags16)
    align16();
    net.wmf16_off = (int)img.size();
    put_frags16(L[1], 1);
    align16();
    net.wmf16_x_off = (int)img.size();
    put_frags16(L[2], 2);
    align16();
    net.wmf16_0_off = (int)img.size();
    put_frags16(L[0], 2);
    // ... and for fc_rollout_kernel_x3h the same with b0 in the pad column kCaX3hBiasSlot (the state holds 1.0 there)
    if (net.qp > 0 && net.qp <= kCaX3hBiasSlot) {
      SlotLayer L0b = L[0];
      for (int r = 0; r < 16 * L0b.mto; ++r) L0b.W(r, kCaX3hBiasSlot) = L0b.b[r];
      align16();
      net.wmf16_0b_off = (int)img.size();
      put_frags16(L0b, 2);
    }
  }
  if (mlp_x3) {
    // fc_wave_mlp_x3_kernel (split bf16 MLP, kernels_fc_x3m.hip): the per-wave bf16 kernel's 16x32 fragments (put_frags'
    // bf16 lane layout and (m-tile, k-step) order) as separate hi and lo (= W - hi, itself rounded) images.  LDS image:
    // hi of W0 | W1 | W2 | W3 (104 fragments), lo of W0 (24) and W3 (16); then, read from global memory per step, lo of
    // W1 and W2 (64).
    auto part_frags = [&](const SlotLayer& S, int part) {
      const int KS = S.mti / 2, KSB = KS / S.blocks, RPB = S.mto / S.blocks;
      for (int mt = 0; mt < S.mto; ++mt)
        for (int kk = 0; kk < KSB; ++kk) {
          const int ks = (S.blocks == 1 ? 0 : (mt / RPB) * KSB) + kk;
          for (int lane = 0; lane < 64; ++lane) {
            const int row = 16 * mt + (lane & 15);
            for (int j = 0; j < 8; ++j) {
              const int col = 32 * ks + 16 * (j >> 2) + 4 * (lane >> 4) + (j & 3);
              const double w = S.W(row, col);
              uint16_t h = f32_to_bf16_rne((float)w);
              if (part == 1) {
                const uint32_t hu = (uint32_t)h << 16;
                float hf;
                std::memcpy(&hf, &hu, 4);
                h = f32_to_bf16_rne((float)(w - (double)hf));
              }
              img.push_back((unsigned char)(h & 0xFF));
              img.push_back((unsigned char)(h >> 8));
            }
          }
        }
    };
    align16();
    net.wmx3_off = (int)img.size();
    for (size_t l = 0; l < 4; ++l) part_frags(L[l], 0);
    part_frags(L[0], 1);
    part_frags(L[3], 1);
    align16();
    net.wmx3_lo_off = (int)img.size();
    part_frags(L[1], 1);
    part_frags(L[2], 1);
    // ... and as 32x32x16 A fragments for fc_wave32_mlp_x3_kernel (32 samples per wave): lane l holds row 32 T + (l & 31)
    // at the k slots 8 (l >> 5) + j, input feature 32 (ks / 2) + 8 (2 (ks % 2) + (j >> 2)) + 4 (l >> 5) + (j & 3) (the
    // previous layer's 32x32 accumulator as it stands; layer 0's k-steps 4, 5 are the controls in that order).  LDS
    // image: hi of W0 (T 6 + ks) | W1 (T 8 + ks) | W2 | W3 (T 8 + ks), lo of W0 and W3; from global memory, lo of W1, W2.
    auto part32 = [&](const SlotLayer& S, int part) {
      for (int T = 0; T < S.mto / 2; ++T)
        for (int ks = 0; ks < S.mti; ++ks)
          for (int lane = 0; lane < 64; ++lane) {
            const int row = 32 * T + (lane & 31), hh = lane >> 5;
            for (int j = 0; j < 8; ++j) {
              const int col = 32 * (ks / 2) + 8 * (2 * (ks % 2) + (j >> 2)) + 4 * hh + (j & 3);
              const double w = S.W(row, col);
              uint16_t b = f32_to_bf16_rne((float)w);
              if (part == 1) {
                const uint32_t hu = (uint32_t)b << 16;
                float hf;
                std::memcpy(&hf, &hu, 4);
                b = f32_to_bf16_rne((float)(w - (double)hf));
              }
              img.push_back((unsigned char)(b & 0xFF));
              img.push_back((unsigned char)(b >> 8));
            }
          }
    };
    align16();
    net.wm32x3_off = (int)img.size();
    for (size_t l = 0; l < 4; ++l) part32(L[l], 0);
    part32(L[0], 1);
    part32(L[3], 1);
    align16();
    net.wm32x3_lo_off = (int)img.size();
    part32(L[1], 1);
    part32(L[2], 1);
  }
  align16();
  net.img_bytes = (int)img.size();
  net.reg_mask = reg_mask;
  return img;
}

// Slot index of original state feature i, and original feature of slot s (-1 = pad).
static int slot_of(const FcNet& n, int i) { return i < n.qp ? i : 32 + (i - n.qp); }
static int src_of(const FcNet& n, int s) {
  if (s < 32) return s < n.qp ? s : -1;
  return (s - 32) < n.qv ? n.qp + (s - 32) : -1;
}

static void pack_frags(std::vector<unsigned char>& img, const Mat& W, int precision);

// One dense layer of a net after folding, in the net's own coordinates (rows = outputs, cols = inputs).
struct DenseLayer {
  Mat W;
  std::vector<double> b;
  bool relu;
};

static bool env_on(const char* name) {
  const char* e = std::getenv(name);
  return e && e[0] == '1';
}

// learning/model.py:6-46 MLPStatePredictor in eval mode: the nn.Sequential's Linear layers in index order, each
// BatchNorm1d (use_batch_norm=True) folded into the Linear before it (y = (x - mean) / sqrt(var + 1e-5) * gamma + beta),
// ReLU after every Linear but the last; Dropout has no parameters.  Any hidden width and depth.
static std::vector<DenseLayer> mlp_layers(const TensorMap& T, int nx, int nu) {
  std::map<int, std::string> mods;  // module index -> "linear" | "bn"
  for (const auto& kv : T) {
    const std::string& k = kv.first;
    if (k.rfind("network.", 0) != 0) continue;
    const size_t dot = k.find('.', 8);
    if (dot == std::string::npos) continue;
    const int idx = std::atoi(k.substr(8, dot - 8).c_str());
    const std::string par = k.substr(dot + 1);
    if (par == "running_mean") mods[idx] = "bn";
    else if (par == "weight" && kv.second.shape.size() == 2 && !mods.count(idx)) mods[idx] = "linear";
  }
  std::vector<DenseLayer> L;
  for (const auto& m : mods) {
    const std::string p = "network." + std::to_string(m.first) + ".";
    auto it = T.find(p + "weight");
    if (m.second == "linear") {
      const Tensor& w = it->second;
      const int o = w.shape[0], i = w.shape[1];
      if (!L.empty() && L.back().W.r != i) throw std::runtime_error("MLP: layer widths do not chain");
      L.push_back(DenseLayer{from(w), vec(get(T, p + "bias", {o})), true});
    } else {
      if (L.empty()) throw std::runtime_error("MLP: BatchNorm before the first Linear");
      DenseLayer& d = L.back();
      const int o = d.W.r;
      const Tensor &ga = get(T, p + "weight", {o}), &be = get(T, p + "bias", {o});
      const Tensor &mu = get(T, p + "running_mean", {o}), &va = get(T, p + "running_var", {o});
      for (int r = 0; r < o; ++r) {
        const double sc = ga.v[r] / std::sqrt(va.v[r] + 1e-5);
        for (int c = 0; c < d.W.c; ++c) d.W(r, c) *= sc;
        d.b[r] = (d.b[r] - mu.v[r]) * sc + be.v[r];
      }
    }
  }
  if (L.size() < 2) throw std::runtime_error("MLP: needs at least two Linear layers");
  if (L.front().W.c != nx + nu || L.back().W.r != nx)
    throw std::runtime_error("MLP: input width must be state_dim + action_dim and output width state_dim");
  L.back().relu = false;
  return L;
}

// learning/model.py:157-202 CrossAttentionStatePredictor folded (oracle/nets_ref.py::ca_fold, ln_fold), any qpos /
// qvel / hidden width (the head count does not matter: attention over one key is the identity on the values):
//   layer 0: [x ; u] -> 2D rows, centred (mean 0 over the 2D rows for every input), gamma's sign folded in, then
//            y = relu(h rstd + beta'), rstd = 1 / sqrt(mean(h^2) + 1e-5)   (beta' returned)
//   layer 1: 2D -> D with |gamma| in its columns (a gamma = 0 row's constant relu(beta) folded into the bias), ReLU
//   layer 2: D -> nx.  The action encoder never reaches the output (its columns stay 0).
static std::vector<DenseLayer> ca_layers(const TensorMap& T, int nq, int nv, int na, int D, int nu,
                                         std::vector<double>& betap) {
  const int nx = nq + nv, in = nx + nu;
  auto lin = [&](const std::string& n, int r, int c) { return from(get(T, n + ".weight", {r, c})); };
  const Tensor& inw1 = get(T, "attn_qpos_to_qvel.in_proj_weight", {3 * D, D});
  const Tensor& inb1 = get(T, "attn_qpos_to_qvel.in_proj_bias", {3 * D});
  const Tensor& inw2 = get(T, "attn_qvel_to_qpos.in_proj_weight", {3 * D, D});
  const Tensor& inb2 = get(T, "attn_qvel_to_qpos.in_proj_bias", {3 * D});
  const Mat Wv1 = from(inw1, 2 * D, D), Wv2 = from(inw2, 2 * D, D);
  const Mat Wo1 = lin("attn_qpos_to_qvel.out_proj", D, D), Wo2 = lin("attn_qvel_to_qpos.out_proj", D, D);
  const Mat Wqp = lin("qpos_encoder", D, nq), Wqv = lin("qvel_encoder", D, nv);
  (void)get(T, "action_encoder.weight", {D, na});
  const Mat Aqv = matmul(matmul(Wo1, Wv1), Wqv), Aqp = matmul(matmul(Wo2, Wv2), Wqp);
  auto cvec = [&](const Mat& Wo, const Mat& Wv, const std::vector<double>& be, const Tensor& inb, const std::string& bo) {
    std::vector<double> t = matvec(Wv, be);
    for (int i = 0; i < D; ++i) t[i] += inb.v[2 * D + i];
    std::vector<double> c = matvec(Wo, t);
    const Tensor& bb = get(T, bo, {D});
    for (int i = 0; i < D; ++i) c[i] += bb.v[i];
    return c;
  };
  const std::vector<double> cqv = cvec(Wo1, Wv1, vec(get(T, "qvel_encoder.bias", {D})), inb1, "attn_qpos_to_qvel.out_proj.bias");
  const std::vector<double> cqp = cvec(Wo2, Wv2, vec(get(T, "qpos_encoder.bias", {D})), inb2, "attn_qvel_to_qpos.out_proj.bias");
  DenseLayer L0{Mat(2 * D, in), std::vector<double>(2 * D), true};
  for (int h = 0; h < D; ++h) {  // fused[:D] from qvel, fused[D:] from qpos (learning/model.py:199)
    for (int i = 0; i < nv; ++i) L0.W(h, nq + i) = Aqv(h, i);
    for (int i = 0; i < nq; ++i) L0.W(D + h, i) = Aqp(h, i);
    L0.b[h] = cqv[h];
    L0.b[D + h] = cqp[h];
  }
  DenseLayer L1{lin("fusion_layer.2", D, 2 * D), vec(get(T, "fusion_layer.2.bias", {D})), true};
  const Tensor& lg = get(T, "fusion_layer.0.weight", {2 * D});
  const Tensor& lb = get(T, "fusion_layer.0.bias", {2 * D});
  for (int c = 0; c < in; ++c) {  // centre the rows
    double m = 0.0;
    for (int h = 0; h < 2 * D; ++h) m += L0.W(h, c);
    for (int h = 0; h < 2 * D; ++h) L0.W(h, c) -= m / (2 * D);
  }
  double mb = 0.0;
  for (int h = 0; h < 2 * D; ++h) mb += L0.b[h];
  for (int h = 0; h < 2 * D; ++h) L0.b[h] -= mb / (2 * D);
  betap.assign(2 * D, 0.0);
  for (int h = 0; h < 2 * D; ++h) {
    const double ga = lg.v[h], be = lb.v[h];
    if (ga == 0.0) {
      for (int o = 0; o < D; ++o) {
        L1.b[o] += L1.W(o, h) * (be > 0.0 ? be : 0.0);
        L1.W(o, h) = 0.0;
      }
      continue;
    }
    if (ga < 0.0) {
      for (int c = 0; c < in; ++c) L0.W(h, c) = -L0.W(h, c);
      L0.b[h] = -L0.b[h];
    }
    betap[h] = be / std::fabs(ga);
    for (int o = 0; o < D; ++o) L1.W(o, h) *= std::fabs(ga);
  }
  DenseLayer L2{lin("fusion_layer.4", nx, D), vec(get(T, "fusion_layer.4.bias", {nx})), false};
  return {L0, L1, L2};
}

// The generic fc-stack image (kernels_fc_generic.hip): per layer the fragments of W padded to (16 mt, kin) and the
// fp32 bias padded to 16 mt; beta' of the folded LayerNorm (CA) after them.
static std::vector<unsigned char> build_generic(const std::vector<DenseLayer>& L, const std::vector<double>* betap,
                                                int precision, int nx, int nu, FcNet& net) {
  if ((int)L.size() > kGenMaxLayers) throw std::runtime_error("fc stack: more than 16 layers");
  net = FcNet();
  net.arch = kArchGeneric;
  net.precision = precision;
  FcGenNet& g = net.gen;
  g.nl = (int)L.size();
  std::vector<unsigned char> img;
  auto align16 = [&]() {
    while (img.size() % 16) img.push_back(0);
  };
  auto r32 = [](int v) { return (v + 31) / 32 * 32; };
  int maxw = 0;
  for (int l = 0; l < g.nl; ++l) {
    const DenseLayer& d = L[l];
    g.kin[l] = r32(d.W.c);
    g.mt[l] = (d.W.r + 15) / 16;
    maxw = std::max(maxw, std::max(g.kin[l], r32(d.W.r)));
    if (d.relu) g.relu_mask |= 1 << l;
    Mat P(16 * g.mt[l], g.kin[l]);
    for (int r = 0; r < d.W.r; ++r)
      for (int c = 0; c < d.W.c; ++c) P(r, c) = d.W(r, c);
    align16();
    g.w_off[l] = (int)img.size();
    pack_frags(img, P, precision);
  }
  if (maxw > (precision == MPPI_PREC_BF16 ? kGenMaxWidth : kGenMaxWidth / 2))
    throw std::runtime_error("fc stack: a layer wider than 1024 (fp32: 512)");
  g.maxw = maxw;
  auto put_f32 = [&](double v) {
    const float f = (float)v;
    unsigned char b[4];
    std::memcpy(b, &f, 4);
    img.insert(img.end(), b, b + 4);
  };
  for (int l = 0; l < g.nl; ++l) {
    align16();
    g.b_off[l] = (int)img.size();
    for (int r = 0; r < 16 * g.mt[l]; ++r) put_f32(r < (int)L[l].b.size() ? L[l].b[r] : 0.0);
  }
  if (betap) {
    align16();
    g.lnb_off = (int)img.size();
    g.ln_n = (int)betap->size();
    for (int r = 0; r < 16 * g.mt[0]; ++r) put_f32(r < (int)betap->size() ? (*betap)[r] : 0.0);
  }
  align16();
  net.img_bytes = (int)img.size();
  if (fc_generic_lds_bytes(g, precision, nx, nu) > 160 * 1024)
    throw std::runtime_error("fc stack: the activation rows do not fit the LDS");
  return img;
}

// Build the packed network for `kind` from a blob. Returns the host image; fills `net`.
std::vector<unsigned char> build_fc_net(int kind, const void* blob, size_t nbytes, int precision, int nx, int nu,
                                        FcNet& net) {
  int bkind = 0, dims[8];
  TensorMap T;
  parse_blob(blob, nbytes, &bkind, dims, T);
  if (bkind != kind) throw std::runtime_error("weight blob kind does not match mppi_load_dynamics kind");
  net = FcNet();
  net.precision = precision;
  std::vector<SlotLayer> L;

  if (kind == MPPI_DYN_CROSS_ATTN) {
    // learning/model.py:157-202 folded (oracle/nets_ref.py::ca_fold states the algebra).
    const int nq = dims[0], nv = dims[1], na = dims[2], D = dims[3];
    if (nq < 1 || nv < 0 || D < 1 || nq + nv != nx || na != nu)
      throw std::runtime_error("cross-attention: qpos_dim + qvel_dim must be state_dim (nx) and action_dim nu");
    if (D != 128 || nq != 28 || nv > 32 || env_on("MPPI_FC_GENERIC")) {  // any other shape: the generic kernel
      if (precision == MPPI_PREC_BF16X3)
        throw std::runtime_error("MPPI_PREC_BF16X3: built for the humanoid CA shape (28, 27, hidden 128) only");
      std::vector<double> betap;
      const std::vector<DenseLayer> L = ca_layers(T, nq, nv, na, D, nu, betap);
      return build_generic(L, &betap, precision, nx, nu, net);
    }
    net.arch = kArchCA;
    net.qp = nq;
    net.qv = nv;
    const Tensor& inw1 = get(T, "attn_qpos_to_qvel.in_proj_weight", {3 * D, D});
    const Tensor& inb1 = get(T, "attn_qpos_to_qvel.in_proj_bias", {3 * D});
    const Tensor& inw2 = get(T, "attn_qvel_to_qpos.in_proj_weight", {3 * D, D});
    const Tensor& inb2 = get(T, "attn_qvel_to_qpos.in_proj_bias", {3 * D});
    const Mat Wv1 = from(inw1, 2 * D, D), Wv2 = from(inw2, 2 * D, D);
    const std::vector<double> bv1 = vec(inb1, 2 * D, D), bv2 = vec(inb2, 2 * D, D);
    const Mat Wo1 = from(get(T, "attn_qpos_to_qvel.out_proj.weight", {D, D}));
    const Mat Wo2 = from(get(T, "attn_qvel_to_qpos.out_proj.weight", {D, D}));
    const std::vector<double> bo1 = vec(get(T, "attn_qpos_to_qvel.out_proj.bias", {D}));
    const std::vector<double> bo2 = vec(get(T, "attn_qvel_to_qpos.out_proj.bias", {D}));
    const Mat Wqp = from(get(T, "qpos_encoder.weight", {D, nq})), Wqv = from(get(T, "qvel_encoder.weight", {D, nv}));
    const std::vector<double> bqp = vec(get(T, "qpos_encoder.bias", {D})), bqv = vec(get(T, "qvel_encoder.bias", {D}));
    // fused[:D] = Wo1 Wv1 (Wqv qvel + bqv) + ... (depends on qvel);  fused[D:] depends on qpos.
    const Mat Aqv = matmul(matmul(Wo1, Wv1), Wqv);  // [D][nv]
    const Mat Aqp = matmul(matmul(Wo2, Wv2), Wqp);  // [D][nq]
    std::vector<double> cqv = matvec(Wo1, [&] {
      auto t = matvec(Wv1, bqv);
      for (int i = 0; i < D; ++i) t[i] += bv1[i];
      return t;
    }());
    std::vector<double> cqp = matvec(Wo2, [&] {
      auto t = matvec(Wv2, bqp);
      for (int i = 0; i < D; ++i) t[i] += bv2[i];
      return t;
    }());
    for (int i = 0; i < D; ++i) {
      cqv[i] += bo1[i];
      cqp[i] += bo2[i];
    }
    // Hidden order in the kernel: [qpos-fed rows (fused[D:]) | qvel-fed rows (fused[:D])] so that
    // rows [0,128) read only state slots [0,32) and rows [128,256) only [32,64) (block-diagonal).
    auto perm = [&](int h) { return h < D ? D + h : h - D; };  // kernel row h <- fused index
    SlotLayer L0{16, 4, Mat(256, 64), std::vector<double>(256, 0.0), 1};
    for (int h = 0; h < 2 * D; ++h) {
      const int f = perm(h);
      if (f < D) {  // qvel-fed
        for (int i = 0; i < nv; ++i) L0.W(h, slot_of(net, nq + i)) = Aqv(f, i);
        L0.b[h] = cqv[f];
      } else {
        for (int i = 0; i < nq; ++i) L0.W(h, slot_of(net, i)) = Aqp(f - D, i);
        L0.b[h] = cqp[f - D];
      }
    }
    const Tensor& lg = get(T, "fusion_layer.0.weight", {2 * D});
    const Tensor& lb = get(T, "fusion_layer.0.bias", {2 * D});
    const Tensor& w2 = get(T, "fusion_layer.2.weight", {D, 2 * D});
    SlotLayer L1{8, 16, Mat(128, 256), vec(get(T, "fusion_layer.2.bias", {D}))};
    for (int o = 0; o < D; ++o)
      for (int h = 0; h < 2 * D; ++h) L1.W(o, h) = w2.v[(size_t)o * 2 * D + perm(h)];
    // LayerNorm folded into the weights (exact in fp64; oracle/nets_ref.py::ln_fold states it):
    //  * layer 0 centred: W0 -= 1 (1^T W0)/256, b0 -= mean(b0), so the 256 rows have mean 0 for every input and
    //    LN's (h - mean) is h itself; rows with gamma < 0 are negated (the variance is sign-blind);
    //  * relu(gamma z + beta) = |gamma| relu(s z + beta/|gamma|): |gamma| goes into W1's columns, beta' = beta/|gamma|;
    //    a row with gamma = 0 outputs the constant relu(beta): folded into b1, its W1 column zeroed.
    // The kernel then evaluates y = relu(h rstd + beta'), rstd = rsqrt(mean(h^2) + 1e-5).
    std::vector<double> ln_b(256, 0.0);
    const SlotLayer L0u = L0;  // uncentred (fc_wave32_kernel's block-diagonal layer 0)
    {
      for (int s = 0; s < 64; ++s) {
        double m = 0.0;
        for (int h = 0; h < 2 * D; ++h) m += L0.W(h, s);
        m /= 2 * D;
        for (int h = 0; h < 2 * D; ++h) L0.W(h, s) -= m;
      }
      double mb = 0.0;
      for (int h = 0; h < 2 * D; ++h) mb += L0.b[h];
      mb /= 2 * D;
      for (int h = 0; h < 2 * D; ++h) L0.b[h] -= mb;
      for (int h = 0; h < 2 * D; ++h) {
        const double g = lg.v[perm(h)], be = lb.v[perm(h)];
        if (g == 0.0) {
          for (int o = 0; o < D; ++o) {
            L1.b[o] += L1.W(o, h) * (be > 0.0 ? be : 0.0);
            L1.W(o, h) = 0.0;
          }
          continue;
        }
        if (g < 0.0) {
          for (int s = 0; s < 64; ++s) L0.W(h, s) = -L0.W(h, s);
          L0.b[h] = -L0.b[h];
        }
        const double ag = std::fabs(g);
        ln_b[h] = be / ag;
        for (int o = 0; o < D; ++o) L1.W(o, h) *= ag;
      }
    }
    const Tensor& w3 = get(T, "fusion_layer.4.weight", {nx, D});
    const Tensor& b3 = get(T, "fusion_layer.4.bias", {nx});
    SlotLayer L2{4, 8, Mat(64, 128), std::vector<double>(64, 0.0)};
    for (int s = 0; s < 64; ++s) {
      const int src = src_of(net, s);
      if (src < 0) continue;
      for (int h = 0; h < D; ++h) L2.W(s, h) = w3.v[(size_t)src * D + h];
      L2.b[s] = b3.v[src];
    }
    if (precision == MPPI_PREC_BF16 && nq <= kCaBiasSlotHi) {
      // b0 as a bf16 hi / lo pair in the pad slots 28, 29 (exact to ~2^-16 of |b0|), for fc_pipe_kernel's 1.0 there
      for (int h = 0; h < 2 * D; ++h) {
        uint32_t u;
        const float bh = (float)L0.b[h];
        std::memcpy(&u, &bh, 4);
        const uint16_t hb = f32_to_bf16_rne(bh);
        const uint32_t hu = (uint32_t)hb << 16;
        float hi;
        std::memcpy(&hi, &hu, 4);
        L0.W(h, kCaBiasSlotHi) = hi;
        L0.W(h, kCaBiasSlotLo) = L0.b[h] - (double)hi;
      }
    }
    std::vector<SlotLayer> gram;
    if (precision == MPPI_PREC_BF16 && nq <= kCaBiasSlotHi && nv <= kCaBetaSlotHi1 - 32) {
      // the per-wave kernel (kernels_fc_wave.hip) evaluates the folded LayerNorm as relu(h + beta' s) rstd, with
      // rstd = 1/s = rsqrt(mean(h^2) + eps) known BEFORE layer 0 from the Gram matrix: mean(h^2) = x~^T G x~ / n,
      // G = W~^T W~ over the bf16 layer-0 columns it multiplies (state slots, the b0 pair; x~ = the bf16 operand with
      // 1.0 in the b0 slots), as |R x~|^2 with G's Cholesky factor R (hi / lo bf16 fragments at g_off).  beta' rides in
      // the MFMA as a hi / lo pair against (s_hi, s_hi, s_lo) in pad slots.
      for (int h = 0; h < 2 * D; ++h) {
        const uint16_t hb = f32_to_bf16_rne((float)ln_b[h]);
        const uint32_t hu = (uint32_t)hb << 16;
        float hi;
        std::memcpy(&hi, &hu, 4);
        L0.W(h, kCaBetaSlotHi0) = hi;
        L0.W(h, kCaBetaSlotLo) = ln_b[h] - (double)hi;
        L0.W(h, kCaBetaSlotHi1) = hi;
      }
      Mat Wt(2 * D, 64);
      std::vector<int> var;  // the slots the kernel multiplies (state slots and the b0 pair), in slot order
      for (int c = 0; c < 64; ++c)
        if (src_of(net, c) >= 0 || c == kCaBiasSlotHi || c == kCaBiasSlotLo) var.push_back(c);
      for (int h = 0; h < 2 * D; ++h)
        for (int c : var) {
          const uint32_t wu = (uint32_t)f32_to_bf16_rne((float)L0.W(h, c)) << 16;
          float w;
          std::memcpy(&w, &wu, 4);
          Wt(h, c) = w;
        }
      // Cholesky factor of the Gram matrix in slot order, G = W~^T W~ = R^T R with R upper triangular, so that
      // mean(h^2) = |R x~|^2 / n and R's rows 32.. (the qvel slots) read only slots 32..: the kernel's m-tiles 2, 3
      // skip k-step 0
      const int nv_ = (int)var.size();
      Mat Gv(nv_, nv_), Lc(nv_, nv_);
      for (int i = 0; i < nv_; ++i)
        for (int j = 0; j < nv_; ++j) {
          double g = 0.0;
          for (int h = 0; h < 2 * D; ++h) g += Wt(h, var[i]) * Wt(h, var[j]);
          Gv(i, j) = g;
        }
      for (int j = 0; j < nv_; ++j) {
        double d = Gv(j, j);
        for (int k = 0; k < j; ++k) d -= Lc(j, k) * Lc(j, k);
        if (!(d > 0.0)) throw std::runtime_error("CROSS_ATTN: layer-0 Gram matrix not positive definite");
        Lc(j, j) = std::sqrt(d);
        for (int i = j + 1; i < nv_; ++i) {
          double v = Gv(i, j);
          for (int k = 0; k < j; ++k) v -= Lc(i, k) * Lc(j, k);
          Lc(i, j) = v / Lc(j, j);
        }
      }
      SlotLayer Gh{4, 4, Mat(64, 64), std::vector<double>(64, 0.0)}, Gl = Gh;
      for (int i = 0; i < nv_; ++i)
        for (int j = i; j < nv_; ++j) {  // R(i, j) = L(j, i), row i at slot var[i]
          const double r = Lc(j, i);
          const uint32_t ru = (uint32_t)f32_to_bf16_rne((float)r) << 16;
          float rhi;
          std::memcpy(&rhi, &ru, 4);
          Gh.W(var[i], var[j]) = rhi;
          Gl.W(var[i], var[j]) = r - (double)rhi;
        }
      gram = {Gh, Gl};
    }
    // fc_wave32_kernel's block-diagonal layer 0 (every gamma > 0, so no row is negated; MPPI_W32_BD=0 at load keeps
    // the dense form for A/B).  The fold above centres the rows, which mixes the qpos and qvel columns into every
    // row: 32 MFMAs per wave-step.  Uncentred, rows [0,128) read slots [0,32) and rows [128,256) slots [32,64): the
    // kernel subtracts the row mean mu = m~ x~ itself (its accumulators start at -mu), m~ = the mean of the bf16
    // rows, computed by the statistic MFMAs as row 30 of the Gram factor, whose other rows factor the Gram matrix of
    // the centred rows (bf16 W0 - 1 m~^T, the b0c pair): the same variance, 112 MFMAs per wave-step instead of 124.
    // Pads: qpos rows b0c 28, 29, beta' 30, 31 (s_hi), 59 (s_lo, k-step 3); qvel rows 59, b0c 60, 61, beta' 62, 63.
    // Form 2 (the default, 108 MFMAs): the qpos rows take b0c through their accumulators (the kernel adds the fp32
    // image bias, LDS) and their beta' s terms in slots 29 (s_lo), 30, 31 (s_hi), so they skip k-step 3.
    // MPPI_W32_BD=1 keeps form 1, =0 the dense layer 0 (read at load, for A/B).
    SlotLayer L0bd{16, 4, Mat(256, 64), std::vector<double>(256, 0.0), 1};
    std::vector<SlotLayer> gram_bd;
    bool bd = !gram.empty();
    for (int h = 0; h < 2 * D && bd; ++h) bd = lg.v[perm(h)] > 0.0f;
    int bd_form = 2;
    if (const char* e = std::getenv("MPPI_W32_BD")) bd_form = e[0] == '0' ? 0 : (e[0] == '1' ? 1 : 2);
    bd = bd && bd_form != 0;
    if (bd) {
      auto bf = [](double v) {
        const uint32_t u = (uint32_t)f32_to_bf16_rne((float)v) << 16;
        float f;
        std::memcpy(&f, &u, 4);
        return (double)f;
      };
      std::vector<int> st;  // state slots
      for (int c = 0; c < 64; ++c)
        if (src_of(net, c) >= 0) st.push_back(c);
      std::vector<double> mt(64, 0.0);  // m~: row mean of the bf16 uncentred layer 0
      for (int c : st) {
        for (int h = 0; h < 2 * D; ++h) mt[c] += bf(L0u.W(h, c));
        mt[c] /= 2 * D;
      }
      for (int h = 0; h < 2 * D; ++h) {
        const bool qp_row = h < D;  // kernel rows [0, D) read the qpos slots (perm above)
        for (int c : st)
          if ((c < 32) == qp_row) L0bd.W(h, c) = bf(L0u.W(h, c));
        const double b0c = L0.b[h], bh = bf(b0c), be = ln_b[h], beh = bf(be);
        if (qp_row && bd_form == 2) {  // b0c from the accumulators; slot 29 holds s_lo
          L0bd.W(h, kCaBiasSlotLo) = beh;
          L0bd.W(h, kCaBetaSlotHi0) = beh;
          L0bd.W(h, kCaBetaSlotLo) = be - beh;
          continue;
        }
        L0bd.W(h, qp_row ? kCaBiasSlotHi : kCaBdBiasSlotHi) = bh;
        L0bd.W(h, qp_row ? kCaBiasSlotLo : kCaBdBiasSlotLo) = b0c - bh;
        L0bd.W(h, qp_row ? kCaBetaSlotHi0 : kCaBdBetaSlotHi) = beh;
        L0bd.W(h, qp_row ? kCaBetaSlotLo : kCaBdBetaSlotLo) = be - beh;
        L0bd.W(h, kCaBetaSlotHi1) = beh;
      }
      // Gram factor of the centred rows as the kernel evaluates them (statistic operand: state, 1.0 in 28, 29)
      std::vector<int> var = st;
      var.push_back(kCaBiasSlotHi);
      var.push_back(kCaBiasSlotLo);
      std::sort(var.begin(), var.end());
      const int nv_ = (int)var.size();
      Mat Wc(2 * D, 64);
      for (int h = 0; h < 2 * D; ++h) {
        const bool qp_row = h < D;
        for (int c : st) Wc(h, c) = ((c < 32) == qp_row ? bf(L0u.W(h, c)) : 0.0) - mt[c];
        Wc(h, kCaBiasSlotHi) = bf(L0.b[h]);
        Wc(h, kCaBiasSlotLo) = bf(L0.b[h] - bf(L0.b[h]));
      }
      Mat Gv(nv_, nv_), Lc(nv_, nv_);
      for (int i = 0; i < nv_; ++i)
        for (int j = 0; j < nv_; ++j) {
          double g = 0.0;
          for (int h = 0; h < 2 * D; ++h) g += Wc(h, var[i]) * Wc(h, var[j]);
          Gv(i, j) = g;
        }
      for (int j = 0; j < nv_ && bd; ++j) {
        double d = Gv(j, j);
        for (int k = 0; k < j; ++k) d -= Lc(j, k) * Lc(j, k);
        if (!(d > 0.0)) {
          bd = false;  // not positive definite: keep the dense form
          break;
        }
        Lc(j, j) = std::sqrt(d);
        for (int i = j + 1; i < nv_; ++i) {
          double v = Gv(i, j);
          for (int k = 0; k < j; ++k) v -= Lc(i, k) * Lc(j, k);
          Lc(i, j) = v / Lc(j, j);
        }
      }
      if (bd) {
        SlotLayer Gh{4, 4, Mat(64, 64), std::vector<double>(64, 0.0)}, Gl = Gh;
        for (int i = 0; i < nv_; ++i)
          for (int j = i; j < nv_; ++j) {
            const double r = Lc(j, i), rh = bf(r);
            Gh.W(var[i], var[j]) = rh;
            Gl.W(var[i], var[j]) = r - rh;
          }
        for (int c : st) {  // row 30: m~ (a pad row: slot 30 is not in var)
          Gh.W(kCaBdMeanRow, c) = bf(mt[c]);
          Gl.W(kCaBdMeanRow, c) = mt[c] - bf(mt[c]);
        }
        gram_bd = {Gh, Gl};
      }
    }
    // Split bf16 (MPPI_PREC_BF16X3), per-wave kernel (fc_wave32_x3_kernel): the block-diagonal, uncentred layer 0 in
    // fp64 (the kernel's three products keep ~16 bits of every weight and operand), b0c against 1.0 in slot 28 (qpos
    // rows) / 60 (qvel rows), beta' against s in slot 30 / 62 (the kernel splits s into hi / lo like any operand);
    // the row mean m~ (exact) as row 30 of the Gram factor of the centred rows (state slots, the b0c column 28).
    SlotLayer L0x{16, 4, Mat(256, 64), std::vector<double>(256, 0.0), 1}, Rx{4, 4, Mat(64, 64), std::vector<double>(64, 0.0)};
    bool x3w = precision == MPPI_PREC_BF16X3 && nq <= kCaBiasSlotHi && nv <= kCaBetaSlotHi1 - 32;
    for (int h = 0; h < 2 * D && x3w; ++h) x3w = lg.v[perm(h)] > 0.0f;
    if (const char* e = std::getenv("MPPI_X3_WAVE")) x3w = x3w && e[0] != '0';
    if (x3w) {
      std::vector<int> st;
      for (int c = 0; c < 64; ++c)
        if (src_of(net, c) >= 0) st.push_back(c);
      std::vector<double> mt(64, 0.0);
      for (int c : st) {
        for (int h = 0; h < 2 * D; ++h) mt[c] += L0u.W(h, c);
        mt[c] /= 2 * D;
      }
      for (int h = 0; h < 2 * D; ++h) {
        const bool qp_row = h < D;
        for (int c : st)
          if ((c < 32) == qp_row) L0x.W(h, c) = L0u.W(h, c);
        L0x.W(h, qp_row ? kCaBiasSlotHi : kCaBdBiasSlotHi) = L0.b[h];   // b0c (centred) against 1.0
        L0x.W(h, qp_row ? kCaBetaSlotHi0 : kCaBdBetaSlotHi) = ln_b[h];  // beta' against s
        L0x.W(h, qp_row ? kCaX3MeanSlot : kCaX3BdMeanSlot) = 1.0;      // against -mu (x3p; 0 in the x3 kernel)
        L0x.W(h, qp_row ? kCaX3MeanLoSlot : kCaX3BdMeanLoSlot) = 1.0;  // ... its lo part (x3p's fp16 form; else 0)
      }
      std::vector<int> var = st;
      var.push_back(kCaBiasSlotHi);
      std::sort(var.begin(), var.end());
      const int nv_ = (int)var.size();
      Mat Wc(2 * D, 64);
      for (int h = 0; h < 2 * D; ++h) {
        const bool qp_row = h < D;
        for (int c : st) Wc(h, c) = ((c < 32) == qp_row ? L0u.W(h, c) : 0.0) - mt[c];
        Wc(h, kCaBiasSlotHi) = L0.b[h];
      }
      Mat Gv(nv_, nv_), Lc(nv_, nv_);
      for (int i = 0; i < nv_; ++i)
        for (int j = 0; j < nv_; ++j) {
          double g = 0.0;
          for (int h = 0; h < 2 * D; ++h) g += Wc(h, var[i]) * Wc(h, var[j]);
          Gv(i, j) = g;
        }
      for (int j = 0; j < nv_ && x3w; ++j) {
        double d = Gv(j, j);
        for (int k = 0; k < j; ++k) d -= Lc(j, k) * Lc(j, k);
        if (!(d > 0.0)) {
          x3w = false;
          break;
        }
        Lc(j, j) = std::sqrt(d);
        for (int i = j + 1; i < nv_; ++i) {
          double v = Gv(i, j);
          for (int k = 0; k < j; ++k) v -= Lc(i, k) * Lc(j, k);
          Lc(i, j) = v / Lc(j, j);
        }
      }
      if (x3w) {
        for (int i = 0; i < nv_; ++i)
          for (int j = i; j < nv_; ++j) Rx.W(var[i], var[j]) = Lc(j, i);
        for (int c : st) Rx.W(kCaBdMeanRow, c) = mt[c];
      }
    }
    L = {L0, L1, L2};
    net.ln_n = 2 * D;
    net.wave = gram.empty() ? 0 : 1;
    net.w32_bd = bd ? bd_form : 0;  // (pack_image reads it: the 16x16 copies of form 2)
    return pack_image(L, &ln_b, precision, kCaRegMask, net, gram.empty() ? nullptr : &gram, bd ? &L0bd : nullptr,
                      bd ? &gram_bd : nullptr, x3w ? &L0x : nullptr, x3w ? &Rx : nullptr);
  }

  if (kind == MPPI_DYN_MLP) {
    // learning/model.py:6-46 (any depth / width; BatchNorm folded): Linear(nx+nu, h) ReLU, hidden_layers x
    // [Linear(h,h) ReLU], Linear(h, nx).  The register-resident kernel takes h = 128 with 2 hidden layers.
    const int sd = dims[0], ad = dims[1];
    if (sd != nx || ad != nu) throw std::runtime_error("MLP: state_dim / action_dim differ from the config");
    const std::vector<DenseLayer> M = mlp_layers(T, nx, nu);
    const bool spec = M.size() == 4 && M[0].W.r == 128 && M[1].W.r == 128 && M[2].W.r == 128 && nx <= 64 && nu <= 32;
    if (!spec || env_on("MPPI_FC_GENERIC")) {
      if (precision == MPPI_PREC_BF16X3)
        throw std::runtime_error("MPPI_PREC_BF16X3: built for MLPs of hidden 128 x 2 (nx <= 64, nu <= 32) only");
      return build_generic(M, nullptr, precision, nx, nu, net);
    }
    const int h = 128;
    net.arch = kArchMLP;
    net.qp = nx < 32 ? nx : 32;
    net.qv = nx - net.qp;
    SlotLayer L0{8, 6, Mat(128, 96), M[0].b};
    for (int o = 0; o < h; ++o) {
      for (int s2 = 0; s2 < 64; ++s2) {
        const int src = src_of(net, s2);
        if (src >= 0) L0.W(o, s2) = M[0].W(o, src);
      }
      for (int j = 0; j < nu; ++j) L0.W(o, 64 + j) = M[0].W(o, nx + j);
    }
    SlotLayer L1{8, 8, M[1].W, M[1].b};
    SlotLayer L2{8, 8, M[2].W, M[2].b};
    SlotLayer L3{4, 8, Mat(64, 128), std::vector<double>(64, 0.0)};
    for (int s2 = 0; s2 < 64; ++s2) {
      const int src = src_of(net, s2);
      if (src < 0) continue;
      for (int k = 0; k < h; ++k) L3.W(s2, k) = M[3].W(src, k);
      L3.b[s2] = M[3].b[src];
    }
    const bool wave_ok = nx <= kMlpBiasSlotHi && nu <= 32;
    if ((precision == MPPI_PREC_BF16 || precision == MPPI_PREC_BF16X3) && wave_ok) {
      // b0 as a bf16 hi / lo pair in the pad state columns 62, 63 (their last-layer rows are 0): the per-wave kernels
      // hold 1.0 there and get W0 [x; u] + b0 from the MFMA alone (the M-split kernels hold 0 there and add b0)
      for (int o = 0; o < h; ++o) {
        const uint32_t hu = (uint32_t)f32_to_bf16_rne((float)L0.b[o]) << 16;
        float hi;
        std::memcpy(&hi, &hu, 4);
        L0.W(o, kMlpBiasSlotHi) = hi;
        L0.W(o, kMlpBiasSlotLo) = L0.b[o] - (double)hi;
      }
      net.wave = precision == MPPI_PREC_BF16 ? 1 : 0;
    }
    L = {L0, L1, L2, L3};
    return pack_image(L, nullptr, precision, kMlpRegMask, net, nullptr, nullptr, nullptr, nullptr, nullptr,
                      precision == MPPI_PREC_BF16X3 && wave_ok);
  }
  throw std::runtime_error("unsupported dynamics kind for an fc stack");
}

// ------------------------------------------------------------------------------------------- feature attention

// Pack W [M][K] (M % 16 == 0, K % 32 == 0) as MFMA A fragments, fragment (mt, kb) at (mt * K/32 + kb) * FRAG
// (kernels_fa.hip::fa_gemm).  bf16 lane l: W[16mt + (l&15)][32kb + 8(l>>4) + e], e < 8.
// fp32 lane l: W[16mt + (l&15)][32kb + 16h + 4(l>>4) + m], h < 2, m < 4 (h-major).
static void pack_frags(std::vector<unsigned char>& img, const Mat& W, int precision) {
  if (W.r % 16 || W.c % 32) throw std::runtime_error("pack_frags: shape not a multiple of the 16x32 fragment");
  auto put_f32 = [&](float f) {
    unsigned char b[4];
    std::memcpy(b, &f, 4);
    img.insert(img.end(), b, b + 4);
  };
  for (int mt = 0; mt < W.r / 16; ++mt)
    for (int kb = 0; kb < W.c / 32; ++kb)
      for (int lane = 0; lane < 64; ++lane) {
        const int row = 16 * mt + (lane & 15), g = lane >> 4;
        if (precision == MPPI_PREC_BF16) {
          for (int e = 0; e < 8; ++e) {
            const uint16_t h = f32_to_bf16_rne((float)W(row, 32 * kb + 8 * g + e));
            img.push_back((unsigned char)(h & 0xFF));
            img.push_back((unsigned char)(h >> 8));
          }
        } else {
          for (int hh = 0; hh < 2; ++hh)
            for (int m = 0; m < 4; ++m) put_f32((float)W(row, 32 * kb + 16 * hh + 4 * g + m));
        }
      }
}

// Small-net kernel packing (kernels_fa.hip::fa_small_kernel).  Its GEMM inputs that come from registers (the
// LayerNorm outputs, the FFN hidden slice) hold, in lane group g of k-block kb, the features of the two 16-row MFMA
// accumulator tiles 2kb and 2kb+1: element e <-> feature 32kb + 16(e >> 2) + 4g + (e & 3).  The A fragments of the
// matrices they multiply are packed in that k order (bf16): lane l = row 16mt + (l & 15).
static int small_k(int kb, int g, int e) { return 32 * kb + 16 * (e >> 2) + 4 * g + (e & 3); }
static void put_bf16(std::vector<unsigned char>& img, double v) {
  const uint16_t h = f32_to_bf16_rne((float)v);
  img.push_back((unsigned char)(h & 0xFF));
  img.push_back((unsigned char)(h >> 8));
}
// fragment (rows [r0, r0+16), k-block kb) of W in the register-operand k order, 1 KB
static void pack_frag_perm(std::vector<unsigned char>& img, const Mat& W, int r0, int kb) {
  for (int lane = 0; lane < 64; ++lane)
    for (int e = 0; e < 8; ++e) put_bf16(img, W(r0 + (lane & 15), small_k(kb, lane >> 4, e)));
}

// learning/model.py:48-153.  dims = {state_dim, action_dim, hidden_dim, num_heads, attn_layers}.
// Image: fp32 vectors (encoding w/b, LN gamma/beta, pos_embedding [L][D], biases, output weights), then per
// layer the packed matrices, chunked as the kernel consumes them:
//   Wqkv: for each attention chunk c (fa_cw(D) columns = whole heads): [Wq_c * s; Wk_c; Wv_c]  (3*CW x D),
//         s = 1/sqrt(head_dim) (torch scales q after the in-projection, bias included)
//   Wo:   for each chunk c: Wo[:, c*CW:(c+1)*CW]  (D x CW)
//   W1:   for each FFN chunk f: W1[f*FC:(f+1)*FC, :]  (FC x D);  W2: W2[:, f*FC:(f+1)*FC]  (D x FC)
std::vector<unsigned char> build_fa_net(const void* blob, size_t nbytes, int precision, int nx, int nu, FaNet& net) {
  int bkind = 0, dims[8];
  TensorMap T;
  parse_blob(blob, nbytes, &bkind, dims, T);
  if (bkind != MPPI_DYN_FEATURE_ATTN) throw std::runtime_error("weight blob kind does not match mppi_load_dynamics kind");
  const int sd = dims[0], ad = dims[1], D = dims[2], nh = dims[3], nl = dims[4];
  const int L = sd + ad;
  if (sd != nx || ad != nu) throw std::runtime_error("feature attention: state/action dims differ from the config");
  if ((nh != 4 && nh != 8) || D % nh != 0) throw std::runtime_error("feature attention: num_heads 4 or 8");
  if (!(D == 64 || D == 128 || D == 512) || (precision == MPPI_PREC_FP32 && D != 64))
    throw std::runtime_error("feature attention: hidden_dim 64 (fp32|bf16), 128 or 512 (bf16)");
  if (L > kFaRows || (D == 512 && L > 64))
    throw std::runtime_error("feature attention: state_dim + action_dim must be <= 80 (hidden 512: <= 64)");
  if (nl < 1 || nl > kFaMaxLayers) throw std::runtime_error("feature attention: 1..8 attention layers");
  net = FaNet();
  net.D = D;
  net.L = L;
  net.nlayers = nl;
  net.nh = nh;
  net.precision = precision;
  const int HD = D / nh, CW = fa_cw(D, nh, fa_nt_min(L)), FC = fa_fc(D), F4 = 4 * D;
  const double qs = 1.0 / std::sqrt((double)HD);

  std::vector<unsigned char> img;
  auto align16 = [&]() {
    while (img.size() % 16) img.push_back(0);
  };
  auto put_vec = [&](const std::vector<double>& v) {
    align16();
    const int off = (int)img.size();
    for (double x : v) {
      const float f = (float)x;
      unsigned char b[4];
      std::memcpy(b, &f, 4);
      img.insert(img.end(), b, b + 4);
    }
    return off;
  };
  const Tensor& we = get(T, "feature_encoding.0.weight", {D, 1});
  const Tensor& be = get(T, "feature_encoding.0.bias", {D});
  net.we = put_vec(vec(we));
  net.be = put_vec(vec(be));
  net.ge = put_vec(vec(get(T, "feature_encoding.1.weight", {D})));
  net.bte = put_vec(vec(get(T, "feature_encoding.1.bias", {D})));
  net.pos = put_vec(vec(get(T, "pos_embedding", {1, L, D})));
  net.wout = put_vec(vec(get(T, "output_layer.weight", {1, D})));
  net.b_out = (float)get(T, "output_layer.bias", {1}).v[0];
  {  // population moments of h_f = w_f v + b_f over f: mean = v mw + mb, var = v^2 vw + 2 v cwb + vb
    double mw = 0, mb = 0;
    for (int i = 0; i < D; ++i) {
      mw += we.v[i];
      mb += be.v[i];
    }
    mw /= D;
    mb /= D;
    double vw = 0, vb = 0, cwb = 0;
    for (int i = 0; i < D; ++i) {
      vw += (we.v[i] - mw) * (we.v[i] - mw);
      vb += (be.v[i] - mb) * (be.v[i] - mb);
      cwb += (we.v[i] - mw) * (be.v[i] - mb);
    }
    net.enc_mw = (float)mw;
    net.enc_mb = (float)mb;
    net.enc_vw = (float)(vw / D);
    net.enc_vb = (float)(vb / D);
    net.enc_cwb = (float)(cwb / D);
    // small-net kernel: LN(w v + b) gamma = rstd(v) (v c1 + c2), c1 = (w - mean w) gamma, c2 = (b - mean b) gamma
    const Tensor& ge = get(T, "feature_encoding.1.weight", {D});
    std::vector<double> c1(D), c2(D);
    for (int i = 0; i < D; ++i) {
      c1[i] = (we.v[i] - mw) * ge.v[i];
      c2[i] = (be.v[i] - mb) * ge.v[i];
    }
    net.s_c1 = put_vec(c1);
    net.s_c2 = put_vec(c2);
  }
  std::vector<Mat> Wqkv(nl), Wo(nl), W1(nl), W2(nl);
  // small-net kernel (bf16, hidden 64, L <= 16): the LayerNorm affine maps folded into the GEMM that follows each
  // LayerNorm (its LayerNorms output (x - mean) rstd): W' = W diag(gamma), b' = b + W beta for Q|K|V (LN1) and FFN1
  // (LN2); the folded biases s_bqkv / s_b1 are fp32 vectors, so they join the image's vector prefix here
  const bool small = precision == MPPI_PREC_BF16 && D == 64 && L <= 16 && nh == kFaHeads && nl <= 4;
  std::vector<Mat> s_qf(nl), s_w1f(nl);
  auto fold = [&](const Mat& W, const std::vector<double>& bias, const Tensor& ga, const Tensor& bt, Mat& Wf) {
    Wf = W;
    std::vector<double> bf = bias;
    for (int r = 0; r < W.r; ++r)
      for (int k = 0; k < W.c; ++k) {
        Wf(r, k) = W(r, k) * ga.v[k];
        bf[r] += W(r, k) * bt.v[k];
      }
    return put_vec(bf);
  };
  for (int l = 0; l < nl; ++l) {
    const std::string p = "layers." + std::to_string(l) + ".";
    net.ln1g[l] = put_vec(vec(get(T, p + "norm1.weight", {D})));
    net.ln1b[l] = put_vec(vec(get(T, p + "norm1.bias", {D})));
    const Tensor& inw = get(T, p + "attention.in_proj_weight", {3 * D, D});
    const Tensor& inb = get(T, p + "attention.in_proj_bias", {3 * D});
    Mat q(3 * D, D);
    std::vector<double> bq(3 * D);
    for (int c = 0; c < D / CW; ++c)
      for (int part = 0; part < 3; ++part)
        for (int rr = 0; rr < CW; ++rr) {
          const int src = part * D + c * CW + rr, dst = c * 3 * CW + part * CW + rr;
          const double sc = part == 0 ? qs : 1.0;
          for (int k = 0; k < D; ++k) q(dst, k) = sc * inw.v[(size_t)src * D + k];
          bq[dst] = sc * inb.v[src];
        }
    Wqkv[l] = q;
    net.bqkv[l] = put_vec(bq);
    if (small) net.s_bqkv[l] = fold(q, bq, get(T, p + "norm1.weight", {D}), get(T, p + "norm1.bias", {D}), s_qf[l]);
    const Tensor& wo = get(T, p + "attention.out_proj.weight", {D, D});
    Mat o(D, D);  // chunk-major: rows of chunk c's (D x CW) block stacked
    for (int c = 0; c < D / CW; ++c)
      for (int r = 0; r < D; ++r)
        for (int k = 0; k < CW; ++k) o.a[((size_t)c * D + r) * CW + k] = wo.v[(size_t)r * D + c * CW + k];
    o.r = D * (D / CW);
    o.c = CW;
    Wo[l] = o;
    net.bo[l] = put_vec(vec(get(T, p + "attention.out_proj.bias", {D})));
    net.ln2g[l] = put_vec(vec(get(T, p + "norm2.weight", {D})));
    net.ln2b[l] = put_vec(vec(get(T, p + "norm2.bias", {D})));
    W1[l] = from(get(T, p + "ffn.0.weight", {F4, D}));  // row chunks are contiguous already
    net.b1[l] = put_vec(vec(get(T, p + "ffn.0.bias", {F4})));
    if (small)
      net.s_b1[l] = fold(W1[l], vec(get(T, p + "ffn.0.bias", {F4})), get(T, p + "norm2.weight", {D}),
                         get(T, p + "norm2.bias", {D}), s_w1f[l]);
    const Tensor& w2 = get(T, p + "ffn.3.weight", {D, F4});
    Mat m2(D * (F4 / FC), FC);
    for (int fc = 0; fc < F4 / FC; ++fc)
      for (int r = 0; r < D; ++r)
        for (int k = 0; k < FC; ++k) m2.a[((size_t)fc * D + r) * FC + k] = w2.v[(size_t)r * F4 + fc * FC + k];
    W2[l] = m2;
    net.b2[l] = put_vec(vec(get(T, p + "ffn.3.bias", {D})));
  }
  // Matrices: a stacked chunk matrix packs as consecutive fragment blocks, exactly the per-chunk offsets the
  // kernel computes (chunk c of Wqkv at c * (3CW/16) * (D/32) fragments, etc.).
  for (int l = 0; l < nl; ++l) {
    align16();
    net.wqkv[l] = (int)img.size();
    pack_frags(img, Wqkv[l], precision);
    align16();
    net.wo[l] = (int)img.size();
    pack_frags(img, Wo[l], precision);
    align16();
    net.w1[l] = (int)img.size();
    pack_frags(img, W1[l], precision);
    align16();
    net.w2[l] = (int)img.size();
    pack_frags(img, W2[l], precision);
  }
  // the layer-by-layer path (hidden 512, bf16): plain row-major bf16 matrices [out][in], Q rows scaled by
  // 1/sqrt(head dim) before rounding (as above), and the Q|K|V bias in natural order
  if (precision == MPPI_PREC_BF16 && D == 512) {
    net.lay = 1;
    auto put_rows = [&](const Tensor& W, int rows, int cols, int scaled_rows, double sc) {
      align16();
      const int off = (int)img.size();
      for (int r = 0; r < rows; ++r)
        for (int k = 0; k < cols; ++k) put_bf16(img, (r < scaled_rows ? sc : 1.0) * W.v[(size_t)r * cols + k]);
      return off;
    };
    for (int l = 0; l < nl; ++l) {
      const std::string p = "layers." + std::to_string(l) + ".";
      const Tensor& inb = get(T, p + "attention.in_proj_bias", {3 * D});
      std::vector<double> bq(3 * D);
      for (int r = 0; r < 3 * D; ++r) bq[r] = (r < D ? qs : 1.0) * inb.v[r];
      net.lbqkv[l] = put_vec(bq);
      net.lwqkv[l] = put_rows(get(T, p + "attention.in_proj_weight", {3 * D, D}), 3 * D, D, D, qs);
      net.lwo[l] = put_rows(get(T, p + "attention.out_proj.weight", {D, D}), D, D, 0, 1.0);
      net.lw1[l] = put_rows(get(T, p + "ffn.0.weight", {F4, D}), F4, D, 0, 1.0);
      net.lw2[l] = put_rows(get(T, p + "ffn.3.weight", {D, F4}), D, F4, 0, 1.0);
    }
  }
  // small-net kernel copies (bf16, D = 64, L <= 16), per layer:
  //   s_wqkv: per head h, 6 fragments: Q_h (scaled), K_h, V_h rows x k-blocks 0, 1 (register k order)
  //   s_w1:   fragment (mt < 16, kb < 2) at (2 mt + kb) KB;  s_w2: fragment (mt < 4, kb < 8) at (8 mt + kb) KB
  //   (the out-proj reads its input from LDS rows: the general image's Wo, natural k order)
  // (the LayerNorm affine maps are folded into s_wqkv / s_w1: see the first per-layer loop)
  if (small) {
    net.small = 1;
    for (int l = 0; l < nl; ++l) {
      const std::string p = "layers." + std::to_string(l) + ".";
      const Mat& qf = s_qf[l];
      const Mat& w1f = s_w1f[l];
      align16();
      net.s_wqkv[l] = (int)img.size();
      for (int h = 0; h < kFaHeads; ++h)
        for (int part = 0; part < 3; ++part)
          for (int kb = 0; kb < 2; ++kb) pack_frag_perm(img, qf, part * CW + 16 * h, kb);  // one chunk (CW = D)
      align16();
      net.s_w1[l] = (int)img.size();
      for (int mt = 0; mt < F4 / 16; ++mt)
        for (int kb = 0; kb < 2; ++kb) pack_frag_perm(img, w1f, 16 * mt, kb);
      const Mat w2 = from(get(T, p + "ffn.3.weight", {D, F4}));
      align16();
      net.s_w2[l] = (int)img.size();
      for (int mt = 0; mt < 4; ++mt)
        for (int kb = 0; kb < F4 / 32; ++kb) pack_frag_perm(img, w2, 16 * mt, kb);
    }
  }
  align16();
  net.img_bytes = (int)img.size();
  return img;
}

}  // namespace mppi
