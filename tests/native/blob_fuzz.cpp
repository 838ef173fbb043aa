// Host-side robustness harness for the weight-blob parser and packers (humanoid_mppi-rl_amd/csrc/mppi_nets.cpp),
// built with AddressSanitizer + UndefinedBehaviorSanitizer by tests/test_sanitizers.py (host code only: no GPU).
// mppi_load_dynamics hands caller bytes straight to build_fc_net / build_fa_net, so every malformed blob must end
// in a std::exception (the ABI turns it into MPPI_E_UNSUPPORTED), never in an out-of-bounds access.
//
// usage: blob_fuzz <kind 2|3|4> <nx> <nu> <blob file> <seed>
//   1. the blob builds at both precisions;
//   2. every prefix shorter than 1 KB, and 128 longer ones, is rejected;
//   3. 600 seeded corruptions (a byte, or an aligned 32-bit word set to 0, 1, 0xFFFFFFFF, 0x7FFFFFFF or random)
//      either build or are rejected.
// Prints "ok <built> <rejected>" and exits 0; a sanitizer report aborts with a non-zero status.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <exception>
#include <fstream>
#include <iterator>
#include <vector>

#include "../../humanoid_mppi-rl_amd/csrc/mppi_internal.h"

namespace mppi {
std::vector<unsigned char> build_fc_net(int kind, const void* blob, size_t nbytes, int precision, int nx, int nu,
                                        FcNet& net);
std::vector<unsigned char> build_fa_net(const void* blob, size_t nbytes, int precision, int nx, int nu, FaNet& net);
}  // namespace mppi

static int g_built = 0, g_rejected = 0;

static bool try_build(int kind, const std::vector<unsigned char>& b, int precision, int nx, int nu) {
  try {
    if (kind == MPPI_DYN_FEATURE_ATTN) {
      mppi::FaNet net;
      const auto img = mppi::build_fa_net(b.data(), b.size(), precision, nx, nu, net);
      if (img.size() != (size_t)net.img_bytes) throw std::logic_error("image size mismatch");
    } else {
      mppi::FcNet net;
      const auto img = mppi::build_fc_net(kind, b.data(), b.size(), precision, nx, nu, net);
      if (img.size() != (size_t)net.img_bytes) throw std::logic_error("image size mismatch");
    }
    ++g_built;
    return true;
  } catch (const std::logic_error& e) {
    std::fprintf(stderr, "FAIL: %s\n", e.what());
    std::exit(3);
  } catch (const std::exception&) {
    ++g_rejected;
    return false;
  }
}

int main(int argc, char** argv) {
  if (argc != 6) {
    std::fprintf(stderr, "usage: blob_fuzz kind nx nu blob seed\n");
    return 2;
  }
  const int kind = std::atoi(argv[1]), nx = std::atoi(argv[2]), nu = std::atoi(argv[3]);
  std::ifstream f(argv[4], std::ios::binary);
  const std::vector<unsigned char> blob((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  uint64_t s = std::strtoull(argv[5], nullptr, 10) * 6364136223846793005ull + 1442695040888963407ull;
  auto rnd = [&]() {
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    return (uint32_t)(s >> 33);
  };
  for (int prec : {MPPI_PREC_FP32, MPPI_PREC_BF16}) {
    if (kind == MPPI_DYN_FEATURE_ATTN && prec == MPPI_PREC_FP32) continue;  // (hidden 64 only; the caller's choice)
    if (!try_build(kind, blob, prec, nx, nu)) {
      std::fprintf(stderr, "FAIL: the valid blob was rejected (precision %d)\n", prec);
      return 4;
    }
  }
  const int prec = MPPI_PREC_BF16;
  std::vector<size_t> cuts;
  for (size_t n = 0; n < blob.size() && n < 1024; ++n) cuts.push_back(n);
  for (int i = 0; i < 128 && blob.size() > 1024; ++i) cuts.push_back(1024 + rnd() % (blob.size() - 1024));
  for (size_t n : cuts) {
    std::vector<unsigned char> b(blob.begin(), blob.begin() + n);
    if (try_build(kind, b, prec, nx, nu)) {
      std::fprintf(stderr, "FAIL: a %zu-byte prefix of a %zu-byte blob was accepted\n", n, blob.size());
      return 5;
    }
  }
  const uint32_t words[] = {0u, 1u, 0xFFFFFFFFu, 0x7FFFFFFFu};
  for (int i = 0; i < 600; ++i) {
    std::vector<unsigned char> b = blob;
    // headers and tensor names sit in the first few hundred bytes: half the corruptions land there
    const size_t span = (i & 1) ? b.size() : std::min<size_t>(b.size(), 1024);
    if (rnd() & 1) {
      b[rnd() % span] = (unsigned char)rnd();
    } else {
      const size_t at = (rnd() % (span / 4)) * 4;
      const uint32_t w = (rnd() & 3) ? words[rnd() % 4] : rnd();
      std::memcpy(b.data() + at, &w, std::min<size_t>(4, b.size() - at));
    }
    try_build(kind, b, prec, nx, nu);
  }
  std::printf("ok %d %d\n", g_built, g_rejected);
  return 0;
}
