"""numpy Philox4x32-10 + Box-Muller, the same counter layout as csrc/philox.h (test helper)."""
import numpy as np

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = 0x9E3779B9, 0xBB67AE85
MASK = np.uint64(0xFFFFFFFF)


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    c0, c1, c2, c3 = (np.asarray(v, np.uint64) & MASK for v in (c0, c1, c2, c3))
    k0, k1 = int(k0) & 0xFFFFFFFF, int(k1) & 0xFFFFFFFF
    for _ in range(10):
        p0 = M0 * c0
        p1 = M1 * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & MASK
        hi1, lo1 = p1 >> np.uint64(32), p1 & MASK
        c0, c1, c2, c3 = (hi1 ^ c1 ^ np.uint64(k0)), lo1, (hi0 ^ c3 ^ np.uint64(k1)), lo0
        k0 = (k0 + W0) & 0xFFFFFFFF
        k1 = (k1 + W1) & 0xFFFFFFFF
    return c0, c1, c2, c3


def device_noise(seed: int, B: int, nu: int, H: int, K: int, sigma: float) -> np.ndarray:
    """eps[b][u][t][k] exactly as noise_kernel computes it (up to fp32 transcendental rounding)."""
    Kq = (K + 3) // 4
    b, u, t, kq = np.meshgrid(np.arange(B), np.arange(nu), np.arange(H), np.arange(Kq), indexing="ij")
    r0, r1, r2, r3 = philox4x32_10(kq, t, u, b, seed & 0xFFFFFFFF, seed >> 32)
    f = lambda v: ((v >> np.uint64(8)).astype(np.float64))
    u1a, u2a = (f(r0) + 1) / 16777216.0, f(r1) / 16777216.0
    u1b, u2b = (f(r2) + 1) / 16777216.0, f(r3) / 16777216.0
    ra, rb = np.sqrt(-2 * np.log(u1a)), np.sqrt(-2 * np.log(u1b))
    z = np.stack([ra * np.cos(2 * np.pi * u2a), ra * np.sin(2 * np.pi * u2a),
                  rb * np.cos(2 * np.pi * u2b), rb * np.sin(2 * np.pi * u2b)], axis=-1)
    return (sigma * z.reshape(B, nu, H, Kq * 4))[..., :K]


def test_philox_known_answer():
    """Random123 KAT: philox4x32-10, ctr = key = 0 -> 6627e8d5 e169c58d bc57ac4c 9b00dbd8."""
    r = philox4x32_10(0, 0, 0, 0, 0, 0)
    assert [int(v) for v in r] == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    r = philox4x32_10(0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF)
    assert [int(v) for v in r] == [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]
