"""Feasibility probe (GPU box): per-step cost of a layer-by-layer FA D=512 step over all K samples with library
GEMMs (torch -> hipBLASLt) and torch LayerNorm / SDPA, to bound a layered design against fa_rollout_kernel.

    python scripts/fa512_layered_probe.py [--K 2048] [--chunks 1]
"""
import argparse
import time

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, default=2048)
    ap.add_argument("--chunks", type=int, default=1)
    args = ap.parse_args()
    dev = torch.device("cuda")
    L, D, HD = 49, 512, 128
    bf = torch.bfloat16
    Wqkv = (torch.randn(3 * D, D, device=dev) * 0.04).to(bf)
    Wo = (torch.randn(D, D, device=dev) * 0.04).to(bf)
    W1 = (torch.randn(4 * D, D, device=dev) * 0.04).to(bf)
    W2 = (torch.randn(D, 4 * D, device=dev) * 0.02).to(bf)
    bq = torch.zeros(3 * D, device=dev, dtype=bf)
    M = args.K // args.chunks * L
    r = torch.randn(args.chunks, M, D, device=dev)

    def gemm_times():
        h = torch.randn(M, D, device=dev).to(bf)
        hid = torch.randn(M, 4 * D, device=dev).to(bf)
        out = {}
        for name, f, flop in [("qkv", lambda: h @ Wqkv.t(), 2 * M * D * 3 * D),
                              ("outproj", lambda: h @ Wo.t(), 2 * M * D * D),
                              ("ffn1", lambda: torch.relu(h @ W1.t()), 2 * M * D * 4 * D),
                              ("ffn2", lambda: hid @ W2.t(), 2 * M * 4 * D * D)]:
            for _ in range(3):
                f()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(20):
                f()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / 20
            out[name] = (dt * 1e3, flop / dt / 1e12)
        return out

    for k, (ms, tf) in gemm_times().items():
        print(f"{k}: {ms:.3f} ms  {tf:.0f} TFLOP/s  (M={M})")

    def layer(x):
        h = torch.nn.functional.layer_norm(x, (D,)).to(bf)
        qkv = h @ Wqkv.t() + bq
        q, k, v = qkv.view(-1, L, 3, 4, HD).permute(2, 0, 3, 1, 4)
        o = torch.nn.functional.scaled_dot_product_attention(q, k, v)
        o = o.permute(0, 2, 1, 3).reshape(-1, D)
        x = x + (o @ Wo.t()).float()
        h2 = torch.nn.functional.layer_norm(x, (D,)).to(bf)
        x = x + (torch.relu(h2 @ W1.t()) @ W2.t()).float()
        return x

    def step():
        for c in range(args.chunks):
            x = r[c]
            for _ in range(2):
                x = layer(x)

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 10
    flop = args.K * (2 * (24 * L * D * D + 4 * L * L * D))
    print(f"torch layered step (2 layers, K={args.K}, chunks={args.chunks}): {dt * 1e3:.3f} ms, "
          f"{flop / dt / 1e12:.0f} TFLOP/s; x40 steps = {dt * 40 * 1e3:.1f} ms per solve (fused kernel: 82.5 ms)")


if __name__ == "__main__":
    main()
