"""Determinism probe: the FA-cartpole graph replay of test_kernel_clock_times_graph_replays on fresh engines with the
kernel clock off / off / on / on; prints each final x0 and the max |difference| to the first."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(ROOT, d) for d in ("tests", "", "humanoid_mppi-rl_amd", "oracle")]
import test_gpu_parity as T  # noqa: E402
import mppi_hip as M  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "fa"
K, H, B, n, reps = 1024, 16, 2, 3, 4
dev = torch.device("cuda")
res = []
for clock in (False, False, True, True):
    eng, x0, U0, _ = T._dev_setup(M, kind, K, H, B, 1)
    eng.set_stream(torch.cuda.current_stream().cuda_stream)
    tx, tU = torch.from_numpy(x0).to(dev), torch.from_numpy(U0).to(dev)
    tu0 = torch.zeros(B, U0.shape[1], device=dev)
    if clock:
        eng.kernel_clock(True)
    eng.graph_capture(B, n, tx.data_ptr(), tU.data_ptr(), tu0.data_ptr(), seed=4)
    for _ in range(reps):
        eng.graph_launch(sync=False)
    torch.cuda.synchronize()
    res.append((tx.cpu().numpy(), tU.cpu().numpy()))
    print("clock", clock, "x", res[-1][0].ravel(), "dx", np.abs(res[-1][0] - res[0][0]).max(),
          "dU", np.abs(res[-1][1] - res[0][1]).max(), flush=True)
