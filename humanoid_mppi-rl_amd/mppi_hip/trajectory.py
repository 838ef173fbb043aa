"""Trajectory logging in the reference's CSV layout.

The reference's data-collection loop logs, before every env step, the state (qpos, qvel [, foot heights]), the
applied control and the sim time (src/Humanoid_datacollection_v2.jl:70-81 log_data!), then writes three
','-delimited CSVs without header (writedlm, :238-249):

    <out>/states_ft/states_<stamp>.csv     T x nx
    <out>/actions_ft/actions_<stamp>.csv   T x nu
    <out>/times_ft/times_<stamp>.csv       T x 1

or, for the older runs under data/<stamp>/, states.csv / actions.csv / times.csv.  learning/data_loader.py:146-166
reads them with pandas.read_csv (first row taken as header) and drops one more row.

run_stream() produces the rows on device: a captured graph of n chained solves whose env steps record
(x_t, u_t) (mppi_graph_capture_traj), so a whole logged episode is one graph launch.  The humanoid foot-height
columns need MuJoCo kinematics (data.xpos) that the learned surrogate does not produce; pass them as
extra_state_columns when they come from a MuJoCo replay.
"""
from __future__ import annotations

import os
import time

import numpy as np


def _fmt(row) -> str:
    # shortest round-trip repr (Julia's writedlm also prints shortest repr; exponent spelling differs)
    return ",".join(repr(float(v)) for v in row)


def write_trajectory_csv(out_dir: str, states: np.ndarray, actions: np.ndarray, dt: float = 0.01, t0: float = 0.0,
                         stamp: str | None = None, layout: str = "ft", extra_state_columns: np.ndarray | None = None
                         ) -> dict:
    """Write one trajectory (states [T, nx], actions [T, nu]); returns the three file paths."""
    states = np.asarray(states, np.float64)
    actions = np.asarray(actions, np.float64)
    if states.ndim != 2 or actions.ndim != 2 or states.shape[0] != actions.shape[0]:
        raise ValueError("states [T, nx] and actions [T, nu] with the same T")
    if extra_state_columns is not None:
        states = np.concatenate([states, np.asarray(extra_state_columns, np.float64).reshape(states.shape[0], -1)],
                                axis=1)
    stamp = stamp or time.strftime("%Y-%m-%d_%H%M%S")
    times = t0 + dt * np.arange(states.shape[0])
    if layout == "ft":
        paths = {k: os.path.join(out_dir, f"{k}_ft", f"{k}_{stamp}.csv") for k in ("states", "actions", "times")}
    elif layout == "run":
        paths = {k: os.path.join(out_dir, stamp, f"{k}.csv") for k in ("states", "actions", "times")}
    else:
        raise ValueError("layout must be 'ft' or 'run'")
    for k, rows in (("states", states), ("actions", actions), ("times", times[:, None])):
        os.makedirs(os.path.dirname(paths[k]), exist_ok=True)
        with open(paths[k], "w") as f:
            f.write("\n".join(_fmt(r) for r in rows) + "\n")
    return paths


def run_stream(engine, x0, U, n_solves: int, seed: int = 0, launches: int = 1, device=None):
    """Run `launches` x n_solves receding-horizon solves on device (shift + env step), logging the trajectory.

    x0 [B, nx], U [B, nu, H] (numpy); returns (states [launches*n_solves, B, nx], actions [..., B, nu],
    final U [B, nu, H]).  One graph launch per n_solves solves; nothing returns to the host in between.
    """
    import torch

    dev = device or torch.device("cuda", engine.device)
    c = engine.config
    tx = torch.as_tensor(np.asarray(x0, np.float32), device=dev).reshape(-1, c.nx).contiguous()
    B = tx.shape[0]
    tU = torch.as_tensor(np.asarray(U, np.float32), device=dev).reshape(B, c.nu, c.H).contiguous()
    tu0 = torch.zeros(B, c.nu, device=dev)
    trx = torch.empty(launches, n_solves, B, c.nx, device=dev)
    tru = torch.empty(launches, n_solves, B, c.nu, device=dev)
    engine.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    for i in range(launches):  # one capture per launch: each writes its own trajectory slice
        engine.graph_capture_traj(B, n_solves, tx.data_ptr(), tU.data_ptr(), tu0.data_ptr(), seed=seed,
                                  traj_x_ptr=trx[i].data_ptr(), traj_u_ptr=tru[i].data_ptr())
        engine.graph_launch(sync=True)
    return (trx.reshape(-1, B, c.nx).cpu().numpy(), tru.reshape(-1, B, c.nu).cpu().numpy(), tU.cpu().numpy())
