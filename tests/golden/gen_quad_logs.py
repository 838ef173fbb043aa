"""Fixture generator (run in the survey container only; /root/reference is not on the GPU box).

Packs a few of the reference's logged quadruped MPPI trajectories (quad_data/<run>/{states,actions}<i>.csv: 37 state
columns qpos[19] + qvel[18], 12 action columns, written by src/quadruped_datacollection.py) into
tests/golden/quad_logs.npz as raw float32 file rows, so the training row and the quadruped
workloads' initial states have the reference's own data on the GPU box.  Data only: no reference code is copied.

    python tests/golden/gen_quad_logs.py [--runs 4]
"""
import argparse
import os

import numpy as np

REF = "/root/reference/quad_data"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "quad_logs.npz")

if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=4)
    args = ap.parse_args()
    runs = []
    for r in sorted(os.listdir(REF)):  # runs with both logs (some runs lack states<i>.csv)
        fs = sorted(os.listdir(os.path.join(REF, r)))
        st = [f for f in fs if f.startswith("states")]
        if st and st[0].replace("states", "actions") in fs:
            runs.append((r, st[0], st[0].replace("states", "actions")))
    runs = runs[: args.runs]
    arrays = {}
    for i, (r, sf, af) in enumerate(runs):
        s = np.loadtxt(os.path.join(REF, r, sf), delimiter=",", dtype=np.float64).astype(np.float32)
        a = np.loadtxt(os.path.join(REF, r, af), delimiter=",", dtype=np.float64).astype(np.float32)
        assert s.shape[1] == 37 and a.shape[1] == 12 and len(s) == len(a), (r, s.shape, a.shape)
        arrays[f"states{i}"], arrays[f"actions{i}"] = s, a
        print(r, s.shape, a.shape)
    arrays["runs"] = np.array([f"{r}/{sf}" for r, sf, _ in runs])
    np.savez_compressed(OUT, **arrays)
    print("wrote", OUT, os.path.getsize(OUT), "bytes")
