"""RealConstellationEnv rollout throughput on one GPU, the
reference's real_constellation_env.yaml shape: 18 x 18 satellites (n = 324), m = 450
tasks, T = 100, L = 3, N = M = 10, per-env injected benefit tables (sparse, like
proximities), random policy written into the int16 actions row.

    python tools/bench_real_env.py [--envs 256] [--steps 40] [--cpu 1]
prints one JSON line: env-steps/s, the step pair (state + obs kernels) against HBM, and
the C oracle (oracle/asg_real_oracle.c, one thread) on a bounded sample as CPU figure."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from marl_sap_amd.components import EpisodeBatch  # noqa: E402
from marl_sap_amd.envs import RealAssignEnvBatch  # noqa: E402
from marl_sap_amd.envs.real_env import obs_size  # noqa: E402


def real_step_bytes(n, m, L, N, M):
    """Algorithmic HBM bytes of one env-step: L benefit slices read (f64) + actions (i16)
    read; obs / beta (f16), avail (bool), one-hot (i16), rewards, prev_assigns (i16),
    terminated, filled written."""
    return 8 * n * m * L + 2 * n + 2 * obs_size(N, M, L) * n + 2 * n * m * L + n * m + 2 * n * m + 2 * n + 2 * n + 9


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--envs", type=int, default=256)
    p.add_argument("--steps", type=int, default=40)
    p.add_argument("--n", type=int, default=324)
    p.add_argument("--m", type=int, default=450)
    p.add_argument("--T", type=int, default=100)
    p.add_argument("--cpu", type=int, default=1)
    a = p.parse_args()
    n, m, T, L, N, M, E = a.n, a.m, a.T, 3, 10, 10, a.envs
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    tables = torch.rand((E, n, m, T), generator=g, device=dev, dtype=torch.float64)
    tables *= torch.rand((E, n, m, 1), generator=g, device=dev, dtype=torch.float64) > 0.8
    env = RealAssignEnvBatch(18, 18, m, T, N, M, L, 0.5, sat_prox_mat=tables, num_envs=E, device=dev)
    del tables
    b = EpisodeBatch(env.scheme, {"agents": n}, E, T + 1, preprocess=env.preprocess, device=dev, time_major=True)
    env.reset(b, 0)
    acts = torch.randint(0, m, (a.steps + 5, E, n), generator=g, device=dev, dtype=torch.int64).to(torch.int16)
    for t in range(5):
        b["actions"][:, t, :, 0] = acts[t]
        env.step(b, t)
    torch.cuda.synchronize()
    ev = []
    t0 = time.perf_counter()
    for t in range(5, 5 + a.steps):
        b["actions"][:, t, :, 0] = acts[t]
        s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s0.record()
        env.step(b, t)
        s1.record()
        ev.append((s0, s1))
    torch.cuda.synchronize()
    secs = time.perf_counter() - t0
    env.sync()
    step_ms = sum(x.elapsed_time(y) for x, y in ev) / len(ev)
    per = real_step_bytes(n, m, L, N, M) * E
    res = {"metric": "env steps/sec, batched RealConstellationEnv (1 GPU)", "value": round(E * a.steps / secs, 1),
           "unit": "env-steps/s", "envs": E, "n": n, "m": m, "T": T, "L": L, "N": N, "M": M,
           "step_ms": round(step_ms, 4),
           "roofline": {"bound": "hbm", "achieved": round(per / (step_ms * 1e-3) / 1e9, 1), "peak": 8000.0,
                        "unit": "GB/s", "frac": round(per / (step_ms * 1e-3) / 1e9 / 8000.0, 4),
                        "bytes_per_launch": per}}
    if a.cpu:
        from oracle import oracle as ora
        tab = np.random.RandomState(0).uniform(size=(n, m, T)) * (np.random.RandomState(1).uniform(size=(n, m, 1)) > 0.8)
        r = ora.OracleRealEnv(tab, N, M, L, 0.5)
        r.reset()
        rng = np.random.RandomState(2)
        t0, steps = time.perf_counter(), 0
        while time.perf_counter() - t0 < 10.0 and steps < T:
            r.step(rng.randint(0, m, size=n))
            steps += 1
        cs = time.perf_counter() - t0
        res["cpu_baseline"] = {"value": round(steps / cs, 2), "unit": "env-steps/s", "cores": 1, "kind": "port",
                               "sample": f"{steps} steps of one env, C oracle (oracle/asg_real_oracle.c)"}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
