"""Calibrate bench.py's CPU baseline (oracle/cpu_parallel_runner.py, a from-scratch
restatement of the reference's ParallelRunner + MockConstellationEnv) against the real
reference ParallelRunner, run here on identical settings.

Runs ONLY in the build container (it imports /root/reference/src through the same
offline stand-ins as tests/golden/make_golden.py; nothing of the reference travels).
Writes profiles/cpu_baseline_calibration.json with both rates and their ratio.

    python tools/calibrate_cpu_baseline.py [--n 64] [--m 64] [--workers 8] [--seconds 20]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def time_reference(n, m, T, workers, seconds, eps):
    import numpy as np
    import torch as th

    import make_golden as mg
    mg._install_stubs()
    th.set_num_threads(1)
    from controllers import REGISTRY as mac_REGISTRY
    from runners.parallel_runner import ParallelRunner

    np.random.seed(0)
    th.manual_seed(0)
    args = mg._args(batch_size_run=workers, action_selector="epsilon_greedy", use_rnn=True,
                    epsilon_start=eps, epsilon_finish=eps, test_nepisode=10 ** 9,
                    env_args=dict(n=n, m=m, T=T, L=3, lambda_=0.5, bids_as_actions=False, seed=0))
    runner = ParallelRunner(args, mg._Logger())
    env = runner.get_env()
    args.n, args.m, args.T = env.n, env.m, env.T
    mac = mac_REGISTRY["basic_mac"](env.scheme, {"agents": n}, args)
    runner.setup(scheme=env.scheme, groups={"agents": n}, preprocess=env.preprocess, mac=mac)
    runner.run(test_mode=False)  # warm-up episode (pipes, first-call overheads)
    t0_env = runner.t_env
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        runner.run(test_mode=False)
    secs = time.perf_counter() - t0
    steps = runner.t_env - t0_env
    runner.close_env()
    return steps / secs, steps, secs


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=64)
    p.add_argument("--m", type=int, default=64)
    p.add_argument("--T", type=int, default=20)
    p.add_argument("--workers", type=int, default=8)
    p.add_argument("--seconds", type=float, default=20.0)
    p.add_argument("--eps", type=float, default=0.05)
    a = p.parse_args()

    from oracle.cpu_parallel_runner import run_parallel_baseline
    port = run_parallel_baseline(n=a.n, m=a.m, T=a.T, workers=a.workers, episodes=1, epsilon=a.eps,
                                 min_seconds=a.seconds)
    ref = time_reference(a.n, a.m, a.T, a.workers, a.seconds, a.eps)
    res = {"n": a.n, "m": a.m, "T": a.T, "workers": a.workers, "host_cpus": os.cpu_count(),
           "reference_parallel_runner": {"env_steps_per_s": ref[0], "env_steps": ref[1], "seconds": ref[2]},
           "port_cpu_parallel_runner": {"env_steps_per_s": port[0], "env_steps": port[1], "seconds": port[2]},
           "port_over_reference": port[0] / ref[0]}
    out = os.path.join(ROOT, "profiles", f"cpu_baseline_calibration_{a.n}x{a.m}.json")
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
