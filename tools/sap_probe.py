"""SAP selector probe on the runner's own Q matrices (GPU):

    python tools/sap_probe.py [--envs 4096] [--eps 0.05] [--use-rnn 1]

Rolls the configs[2] env with BasicMAC + RNNAgent, and at a few episode rows t takes the
agent's Q (mac.forward) and runs asg_sap_select on it with the step-counting instance:
per row, the kernel time (HIP events), the fast-path / scipy-exact step totals and how many
problems the fast path left to the exact solver.  One JSON line per row.
"""
import argparse
import ctypes
import json
import os
import sys
from types import SimpleNamespace

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    from marl_sap_amd import _lib
    from marl_sap_amd.controllers import REGISTRY as MAC
    from marl_sap_amd.runners import REGISTRY as RUN
    p = argparse.ArgumentParser()
    p.add_argument("--envs", type=int, default=4096)
    p.add_argument("--eps", type=float, default=0.05)
    p.add_argument("--use-rnn", type=int, default=1)
    p.add_argument("--rows", default="0,1,2,5,10,19")
    a = p.parse_args()
    dev = torch.device("cuda", 0)
    n = m = 64
    T = 20
    E = a.envs
    args = SimpleNamespace(
        batch_size_run=E, env="mock_constellation_env",
        env_args=dict(n=n, m=m, T=T, L=3, lambda_=0.5, bids_as_actions=False, seed=0, benefits="bump"),
        env_rng="philox", env_quirks=(), runner_protocol="episode", test_nepisode=1, runner_log_interval=10 ** 12,
        n=n, m=m, T=T, hidden_dim=64, use_rnn=bool(a.use_rnn), obs_last_action=False, obs_agent_id=False,
        agent_output_type="q", action_selector="sap", agent="rnn", seed=0, epsilon_start=a.eps,
        epsilon_finish=a.eps, epsilon_anneal_time=1, evaluation_epsilon=0.0, mac="basic_mac", reuse_batch=True,
        fused_rollout=False)
    runner = RUN["gpu"](args, None)
    env = runner.get_env()
    torch.manual_seed(0)
    mac = MAC["basic_mac"](env.scheme, {"agents": n}, args)
    mac.to(dev)
    runner.setup(env.scheme, {"agents": n}, env.preprocess, mac)
    rows = {int(x) for x in a.rows.split(",")}
    L = _lib.lib()
    runner.reset()
    mac.init_hidden(E)
    with torch.no_grad():
        for t in range(T):
            q = mac.forward(runner.batch, t).view(E, n, m).contiguous()
            if t in rows:
                steps = torch.zeros(E, dtype=torch.int32, device=dev)
                out = torch.empty((E, n), dtype=torch.float32, device=dev)
                ms = []
                for rep in range(3):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    _lib.check(L.asg_sap_select(ctypes.c_void_p(q.data_ptr()), _lib.i64arr(q.stride()), E, n, m,
                                                a.eps, 1, 1, 0, ctypes.c_void_p(out.data_ptr()), None,
                                                ctypes.c_void_p(steps.data_ptr()) if rep == 0 else None,
                                                _lib.stream_ptr(dev)))
                    e1.record()
                    torch.cuda.synchronize()
                    ms.append(e0.elapsed_time(e1))
                s = steps.long()
                fast, exact = s & 0xFFFF, s >> 16
                qa = q.abs().mean().item()
                print(json.dumps({"t": t, "ms": [round(x, 4) for x in ms], "fast_steps": int(fast.sum()),
                                  "exact_steps": int(exact.sum()), "exact_problems": int((exact > 0).sum()),
                                  "max_fast": int(fast.max()), "mean_abs_q": qa,
                                  "q_row_spread": float((q - q.mean(1, keepdim=True)).abs().mean() / max(qa, 1e-30))}),
                      flush=True)
            # the selection of this row from the same Q (the hidden state advanced once)
            row = runner.batch["actions"][:, t, :, 0]
            mac.action_selector.select_action(q, runner.batch["avail_actions"][:, t], 0, out=row)
            env.step(runner.batch, ts=t)
    env.close()


if __name__ == "__main__":
    main()
