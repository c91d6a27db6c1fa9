"""A/B: one rollout stream vs two env halves pipelined on two HIP streams (1 GPU).

    python tools/overlap_ab.py [--envs 16384] [--steps 60] [--mode serial|halves]

serial: one env handle of E envs, per step fused agent + epsilon-greedy selection then the
        env step kernel, all on one stream (bench.py's loop).
halves: two handles of E/2 envs (global env indices [0, E/2) and [E/2, E)) over the two
        halves of ONE time-major EpisodeBatch, each with its own MAC hidden state and its
        own stream; the selection of one half can run while the other half's env step
        kernel streams its HBM writes.  Co-residency needs the persistent agent kernel's
        registers to leave room for a step wave (build with -DASG_AGENT_NUM_VGPR=224).
Prints one JSON line with ms/step and env-steps/s.
"""
import argparse
import copy
import json
import os
import sys
import time
from types import SimpleNamespace

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from marl_sap_amd.components import EpisodeBatch  # noqa: E402
from marl_sap_amd.controllers import REGISTRY as mac_REGISTRY  # noqa: E402
from marl_sap_amd.envs import AssignEnvBatch  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--envs", type=int, default=16384)
    p.add_argument("--steps", type=int, default=60)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--mode", default="halves", choices=["serial", "halves"])
    a = p.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.manual_seed(0)
    n = m = 64
    T, L, E = 20, 3, a.envs
    parts = 1 if a.mode == "serial" else 2
    Eh = E // parts
    envs = [AssignEnvBatch(n, m, T, L, 0.5, seed=0, num_envs=Eh, env_index_base=k * Eh, device=dev)
            for k in range(parts)]
    args = SimpleNamespace(n=n, m=m, hidden_dim=64, use_rnn=True, obs_last_action=False, obs_agent_id=False,
                           agent_output_type="q", action_selector="epsilon_greedy", agent="rnn_fused",
                           epsilon_start=0.05, epsilon_finish=0.05, epsilon_anneal_time=1, evaluation_epsilon=0.0)
    mac = mac_REGISTRY["basic_mac"](envs[0].scheme, {"agents": n}, args)
    mac.to(dev)
    macs = [mac] + [copy.copy(mac) for _ in range(parts - 1)]
    for k in range(1, parts):
        macs[k].action_selector = copy.copy(mac.action_selector)
    batch = EpisodeBatch(envs[0].scheme, {"agents": n}, E, T + 1, preprocess=envs[0].preprocess, device=dev,
                         time_major=True)
    views = [batch[k * Eh:(k + 1) * Eh] for k in range(parts)]
    streams = [torch.cuda.current_stream()] if parts == 1 else [torch.cuda.Stream() for _ in range(parts)]
    state = {"t": T}

    def one_step():
        t = state["t"]
        if t >= T:
            t = 0
        for k in range(parts):
            with torch.cuda.stream(streams[k]):
                if t == 0:
                    envs[k].reset(views[k], ts=0)
                    macs[k].init_hidden(Eh)
                row = views[k]["actions"][:, t, :, 0]
                macs[k].select_actions(views[k], t_ep=t, t_env=0, out=row)
                envs[k].step(views[k], ts=t)
        state["t"] = t + 1

    with torch.no_grad():
        for _ in range(a.warmup):
            one_step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            one_step()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
    for e in envs:
        e.sync()
    print(json.dumps({"mode": a.mode, "lib": os.environ.get("ASG_LIB_PATH", "in-tree"), "envs": E,
                      "ms_per_step": round(el / a.steps * 1e3, 4), "env_steps_per_s": round(E * a.steps / el)}))


if __name__ == "__main__":
    main()
