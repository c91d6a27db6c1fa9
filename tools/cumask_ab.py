"""A/B: CU-partitioned pipelining of the rollout on one GPU.

    python tools/cumask_ab.py [--mode serial|split] [--env-cus 32] [--layout lo|spread]

serial: bench.py's loop (one stream, fused agent + epsilon-greedy, then the env step kernel).
split:  the envs in two halves (global env indices [0, E/2), [E/2, E)), each with its own
        MAC hidden state; the agent runs on a stream restricted to 256 - env_cus CUs and the
        env steps on a stream restricted to the other env_cus CUs
        (hipExtStreamCreateWithCUMask), ordered by events, so the step kernel of one half
        streams its HBM writes while the other half's agent kernel keeps the MFMAs busy.
        The persistent agent kernel sizes its grid to its stream's CU count.
Prints one JSON line with ms/step and env-steps/s.
"""
import argparse
import copy
import ctypes
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


def cu_stream(bits):
    """A HIP stream restricted to the CUs whose ids are in `bits`, wrapped for torch."""
    hip = ctypes.CDLL("libamdhip64.so")
    words = [0] * 8
    for b in bits:
        words[b // 32] |= 1 << (b % 32)
    arr = (ctypes.c_uint32 * 8)(*words)
    s = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), 8, arr)
    if rc != 0:
        raise RuntimeError(f"hipExtStreamCreateWithCUMask: {rc}")
    return torch.cuda.ExternalStream(s.value)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--envs", type=int, default=16384)
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--mode", default="split", choices=["serial", "split"])
    p.add_argument("--env-cus", type=int, default=32)
    p.add_argument("--layout", default="lo", choices=["lo", "spread"])
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
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    if parts == 1:
        s_agent = s_env = torch.cuda.current_stream()
    else:
        if a.layout == "lo":
            env_bits = list(range(a.env_cus))
        else:
            stride = ncu // a.env_cus
            env_bits = [i * stride for i in range(a.env_cus)]
        agent_bits = [b for b in range(ncu) if b not in set(env_bits)]
        s_agent, s_env = cu_stream(agent_bits), cu_stream(env_bits)
    ev_sel = [torch.cuda.Event() for _ in range(parts)]
    ev_env = [None] * parts
    state = {"t": T}

    def one_step():
        t = state["t"]
        if t >= T:
            t = 0
        for k in range(parts):
            with torch.cuda.stream(s_agent):
                if ev_env[k] is not None:
                    s_agent.wait_event(ev_env[k])
                if t == 0:
                    with torch.cuda.stream(s_env):
                        s_env.wait_stream(s_agent)
                        envs[k].reset(views[k], ts=0)
                        e0 = torch.cuda.Event()
                        e0.record(s_env)
                    s_agent.wait_event(e0)
                    macs[k].init_hidden(Eh)
                row = views[k]["actions"][:, t, :, 0]
                macs[k].select_actions(views[k], t_ep=t, t_env=0, out=row)
                ev_sel[k].record(s_agent)
            with torch.cuda.stream(s_env):
                s_env.wait_event(ev_sel[k])
                envs[k].step(views[k], ts=t)
                ev = torch.cuda.Event()
                ev.record(s_env)
                ev_env[k] = ev
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
    print(json.dumps({"mode": a.mode, "env_cus": a.env_cus if parts > 1 else None, "layout": a.layout,
                      "envs": E, "ms_per_step": round(el / a.steps * 1e3, 4),
                      "env_steps_per_s": round(E * a.steps / el)}), flush=True)


if __name__ == "__main__":
    main()
