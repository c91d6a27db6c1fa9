"""Headline benchmark: env-steps/s of the batched assignment-env rollout on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--selector eps|sap|random]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one process per GPU, RCCL)

Workload (BASELINE.json configs[2]; configs[3] when N = 8): n = m = 64 agents/tasks,
T = 20, L = 3, lambda = 0.5, E = 16,384 envs per GPU, BasicMAC + RNNAgent (hidden 64,
GRUCell, fp32, PyTorch-ROCm) with the epsilon-greedy selector (eps = 0.05), Philox bump
benefits.  One "step" = one transition of every env on every rank: agent forward +
action selection + actions row write + one HIP env step kernel; every T steps an episode
ends (returns all-gathered over RCCL on the device) and the next one is reset inside the
timed region; the host-side episode checks (device error words, selector status, logging)
run once after it (GpuVecRunner.finish_episode(sync=False) / flush_pending).  value = world * E * K / (max over ranks of the K-step time).

The JSON line also carries:
  roofline: the env step kernel (the HIP hot path): algorithmic bytes per launch
            (B_step * E) / its average duration, timed live with HIP events
            on the stream it is launched on, against the 8 TB/s HBM3E peak; `traffic` is the
            PMC-measured HBM bytes per launch from profiles/ when a matching summary exists.
  cpu_baseline: rank 0 at N = 1 only: the reference's CPU design (subprocess-per-env
            ParallelRunner + numpy env + CPU RNN agent, oracle/cpu_parallel_runner.py) on a
            bounded sample of the same workload.
"""
import argparse
import json
import os
import sys
import time
from types import SimpleNamespace

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def step_bytes(n, m, L):
    """Algorithmic HBM bytes of one env step (DESIGN.md 'Roofline'): obs f32 n*m*(L+1),
    beta f32 n*m, avail_actions bool n*m, actions_onehot i64 n*m, actions i64 n (read),
    rewards f32 n, prev_assigns i64 n, terminated 1 B, filled 8 B."""
    return n * m * (4 * (L + 1) + 4 + 1 + 8) + n * (8 + 4 + 8) + 1 + 8


F32_MFMA_PEAK_TFS = 157.3  # MI355X dense f32 MFMA (= f32 vector peak; MI355X_MICROARCH.md)
BF16_MFMA_PEAK_TFS = 2500.0  # dense bf16 MFMA (MI355X_MICROARCH.md)
# f32 products as three-way-split bf16 MFMAs cost six bf16 products each
X3_PEAK_TFS = BF16_MFMA_PEAK_TFS / 6


def agent_peak(n, m, L, mode, hidden=64, use_rnn=True, onehot=True):
    """f32-equivalent MFMA roof of the agent forward: each layer's flops at the peak of the
    MFMA it runs on (asg_rnn_agent_mfma_mode: bit 0 GRU, bit 1 fc1 on split bf16), combined
    as the time-weighted harmonic mean (flops / sum of per-layer minimum times)."""
    K = m * (L + 1) - (m if onehot else 0)
    fc1, rec, fc2 = 2 * K * hidden, 2 * (2 * 3 * hidden * hidden if use_rnn else hidden * hidden), 2 * hidden * m
    t = (fc1 / (X3_PEAK_TFS if mode & 2 else F32_MFMA_PEAK_TFS) + rec / (X3_PEAK_TFS if mode & 1 else F32_MFMA_PEAK_TFS)
         + fc2 / F32_MFMA_PEAK_TFS)
    return (fc1 + rec + fc2) / t


def agent_flops(n, m, L, hidden=64, use_rnn=True, onehot=True):
    """Algorithmic flops of one agent row: fc1 (m(L+1) -> hidden), GRUCell (two hidden x
    3*hidden products), fc2 (hidden -> m); 2 flops per multiply-add.  onehot: the obs
    one-hot block (the first m inputs) is a column gather of W1, not m*hidden products
    (the fused kernel's one-hot prefix, ASG_AGENT_ONEHOT), so fc1 counts K - m inputs."""
    K = m * (L + 1) - (m if onehot else 0)
    rec = 2 * 3 * hidden * hidden if use_rnn else hidden * hidden
    return 2 * (K * hidden + rec + hidden * m)


def agent_roofline(a, E, sel_ms):
    """The action-selection launch (fused agent forward + epsilon-greedy, or the PyTorch
    agent + selector kernel), timed with HIP events on its stream, against the f32 MFMA
    peak: the kernel that takes most of each step's time next to the env step."""
    if a.selector == "random" or sel_ms <= 0:
        return None
    fused = a.agent == "rnn_fused"
    onehot = fused and os.environ.get("ASG_AGENT_ONEHOT", "1") != "0"
    flops = agent_flops(a.n, a.m, a.L, onehot=onehot) * E * a.n
    tfs = flops / (sel_ms * 1e-3) / 1e12
    from marl_sap_amd import _lib
    mode = int(_lib.lib().asg_rnn_agent_mfma_mode()) if fused else 0
    peak = agent_peak(a.n, a.m, a.L, mode, onehot=onehot)
    return {"bound": "mfma", "achieved": round(tfs, 2), "peak": round(peak, 1), "unit": "TFLOP/s",
            "frac": round(tfs / peak, 4), "traffic": None,
            "peak_note": ("f32-equivalent: GRU products on three-way-split bf16 MFMAs (2.5 PF / 6), fc1/fc2 "
                          "on f32 MFMAs (157.3 TF), time-weighted" if mode else "f32 MFMA peak"),
            "kernel": ("asg::rnn_agent_lds_kernel" if a.agent == "rnn_fused" else "torch agent + selector")
            if a.selector == "eps" else f"{a.agent} forward + asg::sap_select_kernel (whole selection)",
            "kernel_ms": round(sel_ms, 4), "flops_per_launch": flops}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=60)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--envs", type=int, default=16384, help="envs per GPU")
    p.add_argument("--n", type=int, default=64)
    p.add_argument("--m", type=int, default=64)
    p.add_argument("--T", type=int, default=20)
    p.add_argument("--L", type=int, default=3)
    p.add_argument("--selector", default="eps", choices=["eps", "sap", "random"])
    p.add_argument("--benefits", default="bump", choices=["bump", "dense"])
    p.add_argument("--cpu-baseline", type=int, default=1)
    p.add_argument("--cpu-episodes", type=int, default=2, help="minimum CPU-baseline episodes")
    p.add_argument("--cpu-seconds", type=float, default=15.0, help="CPU-baseline sample length (s)")
    p.add_argument("--agent", default="rnn_fused", choices=["rnn_fused", "rnn"],
                   help="rnn_fused: the same RNNAgent (weights, fp32) with its inference forward as one HIP kernel")
    p.add_argument("--seed", type=int, default=0)
    return p.parse_args()


def make_args(a, E):
    sel = {"eps": "epsilon_greedy", "sap": "sap", "random": "epsilon_greedy"}[a.selector]
    return SimpleNamespace(
        batch_size_run=E, env="mock_constellation_env",
        env_args=dict(n=a.n, m=a.m, T=a.T, L=a.L, lambda_=0.5, bids_as_actions=False, seed=a.seed,
                      benefits=a.benefits),
        env_rng="philox", env_quirks=(), runner_protocol="episode", test_nepisode=1,
        runner_log_interval=10 ** 12, n=a.n, m=a.m, T=a.T, hidden_dim=64, use_rnn=True,
        obs_last_action=False, obs_agent_id=False, agent_output_type="q", action_selector=sel, agent=a.agent,
        epsilon_start=0.05, epsilon_finish=0.05, epsilon_anneal_time=1, evaluation_epsilon=0.0, mac="basic_mac")


class NullLogger:
    def log_stat(self, *a, **k):
        pass


def main():
    a = parse()
    from marl_sap_amd import dist as asg_dist
    rank, world = asg_dist.init_from_env()
    # CPU baseline first: its worker processes are forked before this process touches
    # the GPU
    cpu = None
    if rank == 0 and world == 1 and a.cpu_baseline:
        from oracle import oracle as ora
        from oracle.cpu_parallel_runner import run_parallel_baseline
        workers = 8
        rate, steps_done, secs = run_parallel_baseline(n=a.n, m=a.m, T=a.T, L=a.L, workers=workers,
                                                       episodes=a.cpu_episodes, epsilon=0.05,
                                                       min_seconds=a.cpu_seconds)
        # second, stronger CPU number: the C oracle env, multi-threaded, random policy (env only)
        c_envs = 4096 if a.n * a.m <= 4096 else 256
        c_secs, _ = ora.rollout_random(c_envs, a.n, a.m, a.T, a.L, 0.5, a.seed, workers, 1)
        cpu = {"value": round(rate, 2), "unit": "env-steps/s", "cores": workers + 1, "kind": "port",
               "sample": f"{steps_done // (workers * a.T)} episodes x {workers} subprocess envs x T={a.T} at "
                         f"{a.n}x{a.m} ({steps_done} env-steps, {secs:.1f} s): the reference's ParallelRunner design "
                         f"(Pipe protocol, numpy env, CPU RNN agent + eps-greedy; oracle/cpu_parallel_runner.py)",
               "c_env_only": {"value": round(c_envs * a.T / c_secs, 1), "unit": "env-steps/s", "cores": workers,
                              "kind": "port", "sample": f"{c_envs} envs x 1 episode, random policy, C oracle "
                                                        f"(oracle/asg_rollout.c), no agent network"}}

    local = asg_dist.local_device_index()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    torch.manual_seed(a.seed + rank)

    from marl_sap_amd.controllers import REGISTRY as mac_REGISTRY
    from marl_sap_amd.runners import REGISTRY as r_REGISTRY

    E = a.envs
    args = make_args(a, E)
    runner = r_REGISTRY["gpu"](args, NullLogger())
    env = runner.get_env()
    mac = mac_REGISTRY["basic_mac"](env.scheme, {"agents": a.n}, args)
    mac.to(dev)
    runner.setup(env.scheme, {"agents": a.n}, env.preprocess, mac)

    ev_pairs = []   # (start, end) HIP events around each env step kernel in the timed region
    sel_pairs = []  # ... and around each action selection (agent forward + selector)
    state = {"t": a.T, "timing": False}

    def one_step():
        """One transition of all envs; resets / finishes episodes at boundaries."""
        if state["t"] >= a.T:
            if runner.batch is not None and runner.env.k == a.T:
                runner.finish_episode(sync=False)  # returns gathered on the device; host checks deferred
            runner.reset()
            mac.init_hidden(E)
            state["t"] = 0
        t = state["t"]
        with torch.no_grad():
            if state["timing"]:
                a0, a1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a0.record()
            if a.selector == "random":
                env.random_actions(runner.batch, ts=t)
            else:
                runner.select_into_batch(t)
            if state["timing"]:
                a1.record()
                sel_pairs.append((a0, a1))
            if state["timing"]:
                s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s0.record()
                env.step(runner.batch, ts=t)
                s1.record()
                ev_pairs.append((s0, s1))
            else:
                env.step(runner.batch, ts=t)
        state["t"] = t + 1

    for _ in range(a.warmup):
        one_step()
    asg_dist.barrier()
    torch.cuda.synchronize()
    state["timing"] = True
    t0 = time.perf_counter()
    for _ in range(a.steps):
        one_step()
    torch.cuda.synchronize()
    asg_dist.barrier()
    elapsed = time.perf_counter() - t0
    state["timing"] = False
    if runner.env.k == a.T:
        runner.finish_episode(sync=False)
    runner.flush_pending()  # surfaces any sticky device error of the timed steps
    kern_ms = sum(s.elapsed_time(e) for s, e in ev_pairs) / max(1, len(ev_pairs))
    sel_ms = sum(s.elapsed_time(e) for s, e in sel_pairs) / max(1, len(sel_pairs))

    if world > 1:
        import torch.distributed as tdist
        t = torch.tensor([elapsed, kern_ms, sel_ms], dtype=torch.float64, device=dev)
        if tdist.get_backend() == "gloo":
            t = t.cpu()
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        elapsed, kern_ms, sel_ms = float(t[0]), float(t[1]), float(t[2])

    total_steps = world * E * a.steps
    value = total_steps / elapsed
    per_launch = step_bytes(a.n, a.m, a.L) * E
    achieved = per_launch / (kern_ms * 1e-3) / 1e9
    traffic = None
    pmc_path = os.path.join(ROOT, "profiles", "pmc_step_kernel.json")
    if os.path.exists(pmc_path):
        try:
            pm = json.load(open(pmc_path))
            if pm.get("n") == a.n and pm.get("m") == a.m and pm.get("E") == E and pm.get("L") == a.L:
                traffic = pm.get("hbm_bytes_per_launch")
        except (ValueError, OSError):
            traffic = None

    if rank == 0:
        line = {
            "metric": "env steps/sec (whole node), 64-agent assignment env, 1/2/4/8 MI355X",
            "value": round(value, 1), "unit": "env-steps/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(elapsed / a.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (Philox bump benefits, random-init RNN agent)",
            "config": {"workload": f"{a.n}-agent/{a.m}-task assignment env, {E} envs per GPU, T={a.T}, L={a.L}, "
                                   f"BasicMAC+{a.agent}(GRU 64, fp32) + {args.action_selector if a.selector != 'random' else 'random'} "
                                   f"selector, {a.benefits} benefits",
                       "envs_per_gpu": E, "global_envs": world * E, "n": a.n, "m": a.m, "T": a.T, "L": a.L,
                       "parallelism": f"env-sharded x{world} (RCCL gather of returns per episode)"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "kernel": "asg::step_kernel", "kernel_ms": round(kern_ms, 4),
                         "bytes_per_launch": per_launch},
            "roofline_agent": agent_roofline(a, E, sel_ms),
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        import torch.distributed as tdist
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
