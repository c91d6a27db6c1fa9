"""CPU baseline: a faithful from-scratch restatement of the reference's CPU hot path
(TEST / BASELINE INFRASTRUCTURE ONLY -- timed by bench.py's cpu_baseline leg).

It keeps the reference design that the GPU build replaces:
  * NumpyMockEnv: MockConstellationEnv with its per-agent Python loops and list-concat
    observations (envs/mock_constellation_env.py:94-175, :228-299), numpy global stream;
  * one OS subprocess per env and the reference's Pipe command protocol
    ("step" / "reset" / "get_stats" / "close", runners/parallel_runner.py:246-284),
    pickled numpy lists both ways;
  * the parent runs the batched RNN agent on the CPU (torch, 1 thread as main.py:90 sets)
    with the epsilon-greedy selector and writes every transition into a CPU EpisodeBatch
    (parallel_runner.py:113-200).
The reference's own ParallelRunner cannot travel to the GPU box; SURVEY.md §8(d) /
BASELINE.md record the calibration of this restatement against it in the survey
container (reference: 1,249 / 619 env-steps/s at 16x16 / 64x64 on 8 workers).
"""
import multiprocessing as mp
import time
from types import SimpleNamespace

import numpy as np


class NumpyMockEnv:
    """MockConstellationEnv restated with numpy (same loops, same global-stream draws)."""

    def __init__(self, n, m, T, L, lambda_):
        self.n, self.m, self.T, self.L, self.lambda_ = n, m, T, L, lambda_
        self.sat_prox_mat = generate_benefits_over_time(n, m, T, 5, 8)
        self.T_trans = np.ones((m, m)) - np.eye(m)
        self.k = 0

    def reset(self):
        self.curr_assignment = np.zeros((self.n, self.m))
        self.k = 0
        self.sat_prox_mat = generate_benefits_over_time(self.n, self.m, self.T, 3, 6)
        self.beta = self.sat_prox_mat[:, :, self.k]
        self.prev_assigns = np.random.choice(self.m, self.n, replace=False)
        self._build_obs()

    def _build_obs(self):
        self._obs = [self.curr_assignment[i, :] for i in range(self.n)]
        for l in range(self.L):
            if self.k + l < self.T:
                self._obs = [np.concatenate([self._obs[i], self.sat_prox_mat[i, :, self.k + l]]) for i in range(self.n)]
            else:
                self._obs = [np.concatenate([self._obs[i], np.zeros(self.m)]) for i in range(self.n)]

    def beta_hat(self, beta, prev_assigns):
        prev_mat = np.zeros((1, self.n, self.m))
        for i in range(self.n):
            prev_mat[0, i, prev_assigns[i]] = 1
        pen = (prev_mat @ self.T_trans) * (beta[None] > 1e-12)
        return (beta[None] - self.lambda_ * pen)[0]

    def step(self, actions):
        a = np.array(actions, dtype=int)
        bh = self.beta_hat(self.beta, self.prev_assigns)
        cnt = np.zeros(self.m)
        for i in range(self.n):
            cnt[a[i]] += 1
        rewards = []
        for i in range(self.n):
            c = a[i]
            rewards.append(bh[i, c] / cnt[c] if bh[i, c] > 0 else bh[i, c])
        self.curr_assignment = np.zeros((self.n, self.m))
        for i in range(self.n):
            self.curr_assignment[i, a[i]] = 1
        self.k += 1
        self._build_obs()
        done = self.k >= self.T
        self.beta = self.sat_prox_mat[:, :, self.k] if not done else np.zeros((self.n, self.m))
        self.prev_assigns = a
        return rewards, done, {}

    def get_pretransition_data(self):
        return {"obs": [self._obs], "avail_actions": [[[1] * self.m] * self.n], "beta": [self.beta]}


def generate_benefits_over_time(n, m, T, width_min, width_max):
    benefits = np.zeros((n, m, T))
    for j in range(m):
        scale = np.random.choice([1, 1, 1, 10])
        for i in range(n):
            if np.random.rand() > 0.75:
                center = np.random.uniform(0, T)
                spread = np.random.uniform(width_min, width_max)
                s2 = np.sqrt(spread ** 2 / -8 / np.log(0.05))
                for t in range(T):
                    benefits[i, j, t] = scale * np.exp(-(t - center) ** 2 / s2 / 2)
    return benefits


def _worker(remote, cfg):
    import torch
    torch.set_num_threads(1)
    np.random.seed(cfg["seed"])
    env = NumpyMockEnv(cfg["n"], cfg["m"], cfg["T"], cfg["L"], cfg["lambda_"])
    while True:
        cmd, data = remote.recv()
        if cmd == "step":
            r, d, info = env.step(data)
            remote.send([{"rewards": r, "terminated": d, "info": info}, env.get_pretransition_data()])
        elif cmd == "reset":
            env.reset()
            remote.send(env.get_pretransition_data())
        elif cmd == "get_stats":
            remote.send({})
        elif cmd == "close":
            remote.close()
            break


def run_parallel_baseline(n=64, m=64, T=20, L=3, lambda_=0.5, workers=8, episodes=2, hidden=64,
                          epsilon=0.05, seed=0, min_seconds=0.0, max_episodes=10000):
    """Runs ParallelRunner-protocol episodes of `workers` envs -- `episodes` of them, or
    more until `min_seconds` have elapsed (bounded by max_episodes); returns
    (env_steps_per_s, env_steps, seconds, reset_seconds): the rate over the whole loop
    (resets amortised, as the reference runner's wall time includes them) and the time
    spent in the reset round trips, so the step-loop-only rate is
    env_steps / (seconds - reset_seconds) (SURVEY §8(d) asks for both)."""
    import torch

    from marl_sap_amd.components import EpisodeBatch
    from marl_sap_amd.envs.assign_env import make_scheme
    from marl_sap_amd.modules.agents import RNNAgent

    torch.set_num_threads(1)
    torch.manual_seed(seed)
    ctx = mp.get_context("fork")
    pipes = [ctx.Pipe() for _ in range(workers)]
    procs = [ctx.Process(target=_worker, args=(w, dict(n=n, m=m, T=T, L=L, lambda_=lambda_, seed=seed)),
                         daemon=True) for _, w in pipes]
    for p in procs:
        p.start()
    parents = [p for p, _ in pipes]
    scheme, preprocess = make_scheme(n, m, L)
    args = SimpleNamespace(hidden_dim=hidden, use_rnn=True, m=m)
    agent = RNNAgent(m * (L + 1), args)
    steps = 0
    reset_secs = 0.0
    t0 = time.perf_counter()
    with torch.no_grad():
        ep = 0
        while ep < episodes or (time.perf_counter() - t0 < min_seconds and ep < max_episodes):
            ep += 1
            r0 = time.perf_counter()
            batch = EpisodeBatch(scheme, {"agents": n}, workers, T + 1, preprocess=preprocess, device="cpu")
            for c in parents:
                c.send(("reset", None))
            pre = {"obs": [], "avail_actions": [], "beta": []}
            for c in parents:
                for k, v in c.recv().items():
                    pre[k].extend(v)
            batch.update(pre, ts=0)
            reset_secs += time.perf_counter() - r0
            h = agent.init_hidden().unsqueeze(0).expand(workers, n, -1)
            for t in range(T):
                q, h = agent(batch["obs"][:, t].reshape(workers * n, -1), h)
                q = q.view(workers, n, m)
                greedy = q.max(dim=2)[1]
                rnd = torch.randint(0, m, (workers, n))
                pick = torch.rand(workers, n) < epsilon
                actions = torch.where(pick, rnd, greedy)
                batch.update({"actions": actions.unsqueeze(1)}, ts=t, mark_filled=False)
                cpu_actions = actions.numpy()
                for i, c in enumerate(parents):
                    c.send(("step", cpu_actions[i]))
                post = {"rewards": [], "terminated": []}
                pre = {"obs": [], "avail_actions": [], "beta": []}
                for c in parents:
                    d_post, d_pre = c.recv()
                    post["rewards"].append((d_post["rewards"],))
                    post["terminated"].append((d_post["terminated"],))
                    for k, v in d_pre.items():
                        pre[k].extend(v)
                    steps += 1
                batch.update(post, ts=t, mark_filled=False)
                batch.update(pre, ts=t + 1, mark_filled=True)
    secs = time.perf_counter() - t0
    for c in parents:
        c.send(("close", None))
    for p in procs:
        p.join(timeout=5)
    return steps / secs, steps, secs, reset_secs
