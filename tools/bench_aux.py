"""Measurements for the SURVEY §8(f) rows built on the rollout kernels (1 GPU):

  sap_targets  B x (T-1) SAP learner targets: one asg_lsa_batched launch + device gather
               vs the reference's serial scipy loop on the host (sap_q_learner.py:98-108)
  replay       device-resident ReplayBuffer: insert one rollout batch (time-major, as the
               GpuVecRunner returns it) and sample a learner batch, as HBM GB/s

    python tools/bench_aux.py [--envs 4096] [--buffer 8192] [--lsa-batch 32]
prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import scipy.optimize  # noqa: E402
import torch  # noqa: E402

from marl_sap_amd.components import EpisodeBatch, ReplayBuffer  # noqa: E402
from marl_sap_amd.envs import AssignEnvBatch  # noqa: E402
from marl_sap_amd.learners import sap_target_max_qvals  # noqa: E402


def timed(fn, iters):
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def bench_sap_targets(B, T, n, m, dev):
    g = torch.Generator().manual_seed(0)
    q_t = torch.randn((B, T - 1, n, m), generator=g)
    avail = torch.ones((B, T, n, m), dtype=torch.bool)
    qd, ad = q_t.to(dev), avail.to(dev)
    sap_target_max_qvals(qd, ad)
    gpu_ms = timed(lambda: sap_target_max_qvals(qd, ad), 5)
    t0 = time.perf_counter()
    tm = q_t.clone()
    tm[avail[:, 1:] == 0] = -9999
    out = torch.zeros((B, T - 1, n))
    for bn in range(B):
        for t in range(T - 1):
            r, c = scipy.optimize.linear_sum_assignment(tm[bn, t].numpy(), maximize=True)
            out[bn, t, :] = tm[bn, t, r, c]
    cpu_ms = (time.perf_counter() - t0) * 1e3
    assert torch.equal(sap_target_max_qvals(qd, ad).cpu(), out)
    return {"problems": B * (T - 1), "n": n, "m": m, "gpu_ms": round(gpu_ms, 3), "scipy_loop_ms": round(cpu_ms, 1),
            "speedup": round(cpu_ms / gpu_ms, 1)}


def bench_replay(E, buffer_size, n, m, T, L, batch_size, dev):
    env = AssignEnvBatch(n, m, T, L, 0.5, num_envs=E, device=dev)
    ep = EpisodeBatch(env.scheme, {"agents": n}, E, T + 1, preprocess=env.preprocess, device=dev, time_major=True)
    env.reset(ep, 0)
    for t in range(T):
        env.random_actions(ep, t)
        env.step(ep, t)
    buf = ReplayBuffer(env.scheme, {"agents": n}, buffer_size, T + 1, preprocess=env.preprocess, device=dev)
    ep_bytes = sum(v[0].numel() * v.element_size() for v in ep.data.transition_data.values())
    buf.insert_episode_batch(ep)
    ins_ms = timed(lambda: buf.insert_episode_batch(ep), 3)
    rng = np.random.RandomState(0)
    samp_ms = timed(lambda: buf.sample(batch_size, rng=rng), 5)
    return {"episodes_per_insert": E, "bytes_per_episode": ep_bytes, "insert_ms": round(ins_ms, 3),
            "insert_GBps": round(2 * E * ep_bytes / (ins_ms * 1e-3) / 1e9, 1),
            "sample_batch": batch_size, "sample_ms": round(samp_ms, 3),
            "sample_GBps": round(2 * batch_size * ep_bytes / (samp_ms * 1e-3) / 1e9, 1)}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--envs", type=int, default=4096)
    p.add_argument("--buffer", type=int, default=8192)
    p.add_argument("--lsa-batch", type=int, default=32)
    a = p.parse_args()
    dev = torch.device("cuda", 0)
    res = {"sap_targets": bench_sap_targets(a.lsa_batch, 21, 64, 64, dev),
           "replay": bench_replay(a.envs, a.buffer, 64, 64, 20, 3, 32, dev)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
