"""One rank of a sharded GPU rollout (launched by tests/test_gpu_dist_rollout.py, one
process per rank, every rank on cuda:0 of the one-GPU test box).

    RANK=r WORLD_SIZE=w MASTER_ADDR=127.0.0.1 MASTER_PORT=p \
        python tests/dist_rollout_worker.py OUT.pt E_0,E_1,... EPS SELECTOR EPISODES \
            [--backend gloo|nccl] [--n 16] [--m 16] [--T 6] [--checksums]

Builds GpuVecRunner (the drop-in runner) for this rank's envs, a BasicMAC whose weights
come from the same torch seed on every rank, runs EPISODES episodes and saves the gathered
returns, t_env and this rank's EpisodeBatch shard for the parent to compare with a
one-rank run over the same global envs (bitwise).

--checksums (the configs[3] size: 16,384 envs of 64 x 64 per rank, a 41 GB batch shard):
instead of the shard, save one 64-bit checksum per (env, field) -- the wrapping sum of the
field's raw bytes read as int64 words, times an odd per-word weight -- plus the full rows
of a few sampled global envs.  --backend nccl with WORLD_SIZE=1 is the RCCL rehearsal:
init_process_group("nccl", device_id=...), device-tensor all-gathers and the device
barrier of marl_sap_amd/dist.py run on a one-rank group."""
import argparse
import os
import sys
from types import SimpleNamespace

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


class _Logger:
    def log_stat(self, *a, **k):
        pass


def field_checksums(t):
    """[E, ...] tensor -> [E] int64: sum over the env's raw bytes as int64 words (zero-padded
    to 8 bytes) weighted by (2 * word index + 1), wrapping."""
    E = t.shape[0]
    out = torch.zeros(E, dtype=torch.int64, device=t.device)
    for c0 in range(0, E, 1024):  # bounded temporaries (the time-major field is a strided view)
        raw = t[c0:c0 + 1024].contiguous().view(torch.uint8).reshape(min(1024, E - c0), -1)
        pad = (-raw.shape[1]) % 8
        if pad:
            raw = torch.cat([raw, torch.zeros((raw.shape[0], pad), dtype=torch.uint8, device=raw.device)], 1)
        words = raw.view(torch.int64)
        w = torch.arange(words.shape[1], device=raw.device, dtype=torch.int64) * 2 + 1
        out[c0:c0 + 1024] = (words * w).sum(1)
    return out


def main():
    p = argparse.ArgumentParser()
    p.add_argument("out")
    p.add_argument("counts")
    p.add_argument("eps", type=float)
    p.add_argument("selector")
    p.add_argument("episodes", type=int)
    p.add_argument("--backend", default="gloo")
    p.add_argument("--n", type=int, default=16)
    p.add_argument("--m", type=int, default=16)
    p.add_argument("--T", type=int, default=6)
    p.add_argument("--checksums", action="store_true")
    p.add_argument("--sample", default="")
    a = p.parse_args()
    counts = [int(c) for c in a.counts.split(",")]
    from marl_sap_amd import dist as asg_dist
    rank, world = asg_dist.init_from_env(backend=a.backend, force=True)
    assert world == len(counts), (world, counts)
    import torch.distributed as dist
    assert dist.get_backend() == a.backend
    torch.cuda.set_device(asg_dist.local_device_index())
    from marl_sap_amd.controllers import REGISTRY as mac_REGISTRY
    from marl_sap_amd.runners import REGISTRY as r_REGISTRY
    n, m, T = a.n, a.m, a.T
    args = SimpleNamespace(
        batch_size_run=counts[rank], env="mock_constellation_env",
        env_args=dict(n=n, m=m, T=T, L=3, lambda_=0.5, bids_as_actions=False, seed=7),
        env_rng="philox", env_quirks=(), runner_protocol="episode", test_nepisode=1, runner_log_interval=10 ** 12,
        n=n, m=m, T=T, hidden_dim=64, use_rnn=True, obs_last_action=False, obs_agent_id=False,
        agent_output_type="q", action_selector=a.selector, agent="rnn_fused", mac="basic_mac", seed=3,
        epsilon_start=a.eps, epsilon_finish=a.eps, epsilon_anneal_time=1, evaluation_epsilon=0.0,
        reuse_batch=a.checksums)
    runner = r_REGISTRY["gpu"](args, _Logger())
    env = runner.get_env()
    torch.manual_seed(1234)  # identical agent weights on every rank
    mac = mac_REGISTRY["basic_mac"](env.scheme, {"agents": n}, args)
    mac.to(torch.device("cuda", torch.cuda.current_device()))
    runner.setup(env.scheme, {"agents": n}, env.preprocess, mac)
    res = {"returns": [], "t_env": [], "env_index_base": env.env_index_base, "rank_envs": runner.rank_envs,
           "backend": dist.get_backend(), "world": world}
    with torch.no_grad():
        res["fused"] = bool(mac.fused_step_ok(env, runner.new_batch() if not a.checksums else _probe(runner)))
    for _ in range(a.episodes):
        batch = runner.run(test_mode=False)
        assert runner.last_returns.is_cuda == (a.backend == "nccl")
        res["returns"].append(runner.last_returns.cpu())
        res["t_env"].append(runner.t_env)
    td = batch.data.transition_data
    if a.checksums:
        res["checksums"] = {k: field_checksums(v).cpu() for k, v in td.items()}
        base, E = env.env_index_base, counts[rank]
        res["sample"] = {}
        for g in (int(s) for s in a.sample.split(",") if s):
            if base <= g < base + E:
                res["sample"][g] = {k: v[g - base].cpu() for k, v in td.items()}
    else:
        res["batch"] = {k: v.cpu() for k, v in td.items()}
    res["train_returns"] = list(runner.train_returns)
    asg_dist.barrier()
    torch.save(res, a.out)
    dist.destroy_process_group()


def _probe(runner):
    from marl_sap_amd.components import EpisodeBatch
    return EpisodeBatch(runner.scheme, runner.groups, 1, runner.T + 1, preprocess=runner.preprocess,
                        device=runner.device, time_major=True)


if __name__ == "__main__":
    main()
