"""One rank of a sharded GPU rollout (launched by tests/test_gpu_dist_rollout.py, one
process per rank, gloo backend, every rank on cuda:0 of the one-GPU test box).

    RANK=r WORLD_SIZE=w MASTER_ADDR=127.0.0.1 MASTER_PORT=p \
        python tests/dist_rollout_worker.py OUT.pt E_0,E_1,... EPS SELECTOR EPISODES

Builds GpuVecRunner (the drop-in runner) for this rank's envs, a BasicMAC whose weights
come from the same torch seed on every rank, runs EPISODES episodes and saves the gathered
returns, t_env and this rank's EpisodeBatch shard for the parent to compare with a
one-rank run over the same global envs (bitwise)."""
import os
import sys
from types import SimpleNamespace

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


class _Logger:
    def log_stat(self, *a, **k):
        pass


def main():
    out, counts, eps, selector, episodes = sys.argv[1], sys.argv[2], float(sys.argv[3]), sys.argv[4], int(sys.argv[5])
    counts = [int(c) for c in counts.split(",")]
    from marl_sap_amd import dist as asg_dist
    rank, world = asg_dist.init_from_env(backend="gloo")
    assert world == len(counts), (world, counts)
    torch.cuda.set_device(asg_dist.local_device_index())
    from marl_sap_amd.controllers import REGISTRY as mac_REGISTRY
    from marl_sap_amd.runners import REGISTRY as r_REGISTRY
    n = m = 16
    T = 6
    args = SimpleNamespace(
        batch_size_run=counts[rank], env="mock_constellation_env",
        env_args=dict(n=n, m=m, T=T, L=3, lambda_=0.5, bids_as_actions=False, seed=7),
        env_rng="philox", env_quirks=(), runner_protocol="episode", test_nepisode=1, runner_log_interval=10 ** 12,
        n=n, m=m, T=T, hidden_dim=64, use_rnn=True, obs_last_action=False, obs_agent_id=False,
        agent_output_type="q", action_selector=selector, agent="rnn_fused", mac="basic_mac", seed=3,
        epsilon_start=eps, epsilon_finish=eps, epsilon_anneal_time=1, evaluation_epsilon=0.0)
    runner = r_REGISTRY["gpu"](args, _Logger())
    env = runner.get_env()
    torch.manual_seed(1234)  # identical agent weights on every rank
    mac = mac_REGISTRY["basic_mac"](env.scheme, {"agents": n}, args)
    mac.to(torch.device("cuda", torch.cuda.current_device()))
    runner.setup(env.scheme, {"agents": n}, env.preprocess, mac)
    res = {"returns": [], "t_env": [], "env_index_base": env.env_index_base, "rank_envs": runner.rank_envs}
    for _ in range(episodes):
        batch = runner.run(test_mode=False)
        res["returns"].append(runner.last_returns.cpu())
        res["t_env"].append(runner.t_env)
    res["batch"] = {k: v.cpu() for k, v in batch.data.transition_data.items()}
    res["train_returns"] = list(runner.train_returns)
    torch.save(res, out)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
