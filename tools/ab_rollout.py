"""Time the fused rollout step (asg_step_select) against the separate env step + fused agent
select at the bench shape, with whichever library ASG_LIB_PATH names (A/B of kernel
variants).  Prints one line: lib, median ms of fused and of step + select."""
import os
import sys
from types import SimpleNamespace

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from marl_sap_amd.action_selectors.classic_selectors import EpsilonGreedyActionSelector  # noqa: E402
from marl_sap_amd.components import EpisodeBatch  # noqa: E402
from marl_sap_amd.envs import AssignEnvBatch  # noqa: E402
from marl_sap_amd.modules.agents import RNNFusedAgent  # noqa: E402


def main(E=16384, n=64, m=64, L=3, T=20, rounds=7, iters=8):
    dev = torch.device("cuda", 0)
    args = SimpleNamespace(hidden_dim=64, use_rnn=True, m=m, epsilon_start=0.05, epsilon_finish=0.05,
                           epsilon_anneal_time=1, evaluation_epsilon=0.0, seed=0)
    env = AssignEnvBatch(n, m, T, L, 0.5, seed=1, num_envs=E, device=dev)
    batch = EpisodeBatch(env.scheme, {"agents": n}, E, T + 1, preprocess=env.preprocess, device=dev, time_major=True)
    agent = RNNFusedAgent(m * (L + 1), args).to(dev)
    sel = EpsilonGreedyActionSelector(args)
    h = torch.zeros((E * n, 64), device=dev)
    K = m * (L + 1)
    res_f, res_s = [], []
    with torch.no_grad():
        for r in range(rounds + 1):
            for mode in ("fused", "split"):
                env.reset(batch, 0)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for t in range(iters):
                    eps, seed, c, st, base = sel.fused_params(0, False, dev)
                    if mode == "fused":
                        h = env.step_select(batch, t, agent, h, eps, seed, c, st)
                    else:
                        env.step(batch, t)
                        x = batch["obs"][:, t + 1].reshape(E * n, K)
                        h = agent.forward_select(x, h, batch["avail_actions"][:, t + 1], n, eps, seed, c,
                                                 batch["actions"][:, t + 1, :, 0], st, env_index_base=base)
                e1.record()
                torch.cuda.synchronize()
                if r:
                    (res_f if mode == "fused" else res_s).append(e0.elapsed_time(e1) / iters)
    res_f.sort()
    res_s.sort()
    print(f"{os.environ.get('ASG_LIB_PATH', 'default')} fused {res_f[len(res_f) // 2]:.4f} ms "
          f"step+select {res_s[len(res_s) // 2]:.4f} ms", flush=True)


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:]])
