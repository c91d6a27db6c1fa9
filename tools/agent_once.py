"""Run the fused agent+select kernel `iters` times at the bench shape (for rocprofv3 PMC
passes: python3 tools/agent_once.py [iters])."""
import os
import sys
from types import SimpleNamespace

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from marl_sap_amd.action_selectors.classic_selectors import EpsilonGreedyActionSelector  # noqa: E402
from marl_sap_amd.modules.agents import RNNFusedAgent  # noqa: E402


def main(iters=10, E=16384, n=64, m=64, K=256):
    dev = torch.device("cuda", 0)
    args = SimpleNamespace(hidden_dim=64, use_rnn=True, m=m, epsilon_start=0.05, epsilon_finish=0.05,
                           epsilon_anneal_time=1, evaluation_epsilon=0.0, seed=0)
    fused = RNNFusedAgent(K, args).to(dev)
    x = torch.randn((E * n, K), device=dev)
    h = torch.randn((E * n, 64), device=dev)
    avail = torch.ones((E, n, m), dtype=torch.bool, device=dev)
    out = torch.empty((E, n), dtype=torch.int64, device=dev)
    sel = EpsilonGreedyActionSelector(args)
    with torch.no_grad():
        for _ in range(iters):
            e, s, c, st = sel.fused_params(0, False, dev)
            fused.forward_select(x, h, avail, n, e, s, c, out, st)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 10)
