"""A/B microbenchmark of the action-selection path on one GPU (interleaved rounds in one
process): PyTorch RNNAgent + fused eps kernel, fused agent + eps kernel, fused agent+select."""
import sys
import os
import time
from types import SimpleNamespace

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from marl_sap_amd.action_selectors.classic_selectors import EpsilonGreedyActionSelector  # noqa: E402
from marl_sap_amd.modules.agents import RNNAgent, RNNFusedAgent  # noqa: E402


def main(E=16384, n=64, m=64, K=256, rounds=5, iters=20):
    dev = torch.device("cuda", 0)
    args = SimpleNamespace(hidden_dim=64, use_rnn=True, m=m, epsilon_start=0.05, epsilon_finish=0.05,
                           epsilon_anneal_time=1, evaluation_epsilon=0.0, seed=0)
    ref = RNNAgent(K, args).to(dev)
    fused = RNNFusedAgent(K, args).to(dev)
    fused.load_state_dict(ref.state_dict())
    x = torch.randn((E * n, K), device=dev)
    h = torch.randn((E * n, 64), device=dev)
    avail = torch.ones((E, n, m), dtype=torch.bool, device=dev)
    out = torch.empty((E, n), dtype=torch.int64, device=dev)
    sel = EpsilonGreedyActionSelector(args)

    def v_torch():
        q, h2 = ref(x, h)
        sel.select_action(q.view(E, n, m), avail, 0, out=out)

    def v_fwd():
        q, h2 = fused(x, h)
        sel.select_action(q.view(E, n, m), avail, 0, out=out)

    def v_sel():
        e, s, c, st = sel.fused_params(0, False, dev)
        fused.forward_select(x, h, avail, n, e, s, c, out, st)

    def v_fwd_only():
        fused(x, h)

    res = {k: [] for k in ["torch", "fused_fwd+eps", "fused_select", "fused_fwd_only"]}
    with torch.no_grad():
        for f in (v_torch, v_fwd, v_sel, v_fwd_only):
            f()
        torch.cuda.synchronize()
        for _ in range(rounds):
            for name, f in zip(res, (v_torch, v_fwd, v_sel, v_fwd_only)):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(iters):
                    f()
                b.record()
                torch.cuda.synchronize()
                res[name].append(a.elapsed_time(b) / iters)
    for k, v in res.items():
        v.sort()
        print(f"{k:16s} median {v[len(v) // 2]:.4f} ms  min {v[0]:.4f} ms")


if __name__ == "__main__":
    main()
