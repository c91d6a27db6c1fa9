"""Time the fused agent+select kernel at the bench shape with whichever library
ASG_LIB_PATH names (A/B of kernel variants: run alternately per library, one process each).
Prints one line: lib, median ms over `rounds` rounds of `iters` launches."""
import os
import sys
from types import SimpleNamespace

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from marl_sap_amd.action_selectors.classic_selectors import EpsilonGreedyActionSelector  # noqa: E402
from marl_sap_amd.modules.agents import RNNFusedAgent  # noqa: E402


def main(E=16384, n=64, m=64, K=256, rounds=7, iters=30):
    dev = torch.device("cuda", 0)
    args = SimpleNamespace(hidden_dim=64, use_rnn=True, m=m, epsilon_start=0.05, epsilon_finish=0.05,
                           epsilon_anneal_time=1, evaluation_epsilon=0.0, seed=0)
    fused = RNNFusedAgent(K, args).to(dev)
    x = torch.rand((E * n, K), device=dev)
    if not os.environ.get("ASG_AB_DENSE"):  # the mock env's obs: onehot(previous task) first
        x[:, :m] = 0.0
        x[torch.arange(E * n, device=dev), torch.randint(0, m, (E * n,), device=dev)] = 1.0
    if os.environ.get("ASG_AB_L2X"):  # diagnostic: every row reads row 0 (L2-resident obs)
        x = torch.randn((1, K), device=dev).expand(E * n, K)
        fused._prep = lambda inputs, hid: (inputs, hid.reshape(-1, 64), 64)
    h = torch.randn((E * n, 64), device=dev)
    avail = torch.ones((E, n, m), dtype=torch.bool, device=dev)
    out = torch.empty((E, n), dtype=torch.int64, device=dev)
    sel = EpsilonGreedyActionSelector(args)
    res = []
    with torch.no_grad():
        for r in range(rounds + 1):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(iters):
                e, s, c, st, base = sel.fused_params(0, False, dev)
                fused.forward_select(x, h, avail, n, e, s, c, out, st, env_index_base=base)
            b.record()
            torch.cuda.synchronize()
            if r:
                res.append(a.elapsed_time(b) / iters)
    if os.environ.get("ASG_AB_STAMPS"):  # profiling build: phase stamps of workgroup 0's waves
        import ctypes
        import numpy as np
        from marl_sap_amd import _lib
        L = _lib.lib()
        buf = np.zeros((16, 4, 8), dtype=np.uint64)
        L.asg_debug_agent_stamps(buf.ctypes.data_as(ctypes.c_void_p))  # re-arm
        torch.cuda.synchronize()
        with torch.no_grad():
            e, s_, c, st, base = sel.fused_params(0, False, dev)
            fused.forward_select(x, h, avail, n, e, s_, c, out, st, env_index_base=base)
        torch.cuda.synchronize()
        L.asg_debug_agent_stamps(buf.ctypes.data_as(ctypes.c_void_p))
        order = [0, 1, 4, 5, 6, 2, 3, 7]
        names = ["fc1", "gru0", "gru1", "gru2", "gru3", "fc2", "select"]
        if os.environ.get("ASG_AB_STAMPS") == "fc1":  # -DASG_STAMP_FC1 builds
            order = [0, 4, 5, 6, 1, 2, 3, 7]
            names = ["prefix", "acc_init", "main_loop", "fc1_tail", "gru", "fc2", "select"]
        d = buf[:8, 1:4, :].astype(np.int64)  # waves 0-7, tiles 1-3 (steady state)
        phases = np.stack([d[..., order[k + 1]] - d[..., order[k]] for k in range(7)], axis=-1)
        med = np.median(phases.reshape(-1, 7), axis=0)
        print("stamps (s_memtime ticks, median over waves 0-7 x tiles 1-3):",
              {nm: int(v) for nm, v in zip(names, med)}, "tile total", int(med.sum()), flush=True)
    res.sort()
    print(f"{os.environ.get('ASG_LIB_PATH', 'default')} kernel={os.environ.get('ASG_AGENT_KERNEL', 'h2')} l2x={bool(os.environ.get('ASG_AB_L2X'))} K={K} m={m} median {res[len(res) // 2]:.4f} ms "
          f"min {res[0]:.4f}", flush=True)


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:]])
