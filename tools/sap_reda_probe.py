"""The SAP selector on REDA's own Q sequence (mock_constellation_reda.yaml as bench.py's `reda`
leg: JumpstartMAC, Linear agent, SAP at eps 0 after the jumpstart episode): captures the Q of
consecutive steps of one episode, then times (HIP events) and counts the augmenting-path steps
of cold (asg_sap_select_into) and warm-started (asg_sap_select_warm) selections of each.
GPU box, repo root:  python tools/sap_reda_probe.py [--eps 0.0]"""
import argparse
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from marl_sap_amd import _lib  # noqa: E402

p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--eps", type=float, default=0.0)
    ap.add_argument("--use-rnn", type=int, default=0)
    ap.add_argument("--save", default=None)
    o = ap.parse_args()
    a = bench.parse(["--cpu-baseline", "0", "--secondary", "0"])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from marl_sap_amd.controllers import REGISTRY as mac_REGISTRY
    from marl_sap_amd.runners import REGISTRY as r_REGISTRY
    js = dict(mac="jumpstart_mac", use_rnn=bool(o.use_rnn), jumpstart_action_selector="haa_selector",
              jumpstart_epsilon_start=0.0, jumpstart_epsilon_finish=0.0, jumpstart_epsilon_anneal_time=1,
              jumpstart_evaluation_epsilon=0.0, epsilon_start=o.eps, epsilon_finish=o.eps, epsilon_anneal_time=1)
    args = bench.make_args(a, a.envs, "sap", "rnn", 1, **js)
    runner = r_REGISTRY["gpu"](args, bench.NullLogger())
    env = runner.get_env()
    torch.manual_seed(a.seed)
    mac = mac_REGISTRY[args.mac](env.scheme, {"agents": a.n}, args)
    mac.to(dev)
    runner.setup(env.scheme, {"agents": a.n}, env.preprocess, mac)
    qs = []
    with torch.no_grad():
        runner.reset()
        mac.init_hidden(a.envs)
        mac.fused_mode(env, runner.batch, runner.t_env)
        runner.select_into_batch(0)
        for t in range(a.T - 1):
            mac.fused_step_select(env, runner.batch, t, runner.t_env)
            qs.append(mac._q_buf.view(a.envs, a.n, a.m).clone())
    torch.cuda.synchronize()
    B, n, m = qs[0].shape
    if "--save" in sys.argv:  # 64 envs' Q sequences for the host model (tools/lsa_fastpath_sim.py)
        import numpy as np
        np.save(sys.argv[sys.argv.index("--save") + 1], torch.stack([q[:64] for q in qs]).cpu().numpy())
    duals = torch.empty((B, 64), dtype=torch.float64, device=dev)
    L = _lib.lib()

    def call(q, warm, kind, counter):
        out = torch.empty((B, n), dtype=torch.int64, device=dev)
        st = torch.zeros((B,), dtype=torch.int32, device=dev)
        steps = torch.zeros((B,), dtype=torch.int32, device=dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for rep in range(2):  # rep 0 counts the steps, rep 1 is timed without the counting instance
            cnt = p(steps) if rep == 0 else None
            d = duals.clone() if kind == "warm" else None
            e0.record()
            if kind == "warm":
                _lib.check(L.asg_sap_select_warm(p(q), _lib.i64arr(q.stride()), B, n, m, o.eps, 3, counter, 0, p(out),
                                                 p(st), cnt, p(d), warm, _lib.stream_ptr(dev)))
            else:
                _lib.check(L.asg_sap_select_into(p(q), _lib.i64arr(q.stride()), B, n, m, o.eps, 3, counter, 0,
                                                 p(out), p(st), cnt, _lib.stream_ptr(dev)))
            e1.record()
            torch.cuda.synchronize()
            if rep == 0 and kind == "warm":
                newd = d
        s = steps.long()
        return out, e0.elapsed_time(e1), int((s & 0xFFFF).sum()), int((s >> 16).sum()), int(((s >> 16) > 0).sum()), \
            (newd if kind == "warm" else None)

    tot = {"cold": [0.0, 0, 0], "warm": [0.0, 0, 0]}
    for t, q in enumerate(qs):
        oc, tc, fc, ec, nc, _ = call(q, 0, "cold", t + 1)
        ow, tw, fw, ew, nw, nd = call(q, int(t > 0), "warm", t + 1)
        duals.copy_(nd)
        print(f"step {t + 1:2d}: cold {tc:.4f} ms fast {fc} exact {ec} ({nc} fallbacks) | warm {tw:.4f} ms fast {fw} "
              f"exact {ew} ({nw} fallbacks) same {bool(torch.equal(oc, ow))}", flush=True)
        if t > 0:
            for k, v in (("cold", (tc, fc, ec)), ("warm", (tw, fw, ew))):
                tot[k] = [tot[k][0] + v[0], tot[k][1] + v[1], tot[k][2] + v[2]]
    print({k: [round(v[0] / (len(qs) - 1), 4), v[1], v[2]] for k, v in tot.items()})


if __name__ == "__main__":
    main()
