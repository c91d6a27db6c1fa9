"""Where the first jumpstart (HAA) episode's time goes: bench.py's `iql` leg (configs[2],
jumpstart_mac + haa_selector, Linear agent) run alone under cProfile, twice in one process
(the second run shows the steady state).  GPU box, repo root:
    python tools/stall_probe.py OUT_DIR"""
import cProfile
import io
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    out = sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].startswith("--") else "gpurun_out/stall"
    os.makedirs(out, exist_ok=True)
    a = bench.parse(["--cpu-baseline", "0", "--secondary", "0"])
    if "--cpu" in sys.argv:  # bench.py's order: the CPU baseline (forked workers) before the GPU is touched
        t0 = time.perf_counter()
        bench.cpu_baseline(a)
        print(f"cpu baseline: {time.perf_counter() - t0:.3f} s", flush=True)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    js = dict(mac="jumpstart_mac", use_rnn=False, jumpstart_action_selector="haa_selector",
              jumpstart_epsilon_start=1.0, jumpstart_epsilon_finish=0.0, jumpstart_epsilon_anneal_time=20000,
              jumpstart_evaluation_epsilon=0.0, epsilon_start=1.0, epsilon_finish=0.0, epsilon_anneal_time=20000)
    # the legs bench.py runs before its `iql` leg (main, pytorch_agent, step / split schedules, sap)
    if "--alone" not in sys.argv:
        sk, sw = a.T, 5
        for kw in (dict(), dict(selector="eps", agent="rnn_torch"), dict(fused=3), dict(fused=0),
                   dict(selector="sap", agent="rnn", count_lsa=True)):
            t0 = time.perf_counter()
            bench.run_leg(a, dev, 1, a.envs, sk, sw, **kw)
            print(f"leg {kw}: {time.perf_counter() - t0:.3f} s", flush=True)
    for rep in range(2):
        pr = cProfile.Profile()
        t0 = time.perf_counter()
        pr.enable()
        res = bench.run_leg(a, dev, 1, a.envs, a.T, a.T, selector="eps", agent="rnn", **js)
        pr.disable()
        wall = time.perf_counter() - t0
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(45)
        with open(os.path.join(out, f"profile_rep{rep}.txt"), "w") as f:
            f.write(f"wall {wall:.3f} s, warmup {res['warmup_elapsed']:.3f} s, timed {res['elapsed']:.4f} s\n")
            f.write(s.getvalue())
        print(f"rep {rep}: wall {wall:.3f} s, warmup (jumpstart episode) {res['warmup_elapsed']:.3f} s", flush=True)


if __name__ == "__main__":
    main()
