"""Run bench.py's REDA leg alone (mock_constellation_reda.yaml: jumpstart_mac + the SAP selector,
Linear + ReLU agent, step_q schedule) for kernel-level profiling:
    rocprofv3 --kernel-trace --stats -- python3 tools/leg_reda.py [--steps 40]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    argv = sys.argv[1:]
    across = "--cold" not in argv  # --cold: each episode's first selection starts cold
    if not across:
        argv.remove("--cold")
    a = bench.parse(argv + ["--cpu-baseline", "0", "--secondary", "0"])
    dev = torch.device("cuda", 0)
    E = a.envs or bench.CONFIGS[a.config]["envs"]
    js = dict(mac="jumpstart_mac", use_rnn=False, jumpstart_action_selector="haa_selector",
              jumpstart_epsilon_start=1.0, jumpstart_epsilon_finish=0.0, jumpstart_epsilon_anneal_time=20000,
              jumpstart_evaluation_epsilon=0.0)
    r = bench.run_leg(a, dev, 1, E, a.steps, 2 * a.T, selector="sap", agent="rnn", count_lsa=False, **js,
                      epsilon_start=1.0, epsilon_finish=0.0, epsilon_anneal_time=20000,
                      sap_warm_across_episodes=across)
    print(json.dumps({"value": round(r["global_envs"] * a.steps / r["elapsed"], 1),
                      "ms_per_step": round(1e3 * r["elapsed"] / a.steps, 4),
                      "kernels_ms": bench.sap_kernels(r)}))


if __name__ == "__main__":
    main()
