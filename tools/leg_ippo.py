"""Run bench.py's ippo_sap leg alone (bids_as_actions + the continuous selector, step_q
schedule) for kernel-level A/B and profiling:  python3 tools/leg_ippo.py [--steps 40]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    a = bench.parse(sys.argv[1:] + ["--cpu-baseline", "0", "--secondary", "0"])
    dev = torch.device("cuda", 0)
    E = a.envs or bench.CONFIGS[a.config]["envs"]
    r = bench.run_leg(a, dev, 1, E, a.steps, a.warmup, selector="bids", agent="rnn", fused=None, count_lsa=False)
    print(json.dumps({"value": round(r["global_envs"] * a.steps / r["elapsed"], 1),
                      "ms_per_step": round(1e3 * r["elapsed"] / a.steps, 4),
                      "step_forward": r.get("step_forward_ms"), "bids_select": r.get("lsa_ms")}))


if __name__ == "__main__":
    main()
