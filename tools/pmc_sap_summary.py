"""Summarise the SQ counter pass of the SAP selector kernel (tools/round_profile.sh, the
`sq_sap` pass over `bench.py --selector sap`) into VALU instructions per augmenting-path step,
the figure bench.py's `roofline_lsa` sets against the VALU issue bound.

    python tools/pmc_sap_summary.py SQ_DIR BENCH_JSON_LOG OUT.json [--n 64 --m 64 --E 16384]

SQ_INSTS_VALU / SQ_INSTS_SALU are per-dispatch sums over all waves (wave instructions);
path steps per launch come from the same run's bench line (the instrumented kernel instance
counts scipy's inner-loop iterations on one selection of that run)."""
import argparse
import collections
import csv
import json
import os


def main():
    p = argparse.ArgumentParser()
    p.add_argument("sq_dir")
    p.add_argument("bench_log")
    p.add_argument("out")
    p.add_argument("--n", type=int, default=64)
    p.add_argument("--m", type=int, default=64)
    p.add_argument("--E", type=int, default=16384)
    p.add_argument("--kernel", default="sap_select_kernel<false",
                   help="kernel-name substring (bids: bids_select_kernel<false)")
    a = p.parse_args()
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(os.path.join(a.sq_dir, "run_counter_collection.csv"))):
        if a.kernel in r["Kernel_Name"]:
            per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    n = len(per)
    avg = {c: sum(d[c] for d in per.values()) / n for c in next(iter(per.values()))}
    line = json.loads([x for x in open(a.bench_log).read().splitlines() if x.startswith("{")][-1])
    lsa = line.get("roofline_lsa") or line["secondary"]["sap"]["roofline_lsa"]
    steps = lsa["path_steps_per_launch"]
    out = {"n": a.n, "m": a.m, "E": a.E, "kernel": "asg::" + a.kernel + ", *>", "dispatches_averaged": n,
           "counters": avg, "path_steps_per_launch": steps,
           "valu_insts_per_path_step": avg["SQ_INSTS_VALU"] / steps,
           "salu_insts_per_path_step": avg.get("SQ_INSTS_SALU", 0.0) / steps,
           "note": "per-dispatch SQ sums / augmenting-path steps of one launch of the same run"}
    if "SQ_WAVE_CYCLES" in avg:
        out["wait_any_frac"] = avg["SQ_WAIT_ANY"] / avg["SQ_WAVE_CYCLES"]
        out["wait_inst_any_frac"] = avg["SQ_WAIT_INST_ANY"] / avg["SQ_WAVE_CYCLES"]
        out["active_inst_any_frac"] = avg["SQ_ACTIVE_INST_ANY"] / avg["SQ_WAVE_CYCLES"]
        if "GRBM_GUI_ACTIVE" in avg:
            # SQ_WAVE_CYCLES counts quad-cycles summed over waves; GRBM_GUI_ACTIVE sums the 8 XCDs
            out["resident_waves_per_simd"] = 4 * avg["SQ_WAVE_CYCLES"] / (avg["GRBM_GUI_ACTIVE"] / 8 * 1024)
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps({k: v for k, v in out.items() if k != "counters"}))


if __name__ == "__main__":
    main()
