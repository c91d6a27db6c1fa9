"""Summarise the SQ counter pass of the fused agent kernel (tools/round_profile.sh, the `sq`
pass) into per-dispatch averages and the derived utilisation figures DESIGN.md quotes.

    python tools/pmc_agent_summary.py SQ_DIR KT_STATS_CSV OUT.json [--rows 1048576] [--note ...]

mfma_busy_frac = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE * 128): the busy counter sums
the SIMDs of the chip (256 CUs x 4) over cycles that GRBM_GUI_ACTIVE counts per XCD (x 8),
so the ratio is normalised by 1024 / 8.  Wait fractions are per wave cycle; instruction
counts are per 32-row wave tile (rows / 32 tiles per dispatch).
"""
import argparse
import collections
import csv
import json
import os


def derived(avg, tiles):
    """The utilisation figures the counters of this pass allow (two passes carry different sets)."""
    d = {}
    if "SQ_VALU_MFMA_BUSY_CYCLES" in avg and "GRBM_GUI_ACTIVE" in avg:
        d["mfma_busy_frac"] = avg["SQ_VALU_MFMA_BUSY_CYCLES"] / (avg["GRBM_GUI_ACTIVE"] * 128)
    if "SQ_WAVE_CYCLES" in avg:
        for c in ("SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_INST_LDS"):
            if c in avg:
                d[c[3:].lower() + "_frac"] = avg[c] / avg["SQ_WAVE_CYCLES"]
    for c in ("SQ_INSTS_MFMA", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_WR",
              "SQ_INSTS_VMEM_RD", "SQ_INSTS_SMEM", "SQ_LDS_BANK_CONFLICT"):
        if c in avg:
            d[c[3:].lower() + "_per_wave_tile"] = avg[c] / tiles
    return d


def main():
    p = argparse.ArgumentParser()
    p.add_argument("sq_dir")
    p.add_argument("kt_stats")
    p.add_argument("out")
    p.add_argument("--kernel", default="rnn_agent_lds_kernel")
    p.add_argument("--rows", type=int, default=16384 * 64)
    p.add_argument("--note", default="")
    p.add_argument("--n", type=int, default=None)
    p.add_argument("--m", type=int, default=None)
    p.add_argument("--E", type=int, default=None)
    p.add_argument("--L", type=int, default=None)
    p.add_argument("--steps-per-launch", type=int, default=1,
                   help="env steps one launch of the kernel runs (the whole-episode rollout: T)")
    p.add_argument("--use-rnn", type=int, default=1)
    a = p.parse_args()
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    name = None
    for r in csv.DictReader(open(os.path.join(a.sq_dir, "run_counter_collection.csv"))):
        if a.kernel in r["Kernel_Name"]:
            name = r["Kernel_Name"]
            per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    n = len(per)
    avg = {c: sum(d[c] for d in per.values()) / n for c in next(iter(per.values()))}
    kt_ms = None
    for r in csv.DictReader(open(a.kt_stats)):
        if a.kernel in r["Name"]:
            kt_ms = float(r["AverageNs"]) / 1e6
    tiles = a.rows / 32
    out = {k: getattr(a, k) for k in ("n", "m", "E", "L") if getattr(a, k) is not None}
    out["steps_per_launch"] = a.steps_per_launch
    out["use_rnn"] = bool(a.use_rnn)
    out.update({
        "kernel": (name or a.kernel).split("(")[0] + (f" -- {a.note}" if a.note else ""),
        "dispatches_averaged": n,
        "kernel_ms_from_kernel_trace": kt_ms,
        "counters": avg,
        "derived": derived(avg, tiles),
    })
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps(out["derived"]))


if __name__ == "__main__":
    main()
