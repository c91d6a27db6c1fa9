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
    out.update({
        "kernel": (name or a.kernel).split("(")[0] + (f" -- {a.note}" if a.note else ""),
        "dispatches_averaged": n,
        "kernel_ms_from_kernel_trace": kt_ms,
        "counters": avg,
        "derived": {
            "mfma_busy_frac": avg["SQ_VALU_MFMA_BUSY_CYCLES"] / (avg["GRBM_GUI_ACTIVE"] * 128),
            "wait_inst_any_frac": avg["SQ_WAIT_INST_ANY"] / avg["SQ_WAVE_CYCLES"],
            "wait_any_frac": avg["SQ_WAIT_ANY"] / avg["SQ_WAVE_CYCLES"],
            "mfma_insts_per_wave_tile": avg["SQ_INSTS_MFMA"] / tiles,
            "valu_insts_per_wave_tile": avg["SQ_INSTS_VALU"] / tiles,
        },
    })
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps(out["derived"]))


if __name__ == "__main__":
    main()
