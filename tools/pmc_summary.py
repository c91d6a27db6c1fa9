"""Summarise rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE collected in separate
--pmc runs, as MI355X_MICROARCH.md prescribes) into per-launch HBM bytes per kernel.

    python tools/pmc_summary.py FETCH_DIR WRITE_DIR OUT.json --kernel step_kernel --n 64 --m 64 --L 3 --E 16384

Units: rocprofv3 reports FETCH_SIZE / WRITE_SIZE in KiB.  gfx950 correction: FETCH_SIZE
counts exactly half of the bytes of a wide (16 B/lane) coalesced streaming read; it is
uncalibrated for narrower reads, so both the raw and the doubled fetch are recorded.
WRITE_SIZE is exact for 16-B-per-lane streaming stores (the env kernel's stores).
"""
import argparse
import collections
import csv
import json
import os


def load(d, counter):
    path = os.path.join(d, "run_counter_collection.csv")
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            agg[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return agg


def main():
    p = argparse.ArgumentParser()
    p.add_argument("fetch_dir")
    p.add_argument("write_dir")
    p.add_argument("out")
    p.add_argument("--kernel", default="step_kernel")
    p.add_argument("--n", type=int, default=64)
    p.add_argument("--m", type=int, default=64)
    p.add_argument("--L", type=int, default=3)
    p.add_argument("--E", type=int, default=16384)
    p.add_argument("--steps-per-launch", type=int, default=1,
                   help="env steps one launch of the kernel runs (the whole-episode rollout: T)")
    p.add_argument("--use-rnn", type=int, default=1)
    p.add_argument("--fetch-doubled", action="store_true",
                   help="headline bytes with FETCH_SIZE doubled (kernels whose reads are 16-B/lane streams)")
    a = p.parse_args()
    fetch, write = load(a.fetch_dir, "FETCH_SIZE"), load(a.write_dir, "WRITE_SIZE")
    kernels = {}
    for name in sorted(set(fetch) | set(write)):
        f = fetch.get(name, [])
        w = write.get(name, [])
        if not f or not w:
            continue
        fk, wk = sum(f) / len(f), sum(w) / len(w)
        kernels[name] = {"launches": len(f), "fetch_kib": fk, "write_kib": wk,
                         "hbm_bytes_raw": (fk + wk) * 1024, "hbm_bytes_fetch_doubled": (2 * fk + wk) * 1024}
    sel = [k for k in kernels if a.kernel in k]
    main_k = max(sel, key=lambda k: kernels[k]["write_kib"]) if sel else None
    out = {"n": a.n, "m": a.m, "L": a.L, "E": a.E, "kernel": main_k, "steps_per_launch": a.steps_per_launch,
           "use_rnn": bool(a.use_rnn),
           "hbm_bytes_per_launch": round(kernels[main_k]["hbm_bytes_fetch_doubled" if a.fetch_doubled
                                                 else "hbm_bytes_raw"]) if main_k else None,
           "note": ("(2 FETCH_SIZE + WRITE_SIZE)" if a.fetch_doubled else "(FETCH_SIZE + WRITE_SIZE)")
                   + " KiB * 1024 per launch, averaged over launches; separate --pmc passes; see kernels[] "
                     "for both variants",
           "kernels": kernels}
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps({k: v for k, v in out.items() if k != "kernels"}))


if __name__ == "__main__":
    main()
