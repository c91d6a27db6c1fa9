"""HBM bytes of one RealConstellationEnv step from two rocprofv3 PMC passes (FETCH_SIZE and
WRITE_SIZE in separate --pmc runs of tools/bench_real_env.py, MI355X_MICROARCH.md's recipe):
the per-launch averages of the three kernels a step runs (real_transition_kernel,
real_strip_kernel, real_obs_kernel) summed.  FETCH_SIZE is doubled for the 16-B/lane streaming
reads the gfx950 note calibrates; the real kernels also read 8-B lanes (the float64 table
slices) and scattered words (the task-major totals), so both the raw and the doubled sums are
kept and the doubled one is reported as the step's traffic (an upper bound for the narrow reads).

    python tools/pmc_real_summary.py FETCH_DIR WRITE_DIR OUT.json --E 512
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import load  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("fetch_dir")
    p.add_argument("write_dir")
    p.add_argument("out")
    p.add_argument("--n", type=int, default=324)
    p.add_argument("--m", type=int, default=450)
    p.add_argument("--L", type=int, default=3)
    p.add_argument("--E", type=int, default=512)
    a = p.parse_args()
    fetch, write = load(a.fetch_dir, "FETCH_SIZE"), load(a.write_dir, "WRITE_SIZE")
    kernels, raw, dbl = {}, 0.0, 0.0
    for name in sorted(set(fetch) | set(write)):
        if "real_" not in name or "table_transpose" in name:
            continue
        f, w = fetch.get(name, []), write.get(name, [])
        if not f or not w:
            continue
        fk, wk = sum(f) / len(f), sum(w) / len(w)
        kernels[name] = {"launches": len(f), "fetch_kib": fk, "write_kib": wk}
        raw += (fk + wk) * 1024
        dbl += (2 * fk + wk) * 1024
    out = {"n": a.n, "m": a.m, "L": a.L, "E": a.E, "hbm_bytes_per_step": round(dbl), "hbm_bytes_per_step_raw": round(raw),
           "note": "sum over the step's kernels of the per-launch (2 FETCH_SIZE + WRITE_SIZE) KiB * 1024; raw = "
                   "FETCH_SIZE undoubled", "kernels": kernels}
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps({k: v for k, v in out.items() if k != "kernels"}))


if __name__ == "__main__":
    main()
