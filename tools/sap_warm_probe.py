"""Warm vs cold SAP fast path on consecutive selections (GPU box): per step, the fast-path and
exact-solver augmenting-path steps and the count of problems that fell back, for
(a) drifting SAP-like Q, (b) identical Q twice (warm from its own duals).
    python tools/sap_warm_probe.py"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from marl_sap_amd import _lib  # noqa: E402

DEV = torch.device("cuda", 0)
p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731


def run(q, eps, counter, duals=None, warm=0):
    B, n, m = q.shape
    out = torch.empty((B, n), dtype=torch.int64, device=DEV)
    st = torch.zeros((B,), dtype=torch.int32, device=DEV)
    steps = torch.zeros((B,), dtype=torch.int32, device=DEV)
    L = _lib.lib()
    if duals is None:
        _lib.check(L.asg_sap_select_into(p(q), _lib.i64arr(q.stride()), B, n, m, eps, 4, counter, 0, p(out), p(st),
                                         p(steps), _lib.stream_ptr(DEV)))
    else:
        _lib.check(L.asg_sap_select_warm(p(q), _lib.i64arr(q.stride()), B, n, m, eps, 4, counter, 0, p(out), p(st),
                                         p(steps), p(duals), warm, _lib.stream_ptr(DEV)))
    s = steps.long()
    return out, int((s & 0xFFFF).sum()), int((s >> 16).sum()), int(((s >> 16) > 0).sum())


def main():
    rng = np.random.RandomState(0)
    B, n = 1024, 64
    base = rng.normal(size=(B, 1, n)) + 0.05 * rng.normal(size=(B, n, n))
    duals = torch.empty((B, 64), dtype=torch.float64, device=DEV)
    for eps in (0.0, 0.05):
        print(f"eps {eps}")
        for t in range(6):
            q = torch.as_tensor((base + 0.01 * rng.normal(size=(B, n, n))).astype(np.float32), device=DEV)
            oc, fc, ec, nc = run(q, eps, t + 1)
            ow, fw, ew, nw = run(q, eps, t + 1, duals, int(t > 0))
            d = duals[:, :n]
            print(f"  t{t}: cold fast {fc} exact {ec} fallbacks {nc} | warm fast {fw} exact {ew} fallbacks {nw} "
                  f"same {bool(torch.equal(oc, ow))} duals finite {bool(torch.isfinite(d).all())} "
                  f"range {float(d.min()):.3g}..{float(d.max()):.3g}")
        q = torch.as_tensor((base + 0.01 * rng.normal(size=(B, n, n))).astype(np.float32), device=DEV)
        run(q, eps, 99, duals, 1)
        _, fw, ew, nw = run(q, eps, 99, duals, 1)
        print(f"  same Q twice: warm fast {fw} exact {ew} fallbacks {nw}")


if __name__ == "__main__":
    main()
