"""Batched LSA microbenchmark (asg_lsa_batched / asg_haa_select, 1 GPU).

    python tools/bench_lsa.py [--iters 10]        (ASG_LIB_PATH selects a library variant)

Cases (B problems of n x m, one launch each):
  sap64_corr   16,384 x 64x64 f32, agent-like Q-values: a shared per-task profile plus a
               small per-agent term (rows highly correlated -> long augmenting paths, as
               the SAP selector sees with RNN Q-values) plus the selector's noise
  sap64_randn  16,384 x 64x64 f32, i.i.d. N(0, 1)
  ties64       16,384 x 64x64 f32, integers in {0, 1, 2} (tie-heavy: the slow path)
  f64_64       16,384 x 64x64 f64, i.i.d. N(0, 1)
  rect64x48    16,384 x 64x48 f32 (transposed working matrix)
  small16      4,096 x 16x16 f32
  big256       2,048 x 256x256 f32
  haa64        16,384 x 64x64 HAA selection (beta_hat + LSA fused)
Prints one JSON line: ms per launch, problems/s and an order-independent digest of the
assignments (to compare library variants for identical results).
"""
import argparse
import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from marl_sap_amd.action_selectors.lsa import linear_sum_assignment_batched  # noqa: E402
from marl_sap_amd.action_selectors.non_rl_selectors import haa_select_batched  # noqa: E402


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def digest(t):
    return hashlib.sha1(t.cpu().numpy().tobytes()).hexdigest()[:12]


def cases(dev, g):
    def randn(*s, dtype=torch.float32):
        return torch.randn(*s, generator=g, device=dev, dtype=dtype)

    B = 16384
    prof = randn(B, 1, 64)
    q = prof + 0.05 * randn(B, 64, 64)
    q = q + randn(B, 64, 64) * (q.abs().mean(dim=(1, 2), keepdim=True) * 0.1)
    yield "sap64_corr", q, True
    yield "sap64_randn", randn(B, 64, 64), True
    yield "ties64", torch.randint(0, 3, (B, 64, 64), generator=g, device=dev).float(), True
    yield "f64_64", randn(B, 64, 64, dtype=torch.float64), False
    yield "rect64x48", randn(B, 64, 48), True
    yield "small16", randn(4096, 16, 16), True
    yield "big256", randn(2048, 256, 256), True


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--iters", type=int, default=10)
    p.add_argument("--scan", action="store_true", help="sap64_corr at 1..16 problems per SIMD (latency vs occupancy)")
    a = p.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    g = torch.Generator(device=dev).manual_seed(0)
    if a.scan:
        prof = torch.randn((65536, 1, 64), generator=g, device=dev)
        q = prof + 0.05 * torch.randn((65536, 64, 64), generator=g, device=dev)
        res = {}
        for B in (256, 1024, 2048, 4096, 5120, 8192, 10240, 15360, 16384, 20480, 32768, 65536):
            ms = timed(lambda: linear_sum_assignment_batched(q[:B], maximize=True, return_status=True), a.iters)
            res[B] = round(ms, 4)
        print(json.dumps({"scan_sap64_corr_ms": res}))
        return
    out = {"lib": os.environ.get("ASG_LIB_PATH", "in-tree")}
    for name, C, maximize in cases(dev, g):
        _, col = linear_sum_assignment_batched(C, maximize=maximize)
        ms = timed(lambda: linear_sum_assignment_batched(C, maximize=maximize, return_status=True), a.iters)
        out[name] = {"B": C.shape[0], "shape": list(C.shape[1:]), "ms": round(ms, 4),
                     "problems_per_s": round(C.shape[0] / ms * 1e3), "digest": digest(col)}
        del C
    B = 16384
    beta = torch.rand((B, 64, 64), generator=g, device=dev) * (torch.rand((B, 64, 64), generator=g,
                                                                          device=dev) > 0.75)
    prev = torch.randint(0, 64, (B, 64), generator=g, device=dev)
    col = haa_select_batched(beta, prev, 0.5)
    ms = timed(lambda: haa_select_batched(beta, prev, 0.5), a.iters)
    out["haa64"] = {"B": B, "shape": [64, 64], "ms": round(ms, 4), "problems_per_s": round(B / ms * 1e3),
                    "digest": digest(col)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
