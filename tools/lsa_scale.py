import json, sys, os
sys.path.insert(0, os.getcwd())
import torch
from marl_sap_amd.action_selectors.lsa import linear_sum_assignment_batched
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
Bmax = 20480
prof = torch.randn(Bmax, 1, 64, generator=g, device=dev)
q = prof + 0.05 * torch.randn(Bmax, 64, 64, generator=g, device=dev)
q = q + torch.randn(Bmax, 64, 64, generator=g, device=dev) * (q.abs().mean(dim=(1, 2), keepdim=True) * 0.1)
out = {}
for B in (1024, 2560, 5120, 10240, 15360, 16384, 20480):
    x = q[:B].contiguous()
    linear_sum_assignment_batched(x, maximize=True)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(5):
        linear_sum_assignment_batched(x, maximize=True)
    b.record(); torch.cuda.synchronize()
    ms = a.elapsed_time(b) / 5
    out[B] = {"ms": round(ms, 4), "us_per_1k": round(ms / B * 1e6, 2)}
print(json.dumps(out))
