#!/bin/bash
# One-line description of the GPU box (for box-to-box variance): CUs, partitions, clocks.
python3 - <<'PY'
import torch
p = torch.cuda.get_device_properties(0)
print("box: cus", p.multi_processor_count, "name", p.name, "gcn", getattr(p, "gcnArchName", "?"),
      "mem_gib", round(p.total_memory / 2**30), "l2", getattr(p, "L2_cache_size", "?"))
PY
rocm-smi --showcomputepartition --showmemorypartition 2>/dev/null | grep -i "partition" | head -4
rocm-smi --showmeminfo vram 2>/dev/null | grep -i "total" | head -2
cat /proc/cpuinfo | grep "model name" | head -1
