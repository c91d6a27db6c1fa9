"""Per-kernel register / scratch / spill table of one HIP source (hipcc's
kernel-resource-usage remarks), e.g.
    python tools/kernel_resources.py marl_sap_amd/csrc/asg_h2.hip rollout_kernel"""
import re
import subprocess
import sys

src = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else ""
extra = sys.argv[3:]
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-ffp-contract=off",
       "-fno-gpu-rdc", "-c", src, "-o", "/tmp/_kres.o", "-Rpass-analysis=kernel-resource-usage", *extra]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark: (.*?) \[-Rpass", line)
    if not m:
        continue
    t = m.group(1).strip()
    if t.startswith("Function Name:"):
        cur = {"name": t.split(":", 1)[1].strip()}
        rows.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.split(":", 1)
        cur[k.strip()] = v.strip()
keys = ["VGPRs", "AGPRs", "SGPRs", "ScratchSize [bytes/lane]", "SGPRs Spill", "VGPRs Spill", "Occupancy [waves/SIMD]",
        "LDS Size [bytes/block]"]
print("name".ljust(64), " ".join(k.split(" [")[0][:8].rjust(8) for k in keys))
for r in rows:
    if pat in r["name"]:
        print(r["name"][:64].ljust(64), " ".join(str(r.get(k, "-")).rjust(8) for k in keys))
