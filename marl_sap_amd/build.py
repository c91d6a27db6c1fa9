"""Build recipe for the HIP extension: one C-ABI shared library for gfx950.

    python -m marl_sap_amd.build        (or __graft_entry__.build())

Produces marl_sap_amd/libmarl_sap_amd.so in-tree (git-ignored, shipped to the GPU box
with the snapshot).  -ffp-contract=off keeps every float64 add/sub/mul of the env and
LSA kernels individually rounded, as numpy/scipy round them on the CPU.
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libmarl_sap_amd.so")
SOURCES = ["asg_abi.hip", "asg_env.hip", "asg_lsa.hip", "asg_select.hip", "asg_agent.hip", "asg_real.hip",
           "asg_filtered.hip", "asg_h2.hip", "asg_rollout_tab.hip", "asg_rollout_q.hip"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("ASG_OFFLOAD_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-shared", f"--offload-arch={ARCH}", "-ffp-contract=off",
         "-fno-gpu-rdc", "-Wall", "-Wno-unused-function"]


def needs_build():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, f) for f in os.listdir(CSRC)] + \
           [os.path.join(HERE, "..", "include", "asg.h")]
    return any(os.path.getmtime(d) > t for d in deps)


def build(force=False, verbose=False, out=None, extra=()):
    """Build the library (`out`/`extra`: experiment variants, e.g. -DASG_AGENT_WAVES=3 into
    build/, loaded with ASG_LIB_PATH; the product library is always LIB)."""
    if out is None and not force and not needs_build():
        return LIB
    target = out or LIB
    # one hipcc per source in parallel (the translation units are independent: -fno-gpu-rdc),
    # then one link
    import tempfile
    from concurrent.futures import ThreadPoolExecutor
    jobs = max(1, min(len(SOURCES), int(os.environ.get("MAX_JOBS", os.cpu_count() or 1))))
    with tempfile.TemporaryDirectory(prefix="asg_build_") as tmp:
        objs = [os.path.join(tmp, os.path.splitext(s)[0] + ".o") for s in SOURCES]
        compile_flags = [f for f in FLAGS if f != "-shared"]
        cmds = [[HIPCC] + compile_flags + list(extra) + ["-c", os.path.join(CSRC, s), "-o", o]
                for s, o in zip(SOURCES, objs)]
        if verbose:
            for c in cmds:
                print(" ".join(c))
        with ThreadPoolExecutor(jobs) as ex:
            results = list(ex.map(lambda c: subprocess.run(c, capture_output=True, text=True), cmds))
        for r in results:
            if r.returncode != 0:
                sys.stderr.write(r.stdout + r.stderr)
                raise RuntimeError("hipcc failed building libmarl_sap_amd.so")
        link = [HIPCC] + FLAGS + list(extra) + objs + ["-o", target + ".tmp"]
        r = subprocess.run(link, capture_output=True, text=True)
        if r.returncode != 0:
            sys.stderr.write(r.stdout + r.stderr)
            raise RuntimeError("hipcc failed linking libmarl_sap_amd.so")
    os.replace(target + ".tmp", target)
    return target


if __name__ == "__main__":
    argv = sys.argv[1:]
    out = None
    if "--out" in argv:
        out = os.path.abspath(argv[argv.index("--out") + 1])
        os.makedirs(os.path.dirname(out), exist_ok=True)
    extra = [a for a in argv if a.startswith("-D")]
    print(build(force="--force" in argv, verbose=True, out=out, extra=extra))
