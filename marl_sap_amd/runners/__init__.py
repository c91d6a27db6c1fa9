"""Runner registry (reference: runners/__init__.py:1-7).  "gpu" is the batched HIP
runner; "episode" and "parallel" are aliases of it with the matching protocol, so an
existing config's `runner:` key keeps working."""
from functools import partial

from .gpu_runner import GpuVecRunner


def _with_protocol(protocol, args, logger):
    if not hasattr(args, "runner_protocol"):
        args.runner_protocol = protocol
    return GpuVecRunner(args, logger)


REGISTRY = {
    "gpu": GpuVecRunner,
    "episode": partial(_with_protocol, "episode"),
    "parallel": partial(_with_protocol, "parallel"),
}
