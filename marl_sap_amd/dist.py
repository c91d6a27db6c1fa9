"""Multi-GPU plumbing: one process per GPU under torch.distributed (backend "nccl" is
RCCL on ROCm; "gloo" for CPU tests).  Envs are independent, so nothing is exchanged per
step; once per episode the float64 returns are all-gathered (env order = global env
index) and the env-step counter is all-reduced."""
import os

import torch
import torch.distributed as dist


def rank_world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def init_from_env(backend=None):
    """Initialise the default process group from torchrun's env vars (no-op for 1 rank)."""
    if int(os.environ.get("WORLD_SIZE", "1")) <= 1 or (dist.is_available() and dist.is_initialized()):
        return rank_world()
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if backend is None:
        backend = os.environ.get("ASG_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
    if backend == "nccl":
        torch.cuda.set_device(local)
        dist.init_process_group(backend, device_id=torch.device("cuda", local))
    else:
        dist.init_process_group(backend)
    return rank_world()


def local_device_index():
    """GPU of this rank: LOCAL_RANK (one process per GPU); ranks beyond the visible GPUs
    wrap around (only meaningful for gloo rehearsals of the multi-rank path)."""
    n = torch.cuda.device_count()
    return int(os.environ.get("LOCAL_RANK", "0")) % max(1, n)


def all_gather_returns(local):
    """[E] per-rank returns -> [world * E] in global env order."""
    rank, world = rank_world()
    if world == 1:
        return local
    if dist.get_backend() == "gloo" and local.is_cuda:
        local = local.cpu()
    out = torch.empty(world * local.numel(), dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(out, local.contiguous())
    return out


def all_reduce_sum(value):
    rank, world = rank_world()
    if world == 1:
        return int(value)
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([int(value)], dtype=torch.int64, device=dev)
    dist.all_reduce(t)
    return int(t.item())


def barrier():
    if rank_world()[1] > 1:
        if dist.get_backend() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()
