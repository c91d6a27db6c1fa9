"""Multi-GPU plumbing: one process per GPU under torch.distributed (backend "nccl" is
RCCL on ROCm; "gloo" for CPU tests).  Envs are independent, so nothing is exchanged per
step.  The per-rank env counts are all-gathered once, at runner construction (the
env-step counter of an episode is then T * sum_r E_r on every rank with no per-episode
collective), and once per episode the float64 returns are all-gathered in global env
order (reference runners/parallel_runner.py:173-179, :220-221).

Every collective here runs whenever a process group is initialised, world size 1
included, so a one-rank RCCL job (`init_from_env(force=True)`) executes the same
device-tensor all-gathers and barrier as an 8-GPU one."""
import os

import torch
import torch.distributed as dist


def rank_world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def _initialized():
    return dist.is_available() and dist.is_initialized()


def init_from_env(backend=None, force=False):
    """Initialise the default process group from torchrun's env vars (no-op for 1 rank
    unless `force`: a one-rank group runs the real collectives, e.g. an RCCL rehearsal)."""
    if (int(os.environ.get("WORLD_SIZE", "1")) <= 1 and not force) or _initialized():
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


def all_gather_returns(local, counts=None):
    """[E_r] per-rank returns -> [sum_r E_r] in global env order.  counts: every rank's
    E_r (from envs_per_rank); equal counts (the sharded rollout) take one
    all_gather_into_tensor, ragged ones are padded to the largest shard and stripped."""
    if not _initialized():
        return local
    rank, world = rank_world()
    if dist.get_backend() == "gloo" and local.is_cuda:
        local = local.cpu()
    local = local.contiguous()
    if counts is None or len(set(counts)) == 1:
        out = torch.empty(world * local.numel(), dtype=local.dtype, device=local.device)
        dist.all_gather_into_tensor(out, local)
        return out
    mx = max(counts)
    pad = torch.zeros(mx, dtype=local.dtype, device=local.device)
    pad[:local.numel()] = local
    out = torch.empty(world * mx, dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(out, pad)
    return torch.cat([out[r * mx:r * mx + c] for r, c in enumerate(counts)])


def envs_per_rank(local_envs):
    """Every rank's env count (one all-gather at runner construction): the env-step
    counter of an episode is T * sum(E_r), the reference's per-env accounting
    (parallel_runner.py:178-179, :220-221) summed over ranks."""
    if not _initialized():
        return [int(local_envs)]
    rank, world = rank_world()
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([int(local_envs)], dtype=torch.int64, device=dev)
    out = torch.empty(world, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(out, t)
    return [int(x) for x in out.tolist()]


def env_index_base(counts, rank):
    """Global index of this rank's env 0: envs [sum(counts[:rank]), ... + counts[rank])."""
    return int(sum(counts[:rank]))


def all_reduce_sum(value):
    if not _initialized():
        return int(value)
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([int(value)], dtype=torch.int64, device=dev)
    dist.all_reduce(t)
    return int(t.item())


def barrier():
    if _initialized():
        if dist.get_backend() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()
