"""Multi-process path on CPU (gloo, world_size 2): the once-per-episode collectives of
the sharded rollout -- all-gather of per-rank float64 returns in global env order and the
all-reduce of env-step counters -- plus the per-rank env-index partition."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, E, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from marl_sap_amd import dist as asg_dist
    r, w = asg_dist.init_from_env(backend="gloo")
    assert (r, w) == (rank, world)
    base = r * E  # GpuVecRunner: env_index_base = rank * batch_size_run
    local = torch.arange(base, base + E, dtype=torch.float64) * 0.5 + 0.25
    counts = asg_dist.envs_per_rank(E)
    assert counts == [E] * world and asg_dist.env_index_base(counts, r) == base
    allr = asg_dist.all_gather_returns(local, counts)
    steps = asg_dist.all_reduce_sum(E * 20)
    # ragged shards (rank r owns E + r envs): padded gather, stripped in global env order
    Er = E + r
    counts = asg_dist.envs_per_rank(Er)
    rb = asg_dist.env_index_base(counts, r)
    ragged = asg_dist.all_gather_returns(torch.arange(rb, rb + Er, dtype=torch.float64), counts)
    asg_dist.barrier()
    q.put((rank, allr.tolist(), steps, counts, ragged.tolist()))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_gather_returns_and_counters(world):
    E = 5
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, E, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    expect = [e * 0.5 + 0.25 for e in range(world * E)]
    for rank, allr, steps, counts, ragged in res:
        assert allr == expect
        assert steps == world * E * 20
        assert counts == [E + r for r in range(world)]
        assert ragged == [float(i) for i in range(sum(counts))]


def test_single_process_is_identity():
    from marl_sap_amd import dist as asg_dist
    t = torch.arange(3, dtype=torch.float64)
    assert asg_dist.rank_world() == (0, 1)
    assert asg_dist.all_gather_returns(t) is t and asg_dist.all_reduce_sum(7) == 7
