"""Multi-rank rollout on one GPU: GpuVecRunner sharded over 2 ranks
(one process per rank, gloo, both on cuda:0) gathers exactly the returns of a 1-rank run
over the same global envs, bitwise -- env draws, epsilon-greedy exploration and SAP noise
are all keyed by global env index -- and every rank's EpisodeBatch shard equals the
matching slice of the 1-rank batch.  Also runs bench.py's multi-rank branch under
torch.distributed.run.  Reference: runners/parallel_runner.py:178-179 (t_env over all
envs), :173-176 (per-env returns)."""
import json
import os
import socket
import subprocess
import sys

import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():
    pytest.skip("needs a ROCm GPU", allow_module_level=True)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, "tests", "dist_rollout_worker.py")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _launch(tmp, counts, eps, selector, episodes=2, tag="run", extra=(), timeout=100):
    world = len(counts)
    port = _free_port()
    procs, outs = [], []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), LOCAL_WORLD_SIZE=str(world))
        out = os.path.join(tmp, f"{tag}_w{world}_r{r}.pt")
        outs.append(out)
        procs.append(subprocess.Popen(
            [sys.executable, WORKER, out, ",".join(map(str, counts)), str(eps), selector, str(episodes), *extra],
            env=env, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    logs = []
    for p in procs:
        try:
            o, _ = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        logs.append(o.decode(errors="replace"))
    for p, log in zip(procs, logs):
        assert p.returncode == 0, log[-3000:]
    return [torch.load(o, weights_only=True) for o in outs]


@pytest.mark.parametrize("selector,eps,counts", [
    ("epsilon_greedy", 0.3, [24, 24]),
    ("epsilon_greedy", 0.0, [24, 24]),
    ("sap", 0.2, [24, 24]),
    ("epsilon_greedy", 0.3, [10, 38]),  # ragged shards: padded all-gather, sum(E_r) t_env
])
def test_two_rank_rollout_equals_one_rank(tmp_path, selector, eps, counts):
    total = sum(counts)
    (one,) = _launch(str(tmp_path), [total], eps, selector, tag="one")
    shards = _launch(str(tmp_path), counts, eps, selector, tag="two")
    base = 0
    for r, sh in enumerate(shards):
        assert sh["env_index_base"] == base and sh["rank_envs"] == counts
        for a, b in zip(sh["returns"], one["returns"]):
            assert a.dtype == torch.float64 and torch.equal(a, b)  # gathered = 1-rank returns, bitwise
        assert sh["t_env"] == one["t_env"] == [total * 6 * (e + 1) for e in range(len(one["t_env"]))]
        assert sh["train_returns"] == one["train_returns"]
        for k, v in one["batch"].items():
            assert torch.equal(sh["batch"][k], v[base:base + counts[r]]), k
        base += counts[r]
    if eps > 0 and selector == "epsilon_greedy":
        # exploration really happened and differs between envs (global keying, not per-rank copies)
        acts = one["batch"]["actions"][:, :6, :, 0]
        assert not torch.equal(acts[:counts[0]], acts[counts[0]:2 * counts[0]])


def test_bench_multi_rank_branch(tmp_path):
    """bench.py --gpus 2 through torch.distributed.run (gloo on one GPU): rank 0 prints one
    JSON line with the whole-job value over both ranks."""
    env = dict(os.environ, ASG_DIST_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "10", "--warmup", "3", "--envs", "256", "--cpu-baseline", "0",
           "--secondary", "0"]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["config"]["global_envs"] == 512 and line["value"] > 0
    assert line["scaling"] == "weak" and line["cpu_baseline"] is None
    # the self-explaining multi-rank keys: backend, per-rank kernel spread, returns all-gather time
    mr = line["multi_rank"]
    assert mr["backend"] == "gloo"
    assert len(mr["kernel_ms_per_rank"]) == 2 and 0 < mr["kernel_ms_min"] <= mr["kernel_ms_max"]
    # 13 steps from t = 0 at T = 20: the window holds no episode end, so no gather was timed
    assert mr["gathers_per_rank"] == 0 and mr["all_gather_returns_ms_max"] == 0.0
    r = subprocess.run(cmd[:-12] + ["--steps", "30", "--warmup", "3", "--envs", "256", "--cpu-baseline", "0",
                                   "--secondary", "0"], env=env, cwd=ROOT, capture_output=True, text=True,
                       timeout=110)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    mr = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])["multi_rank"]
    assert mr["gathers_per_rank"] == 1 and mr["all_gather_returns_ms_max"] > 0.0


def test_configs3_per_rank_size_and_rccl_rehearsal(tmp_path):
    """BASELINE configs[3] at its real per-rank size: 64 x 64 envs, 16,384 per rank, two ranks
    (gloo; two processes on the one GPU of the test box, 2 x 41 GB of batch shards) against a
    one-rank run over the same 32,768 global envs on an RCCL group (backend "nccl", world 1:
    init_process_group(device_id=...), device-tensor all_gather_into_tensor of the env counts
    and the returns, barrier(device_ids=...) -- the code path an 8-GPU node runs).  The
    gathered float64 returns are bitwise equal, every (env, field) checksum of the shards
    equals the one-rank batch's, and sampled env rows are equal.  Both schedules run the fused
    rollout kernel.  Reference: runners/parallel_runner.py:173-179, :220-221."""
    E = 16384
    sample = [0, E - 1, E, E + 4097, 2 * E - 1]
    common = ["--n", "64", "--m", "64", "--T", "20", "--checksums", "--sample", ",".join(map(str, sample))]
    (one,) = _launch(str(tmp_path), [2 * E], 0.05, "epsilon_greedy", episodes=1, tag="one",
                     extra=["--backend", "nccl", *common], timeout=300)
    assert one["backend"] == "nccl" and one["world"] == 1 and one["fused"]
    shards = _launch(str(tmp_path), [E, E], 0.05, "epsilon_greedy", episodes=1, tag="two",
                     extra=["--backend", "gloo", *common], timeout=300)
    assert one["t_env"] == [2 * E * 20]
    for r, sh in enumerate(shards):
        assert sh["backend"] == "gloo" and sh["world"] == 2 and sh["fused"]
        assert sh["env_index_base"] == r * E and sh["rank_envs"] == [E, E]
        assert sh["t_env"] == one["t_env"]
        assert torch.equal(sh["returns"][0], one["returns"][0])  # gathered returns, bitwise
        for k, c in one["checksums"].items():
            assert torch.equal(sh["checksums"][k], c[r * E:(r + 1) * E]), k
        for g, rows in sh["sample"].items():
            for k, v in rows.items():
                assert torch.equal(v, one["sample"][g][k]), (g, k)
    assert sum(len(sh["sample"]) for sh in shards) == len(sample)
    # the rollout really explored and the envs differ (global keying)
    assert not torch.equal(one["checksums"]["actions"][:E], one["checksums"]["actions"][E:])
