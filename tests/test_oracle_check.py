"""The exhaustive C replay checker (oracle/asg_check.c) against the Python replay it replaces
(oracle/check.py:replay_and_compare) on CPU: batches built by the oracle env itself pass, and
each corrupted field is caught at the env and row it was planted in.  Test infrastructure
checking test infrastructure -- the GPU tests then run it over every env of the timed sizes."""
import numpy as np
import pytest
import torch

from oracle import oracle as ora
from oracle.check import replay_all, replay_and_compare


def _oracle_batch(n, m, T, L, E, seed, quirks=()):
    """E envs rolled out by the oracle (same-seed streams seed + e, random actions) laid out
    as the GPU batch's [E, T+1, ...] tensors."""
    rng = np.random.default_rng(seed)
    W = m * (L + 1)
    td = {"obs": np.zeros((E, T + 1, n, W), np.float32), "beta": np.zeros((E, T + 1, n, m), np.float32),
          "actions": np.zeros((E, T + 1, n, 1), np.int64), "rewards": np.zeros((E, T + 1, n), np.float32),
          "actions_onehot": np.zeros((E, T + 1, n, m), np.int64), "terminated": np.zeros((E, T + 1, 1), bool),
          "prev_assigns": np.zeros((E, T + 1, n), np.int64), "avail_actions": np.ones((E, T + 1, n, m), bool),
          "filled": np.ones((E, T + 1, 1), np.int64)}
    tables, prev0, rets = [], [], []
    for e in range(E):
        env = ora.OracleMockEnv(n, m, T, L, 0.5, mt=ora.MT(seed + e))
        env.reset()
        tables.append(env.sat_prox_mat.copy())
        prev0.append(env.prev_assigns.copy())
        td["prev_assigns"][e, 0] = env.prev_assigns
        td["obs"][e, 0], td["beta"][e, 0] = env._obs, env.beta
        ret = 0.0
        for t in range(T):
            a = rng.integers(0, m, n)
            td["actions"][e, t, :, 0] = a
            r, done, _ = env.step(a)
            ret += sum(r)
            td["rewards"][e, t] = r
            td["obs"][e, t + 1], td["beta"][e, t + 1] = env._obs, env.beta
            td["actions_onehot"][e, t, np.arange(n), a] = 1
            td["terminated"][e, t, 0] = done
            td["prev_assigns"][e, t + 1] = a
        rets.append(ret)
    return ({k: torch.from_numpy(v) for k, v in td.items()}, torch.from_numpy(np.stack(tables)),
            torch.from_numpy(np.stack(prev0)), torch.tensor(rets, dtype=torch.float64))


def test_exhaustive_checker_agrees_with_python_replay():
    n, m, T, L, E, seed = 6, 9, 7, 3, 12, 40
    td, table, prev0, ret = _oracle_batch(n, m, T, L, E, seed)
    replay_and_compare(n, m, T, L, 0.5, table.numpy(), prev0.numpy(), {k: v.numpy() for k, v in td.items()},
                       ret.numpy())
    envs, compared = replay_all(n, m, T, L, 0.5, td, table, prev0, ret, env_chunk=5, threads=3)
    assert envs == E and compared > E * T * n * m
    # the same-seed mode: tables and permutations rebuilt from np.random.seed(seed + e)
    replay_all(n, m, T, L, 0.5, td, table, prev0, ret, seed=seed, env_chunk=4, threads=2)
    with pytest.raises(AssertionError, match="env 0: reset permutation"):
        replay_all(n, m, T, L, 0.5, td, table, prev0, ret, seed=seed + 1, threads=2)


@pytest.mark.parametrize("field,index,what", [
    ("obs", (7, 3, 2, 12), "env 7: obs row 3"),
    ("beta", (4, 0, 1, 1), "env 4: beta row 0"),
    ("rewards", (9, 5, 0), "env 9: rewards t=5"),
    ("actions_onehot", (2, 6, 4, 0), "env 2: actions_onehot t=6"),
    ("terminated", (11, 2, 0), "env 11: terminated t=2"),
    ("prev_assigns", (5, 4, 3), "env 5: prev_assigns row 4"),
    ("avail_actions", (3, 7, 5, 8), "env 3: avail_actions"),
    ("filled", (8, 7, 0), "env 8: filled row 7"),
])
def test_exhaustive_checker_catches_each_field(field, index, what):
    n, m, T, L, E, seed = 6, 9, 7, 3, 12, 41
    td, table, prev0, ret = _oracle_batch(n, m, T, L, E, seed)
    t = td[field]
    if t.dtype == torch.bool:
        t[index] = ~t[index]
    elif t.dtype == torch.float32:
        t[index] = torch.nextafter(t[index], torch.tensor(np.inf, dtype=torch.float32))
    else:
        t[index] = 1 - t[index] if field in ("actions_onehot", "filled") else t[index] + 1
    with pytest.raises(AssertionError, match=what):
        replay_all(n, m, T, L, 0.5, td, table, prev0, ret, env_chunk=5, threads=4)
    ret2 = ret.clone()
    ret2[6] += 1e-6
    td2, *_ = _oracle_batch(n, m, T, L, E, seed)
    with pytest.raises(AssertionError, match="env 6: return"):
        replay_all(n, m, T, L, 0.5, td2, table, prev0, ret2, threads=2)


def test_exhaustive_checker_philox_tolerance_and_quirks():
    n, m, T, L, E, seed = 5, 8, 6, 2, 6, 42
    td, table, prev0, ret = _oracle_batch(n, m, T, L, E, seed)
    # Philox mode: obs / beta within 2^-22 (relative) + 10 * 2^-22 (absolute) of float32(table)
    o = td["obs"][:, :, :, m:]
    td["obs"][:, :, :, m:] = torch.where(o > 0, o * (1 + 2.0 ** -23), o)
    with pytest.raises(AssertionError, match="obs row"):
        replay_all(n, m, T, L, 0.5, td, table, prev0, ret, threads=2)
    replay_all(n, m, T, L, 0.5, td, table, prev0, ret, philox=True, threads=2)
    # quirks: prev_assigns never written, ParallelRunner's terminated flags
    td["prev_assigns"][:, 1:] = 0
    td["terminated"][:, :T, 0] = True
    td["terminated"][0, :T, 0] = False
    replay_all(n, m, T, L, 0.5, td, table, prev0, ret, philox=True, threads=2,
               quirks=("prev_assigns_zero", "parallel_terminated"))
