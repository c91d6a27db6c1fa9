"""GPU parity tests: the HIP path (through the C-ABI) against the CPU oracle and the
golden vectors captured from the reference.  Bar (BASELINE.json north_star): integer
assignments / masks bit-exact; float observations / rewards within 1e-5 -- in practice
the float32 values written to the EpisodeBatch are bit-identical to float32(oracle f64).
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # collected on CPU, but never run there
    pytest.skip("needs a ROCm GPU", allow_module_level=True)

from marl_sap_amd.action_selectors.lsa import linear_sum_assignment_batched  # noqa: E402
from marl_sap_amd.components import EpisodeBatch  # noqa: E402
from marl_sap_amd.envs import AssignEnvBatch, MockConstellationEnv  # noqa: E402
from oracle import oracle as ora  # noqa: E402
from oracle.check import replay_and_compare  # noqa: E402

DEV = torch.device("cuda", 0)


def new_batch(env, E, time_major=True):
    return EpisodeBatch(env.scheme, {"agents": env.n}, E, env.T + 1, preprocess=env.preprocess, device=DEV,
                        time_major=time_major)


def host(batch):
    return {k: v.cpu().numpy() for k, v in batch.data.transition_data.items()}


# ------------------------------------------------------------------------------ LSA
def test_lsa_golden(golden):
    g = golden("lsa")
    for k in range(int(g["n_cases"])):
        C = g[f"k{k}_C"]
        if C.size == 0:
            continue
        row, col = linear_sum_assignment_batched(torch.as_tensor(C, device=DEV), maximize=bool(g[f"k{k}_max"]))
        np.testing.assert_array_equal(row[0].cpu().numpy(), g[f"k{k}_row"], err_msg=str(k))
        np.testing.assert_array_equal(col[0].cpu().numpy(), g[f"k{k}_col"], err_msg=str(k))
    for e in range(int(g["n_err"])):
        with pytest.raises(ValueError, match=str(g[f"e{e}_msg"])):
            linear_sum_assignment_batched(torch.as_tensor(g[f"e{e}_C"], device=DEV), maximize=bool(g[f"e{e}_max"]))


@pytest.mark.parametrize("shape,kind,dtype", [
    ((512, 64, 64), "normal", np.float32), ((256, 64, 64), "int3", np.float32),
    ((128, 16, 16), "int2", np.float64), ((64, 20, 37), "round1", np.float64),
    ((64, 37, 20), "round1", np.float64), ((32, 100, 130), "normal", np.float64),
    ((8, 256, 256), "int3", np.float32), ((4, 300, 300), "normal", np.float64),
    # float32 <= 64 x 64 runs register-resident (both orientations, degenerate shapes)
    ((256, 64, 48), "normal", np.float32), ((256, 48, 64), "normal", np.float32),
    ((64, 1, 64), "normal", np.float32), ((64, 64, 1), "normal", np.float32),
    ((256, 33, 40), "int2", np.float32), ((256, 64, 64), "corr", np.float32),
    # float32 keys collide while float64 values differ (the exact selection path)
    ((256, 64, 64), "near64", np.float64), ((256, 40, 64), "near32", np.float32)])
def test_lsa_random_batches_vs_oracle(shape, kind, dtype):
    rng = np.random.RandomState(sum(shape) * 31 + len(kind))
    if kind == "normal":
        C = rng.normal(size=shape)
    elif kind == "corr":  # SAP-like Q-values: shared task profile + small per-agent term
        C = rng.normal(size=(shape[0], 1, shape[2])) + 0.05 * rng.normal(size=shape)
    elif kind == "near64":
        C = 1.0 + rng.randint(0, 1000, size=shape) * 2.0 ** -40
    elif kind == "near32":
        C = 1.0 + rng.randint(0, 8, size=shape) * 2.0 ** -23
    elif kind == "int3":
        C = rng.randint(0, 3, size=shape).astype(np.float64)
    elif kind == "int2":
        C = rng.randint(0, 2, size=shape).astype(np.float64)
    else:
        C = np.round(rng.uniform(size=shape), 1)
    C = C.astype(dtype)
    for maximize in (True, False):
        row, col = linear_sum_assignment_batched(torch.as_tensor(C, device=DEV), maximize=maximize)
        row, col = row.cpu().numpy(), col.cpu().numpy()
        for b in range(shape[0]):
            r0, c0 = ora.lsa(C[b].astype(np.float64), maximize=maximize)
            assert np.array_equal(row[b], r0) and np.array_equal(col[b], c0), (b, maximize)


def test_lsa_strided_and_status():
    rng = np.random.RandomState(5)
    big = torch.as_tensor(rng.normal(size=(6, 20, 24)), device=DEV)
    C = big[:, 2:18, 4:20].transpose(1, 2)  # non-contiguous view
    row, col = linear_sum_assignment_batched(C, maximize=True)
    for b in range(6):
        r0, c0 = ora.lsa(C[b].cpu().numpy(), maximize=True)
        assert np.array_equal(col[b].cpu().numpy(), c0)
    bad = torch.ones((3, 4, 4), device=DEV, dtype=torch.float64)
    bad[1, 2, 2] = float("nan")
    _, col, status = linear_sum_assignment_batched(bad, return_status=True)
    assert status.cpu().tolist() == [0, -4, 0]
    assert (col[1] == -1).all()


def test_lsa_register_path_status():
    """float32 <= 64 x 64 (register-resident working matrix): scipy's errors per matrix."""
    C = torch.as_tensor(np.random.RandomState(3).normal(size=(5, 6, 6)), device=DEV, dtype=torch.float32)
    C[1, 2, 3] = float("nan")                # invalid
    C[2, 0, :] = float("inf")                # row 0 has no finite entry: infeasible
    C[3, 4, 1] = -float("inf")               # invalid when minimizing
    C[4, 5, 5] = float("inf")                # feasible: +inf is only avoided
    _, col, status = linear_sum_assignment_batched(C, return_status=True)
    assert status.cpu().tolist() == [0, -4, -5, -4, 0]
    for b in (0, 4):
        assert np.array_equal(col[b].cpu().numpy(), ora.lsa(C[b].cpu().numpy().astype(np.float64))[1])
    _, _, st_max = linear_sum_assignment_batched(C[4:5], maximize=True, return_status=True)
    assert st_max.cpu().tolist() == [-4]     # +inf becomes -inf under maximize
    with pytest.raises(ValueError, match="infeasible"):
        linear_sum_assignment_batched(C[2:3])


# ------------------------------------------------------------------------------ beta_hat / HAA
def test_beta_hat_golden(golden):
    g = golden("mock_step")
    n, m = g["bh_beta"].shape[1:]
    env = AssignEnvBatch(n, m, 4, 2, float(g["bh_lambda"]), T_trans=g["bh_T_trans"], num_envs=1, device=DEV)
    out = env.beta_hat(torch.as_tensor(g["bh_beta"], device=DEV), torch.as_tensor(g["bh_prev"], device=DEV))
    np.testing.assert_array_equal(out.cpu().numpy(), g["bh_out"])
    out2 = env.beta_hat(g["bh_beta"][0], g["bh_prev"][0])
    np.testing.assert_array_equal(out2.cpu().numpy(), g["bh_out2d"])


@pytest.mark.parametrize("n,m,custom_T", [(8, 8, False), (16, 24, True), (64, 64, False), (100, 128, False)])
def test_haa_select_vs_oracle(n, m, custom_T):
    from types import SimpleNamespace

    from marl_sap_amd.action_selectors.non_rl_selectors import HAASelector
    rng = np.random.RandomState(n * 1000 + m)
    B = 64
    beta = rng.uniform(-0.5, 2.0, size=(B, n, m)).astype(np.float32)
    beta[beta < 0.2] = 0.0
    beta[:, 0, :3] = 1e-13
    prev = rng.randint(0, m, size=(B, n))
    T_trans = (rng.uniform(size=(m, m)) > 0.3).astype(np.float64) if custom_T else None
    env = AssignEnvBatch(n, m, 5, 2, 0.7, T_trans=T_trans, num_envs=B, device=DEV)
    sel = HAASelector(SimpleNamespace(m=m, env_args={"lambda_": 0.7}))
    sel.envs = env
    data = {"beta": torch.as_tensor(beta, device=DEV).unsqueeze(1),
            "prev_assigns": torch.as_tensor(prev, device=DEV).unsqueeze(1)}
    out = sel.select_action(_DictBatch(data)).cpu().numpy()
    sel.status.flush()
    for b in range(B):
        bh = ora.beta_hat(beta[b].astype(np.float64), prev[b], 0.7, T_trans)
        assert np.array_equal(out[b], ora.lsa(bh, maximize=True)[1].astype(np.float32)), b


def test_haa_non_finite_transition_matrix():
    """A NaN T_trans entry makes beta_hat invalid (scipy raises); the host check raises the
    same ValueError, and the kernel itself, fed the NaN directly through the ABI, still
    terminates with a per-env status (the solver's guard against NaN-only candidates)."""
    import ctypes

    from marl_sap_amd import _lib
    from marl_sap_amd.action_selectors.non_rl_selectors import haa_select_batched
    B, n, m = 8, 6, 8
    rng = np.random.RandomState(7)
    beta = torch.as_tensor(rng.uniform(0.0, 1.0, size=(B, n, m)).astype(np.float32), device=DEV)
    prev = torch.as_tensor(rng.randint(0, m, size=(B, n)), device=DEV)
    tt = np.ones((m, m)) - np.eye(m)
    tt[:, 3] = np.nan
    with pytest.raises(ValueError, match="invalid numeric entries"):
        haa_select_batched(beta, prev, 0.5, tt)
    tt_dev = torch.as_tensor(tt, device=DEV)
    out = torch.empty((B, n), dtype=torch.float32, device=DEV)
    status = torch.empty((B,), dtype=torch.int32, device=DEV)
    _lib.check(_lib.lib().asg_haa_select(
        ctypes.c_void_p(beta.data_ptr()), _lib.i64arr(beta.stride()), ctypes.c_void_p(prev.data_ptr()),
        _lib.i64arr(prev.stride()), B, n, m, ctypes.c_void_p(tt_dev.data_ptr()), 0.5,
        ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(status.data_ptr()), _lib.stream_ptr(DEV)))
    torch.cuda.synchronize()
    assert set(status.cpu().tolist()) <= {0, -4}


class _DictBatch:
    def __init__(self, d):
        self.d = d

    def __getitem__(self, k):
        return self.d[k]


# ------------------------------------------------------------------------------ env: MT19937 compat
def test_mt_construct_reset_golden(golden):
    g = golden("mock_reset")
    for c in range(int(g["n_cases"])):
        n, m, T, L, s = [int(x) for x in g[f"c{c}_shape"]]
        env = AssignEnvBatch(n, m, T, L, 0.5, seed=s, num_envs=1, device=DEV, rng="mt19937")
        b = new_batch(env, 1)
        env.reset(b, 0)
        tab = env.export_benefits()[0].cpu().numpy()
        np.testing.assert_allclose(tab, g[f"c{c}_table"], rtol=1e-12, atol=0, err_msg=str(c))
        np.testing.assert_array_equal(tab == 0, g[f"c{c}_table"] == 0)
        np.testing.assert_array_equal(env.export_prev_assigns()[0].cpu().numpy(), g[f"c{c}_prev_assigns"])
        td = host(b)
        np.testing.assert_array_equal(td["obs"][0, 0], g[f"c{c}_obs"].astype(np.float32))
        np.testing.assert_array_equal(td["beta"][0, 0], g[f"c{c}_beta"].astype(np.float32))
        assert td["avail_actions"][0, 0].all() and td["filled"][0, 0, 0] == 1


@pytest.mark.parametrize("replicate", [False, True])
def test_mt_multi_env_streams(replicate):
    n, m, T, L, s, E = 12, 16, 8, 3, 77, 5
    env = AssignEnvBatch(n, m, T, L, 0.5, seed=s, num_envs=E, device=DEV, rng="mt19937",
                         quirks=("replicate_stream",) if replicate else ())
    b = new_batch(env, E)
    for episode in range(2):
        env.reset(b, 0)
        tab = env.export_benefits().cpu().numpy()
        prev = env.export_prev_assigns().cpu().numpy()
        for e in range(E):
            mt = ora.MT(s if replicate else s + e)
            oe = ora.OracleMockEnv(n, m, T, L, 0.5, mt=mt)
            oe.reset()
            for _ in range(episode):
                oe.reset()
            np.testing.assert_allclose(tab[e], oe.sat_prox_mat, rtol=1e-12, atol=0)
            np.testing.assert_array_equal(prev[e], oe.prev_assigns)


@pytest.mark.parametrize("n,m,T,L", [(12, 16, 8, 3), (64, 64, 20, 3), (5, 9, 6, 2)])
def test_mt_generated_steps_exact_on_export(n, m, T, L):
    """Same-seed mode keeps no float64 table: the rows come from the reset's float32 table and
    the rewards / export evaluate the recorded draws.  Replaying the exported table through the
    oracle must reproduce every row bit for bit (obs == float32 of the export, rewards exact)."""
    E = 4
    env = AssignEnvBatch(n, m, T, L, 0.5, seed=21, num_envs=E, device=DEV, rng="mt19937")
    b = new_batch(env, E)
    for episode in range(2):
        env.reset(b, 0)
        table = env.export_benefits().cpu().numpy()
        prev0 = env.export_prev_assigns().cpu().numpy()
        for t in range(T):
            env.random_actions(b, t)
            env.step(b, t)
        env.sync()
        replay_and_compare(n, m, T, L, 0.5, table, prev0, host(b), env.get_returns().cpu().numpy())


def test_mt_injected_steps_golden(golden):
    """Injected tables (sat_prox_mat=) + fixed action sequences, incl. bids."""
    g = golden("mock_step")
    for c in range(int(g["n_cases"])):
        n, m, T, L = [int(x) for x in g[f"c{c}_spec"]]
        lam = float(g[f"c{c}_lambda"])
        kind = str(g[f"c{c}_kind"])
        bids = kind.startswith("bids")
        mt = ora.MT(100 + c)
        if kind != "dense":
            ora.generate(mt, n, m, T, 3.0, 6.0)
        env = AssignEnvBatch(n, m, T, L, lam, bids_as_actions=bids, seed=100 + c, sat_prox_mat=g[f"c{c}_table"],
                             num_envs=1, device=DEV, rng="mt19937", quirks=("prev_assigns_zero",))
        env.advance_stream(mt.drawn())
        b = new_batch(env, 1)
        env.reset(b, 0)
        np.testing.assert_array_equal(env.export_prev_assigns()[0].cpu().numpy(), g[f"c{c}_prev0"])
        ret = 0.0
        for t in range(T):
            a = torch.as_tensor(g[f"c{c}_actions"][t], device=DEV)
            b["actions"][0, t].copy_(a.reshape(b["actions"][0, t].shape).to(b["actions"].dtype))
            env.step(b, t)
            ret += g[f"c{c}_rewards"][t].sum()
        env.sync()
        td = host(b)
        np.testing.assert_array_equal(td["rewards"][0, :T], g[f"c{c}_rewards"].astype(np.float32), err_msg=kind)
        np.testing.assert_array_equal(td["obs"][0, 1:], g[f"c{c}_obs"].astype(np.float32))
        np.testing.assert_array_equal(td["beta"][0, 1:], g[f"c{c}_beta"].astype(np.float32))
        np.testing.assert_array_equal(td["terminated"][0, :T, 0], g[f"c{c}_done"])
        assert (td["prev_assigns"] == 0).all()
        if not bids:
            oh = np.zeros((T, n, m), np.int64)
            for t in range(T):
                oh[t, np.arange(n), g[f"c{c}_actions"][t]] = 1
            np.testing.assert_array_equal(td["actions_onehot"][0, :T], oh)
        assert abs(env.get_returns()[0].item() - ret) < 1e-9 * max(1, abs(ret))


# ------------------------------------------------------------------------------ env: Philox native
@pytest.mark.parametrize("n,m,T,L,lam,custom_T,time_major", [
    (8, 8, 6, 3, 0.5, False, True), (16, 16, 20, 3, 0.5, False, True), (7, 10, 5, 2, 0.25, False, True),
    (12, 12, 4, 6, 1.5, True, False), (64, 64, 20, 3, 0.5, False, True), (5, 9, 3, 0, 0.5, False, True)])
def test_philox_rollout_vs_oracle(n, m, T, L, lam, custom_T, time_major):
    E = 24
    rng = np.random.RandomState(n + m + T)
    T_trans = (rng.uniform(size=(m, m)) > 0.4).astype(np.float64) if custom_T else None
    env = AssignEnvBatch(n, m, T, L, lam, seed=9, num_envs=E, T_trans=T_trans, device=DEV)
    b = new_batch(env, E, time_major=time_major)
    for episode in range(2):
        env.reset(b, 0)
        table = env.export_benefits().cpu().numpy()
        prev0 = env.export_prev_assigns().cpu().numpy()
        for t in range(T):
            env.random_actions(b, t)
            env.step(b, t)
        env.sync()
        replay_and_compare(n, m, T, L, lam, table, prev0, host(b), env.get_returns().cpu().numpy(),
                           T_trans=T_trans, philox=True)


def test_philox_quirks_and_dense():
    n, m, T, L, E = 6, 8, 5, 2, 4
    env = AssignEnvBatch(n, m, T, L, 0.5, seed=3, num_envs=E, device=DEV,
                         quirks=("prev_assigns_zero", "parallel_terminated"), benefits="dense")
    b = new_batch(env, E)
    env.reset(b, 0)
    table = env.export_benefits().cpu().numpy()
    assert (table > 0).all()  # dense: every (i, j) pair has a bump (none underflows at T=5)
    prev0 = env.export_prev_assigns().cpu().numpy()
    for t in range(T):
        env.random_actions(b, t)
        env.step(b, t)
    env.sync()
    replay_and_compare(n, m, T, L, 0.5, table, prev0, host(b), env.get_returns().cpu().numpy(),
                       quirks=("prev_assigns_zero", "parallel_terminated"), philox=True)


def test_sharding_is_bitwise_equivalent():
    """Envs keyed by global index: one 8-env handle == two 4-env shards."""
    n, m, T, L = 16, 16, 6, 3
    full = AssignEnvBatch(n, m, T, L, 0.5, seed=11, num_envs=8, device=DEV)
    shards = [AssignEnvBatch(n, m, T, L, 0.5, seed=11, num_envs=4, env_index_base=4 * r, device=DEV)
              for r in range(2)]
    bf = new_batch(full, 8)
    bs = [new_batch(s, 4) for s in shards]
    full.reset(bf, 0)
    for s, b in zip(shards, bs):
        s.reset(b, 0)
    for t in range(T):
        full.random_actions(bf, t)
        full.step(bf, t)
        for s, b in zip(shards, bs):
            s.random_actions(b, t)
            s.step(b, t)
    tf = host(bf)
    for r, b in enumerate(bs):
        tr = host(b)
        for k in tf:
            np.testing.assert_array_equal(tf[k][4 * r:4 * r + 4], tr[k], err_msg=k)
    ret = torch.cat([s.get_returns() for s in shards])
    assert torch.equal(full.get_returns(), ret)


@pytest.mark.parametrize("n,m,E", [(16, 16, 4096), (64, 64, 16384)])
def test_full_size_episode_properties(n, m, E):
    """BASELINE configs[1] (16 x 16, 4,096 envs, random policy -- bench.py --config 1 runs
    exactly this schedule: asg_random_actions + asg_step per step) and configs[2]'s env size
    (64 x 64, 16,384 envs), T = 20: size-independent invariants on every env plus a full
    oracle replay of the first, the last and one env inside each grid stride."""
    T, L = 20, 3
    env = AssignEnvBatch(n, m, T, L, 0.5, seed=2024, num_envs=E, device=DEV)
    b = new_batch(env, E)
    env.reset(b, 0)
    prev0 = env.export_prev_assigns()
    for t in range(T):
        env.random_actions(b, t)
        env.step(b, t)
    env.sync()
    obs, beta = b["obs"], b["beta"]
    acts = b["actions"][:, :T, :, 0]
    # one-hot block of obs[t+1] == actions[t]; == actions_onehot[t]
    oh = torch.zeros((E, T, n, m), dtype=torch.int64, device=DEV).scatter_(-1, acts.unsqueeze(-1), 1)
    assert torch.equal(obs[:, 1:, :, :m].to(torch.int64), oh)
    assert torch.equal(b["actions_onehot"][:, :T], oh)
    assert torch.equal(beta[:, :T], obs[:, :T, :, m:2 * m])           # beta == lookahead block 0
    assert torch.equal(obs[:, 1:T, :, 2 * m:3 * m], obs[:, 2:T + 1, :, m:2 * m])  # window shift
    assert (beta[:, T] == 0).all() and (obs[:, T, :, m:] == 0).all()
    assert b["avail_actions"].all() and (b["filled"] == 1).all()
    assert torch.equal(b["terminated"][:, :, 0].sum(1), torch.ones(E, dtype=torch.int64, device=DEV))
    assert torch.equal(b["prev_assigns"][:, 0], prev0) and torch.equal(b["prev_assigns"][:, 1:], acts)
    # prev0 rows are permutation prefixes (choice without replacement)
    srt = prev0.sort(dim=1)[0]
    assert (srt[:, 1:] != srt[:, :-1]).all() and (prev0 >= 0).all() and (prev0 < m).all()
    # returns == float64 sum of the float32 rewards within float32 rounding
    r = env.get_returns()
    assert torch.allclose(b["rewards"][:, :T].double().sum((1, 2)), r, rtol=1e-5, atol=1e-4)
    # full replay of a sample of envs
    idx = np.array(sorted({0, 1, 777, E // 4 + 3, E // 2 - 1, E // 2 + 5, 3 * E // 4 + 7, E - 2, E - 1}))
    table = env.export_benefits()[idx].cpu().numpy()
    td = {k: v[idx].cpu().numpy() for k, v in b.data.transition_data.items()}
    replay_and_compare(n, m, T, L, 0.5, table, prev0[idx].cpu().numpy(), td, r[idx].cpu().numpy(), philox=True)


def test_native_bump_precision_vs_float64():
    """Philox mode evaluates the bumps of obs / beta in float32 (scale 2^(-(t - c)^2 a2), the
    center on an exact grid); against the float64 evaluation of the SAME bump parameters (the
    reference's arithmetic, mock_constellation_env.py:293, on asg_export_bump_params) every
    obs / beta entry is within 1.5 2^-23 of its pair's task scale (the bump's peak in float32
    ulps) plus 10 FLT_MIN (exp results below FLT_MIN flush to 0), and within 1e-6 relative
    wherever the value is >= 2^-12 of its scale; the rewards -- computed on the GPU from the
    float64 values, including the beta > 1e-12 penalty mask (mock :266) -- equal float32 of the
    host's float64 reward to float32 rounding."""
    from oracle.check import bump_table_from_params
    n, m, T, L, E = 64, 64, 20, 3, 512
    env = AssignEnvBatch(n, m, T, L, 0.5, seed=31, num_envs=E, device=DEV)
    b = new_batch(env, E)
    env.reset(b, 0)
    params = env.export_bump_params().cpu().numpy()
    tab = bump_table_from_params(params, T)                          # [E, n, m, T] float64
    np.testing.assert_allclose(env.export_benefits().cpu().numpy(), tab, rtol=4e-16, atol=0)
    scale = params[..., 0].astype(np.float64)                        # [E, n, m] (0: no bump)
    bound = 1.5 * 2.0 ** -23 * scale + 10.0 * float(np.finfo(np.float32).tiny)
    prev = env.export_prev_assigns().cpu().numpy()
    for t in range(T):
        env.random_actions(b, t)
        env.step(b, t)
    env.sync()
    h = host(b)
    worst = worst_abs = 0.0
    for t in range(T + 1):
        for l in range(L):
            want = tab[..., t + l] if t + l < T else np.zeros((E, n, m))
            got = h["obs"][:, t, :, m * (l + 1):m * (l + 2)].astype(np.float64)
            err = np.abs(got - want)
            assert (err <= bound + 2.0 ** -24 * np.abs(want)).all(), f"obs t={t} l={l}: {float((err - bound).max())}"
            # relative bound over the whole range: value = scale 2^-y, y = x^2 a2 rounded
            # twice in float32 (|dy| <= y 2^-23) and one v_exp_f32 + the scale product (<= 2 ulp), so
            # err <= (y ln2 + 2) 2^-23 want; values that flush below FLT_MIN keep the absolute term
            pos = (want > 0) & (scale > 0)
            y = np.log2(np.where(pos, scale, 1.0) / np.where(pos, want, 1.0))
            rel_bound = (y * np.log(2.0) + 2.0) * 2.0 ** -23 * want + 10.0 * float(np.finfo(np.float32).tiny)
            assert (err[pos] <= rel_bound[pos]).all(), \
                f"obs t={t} l={l}: relative {float(np.max((err[pos] - rel_bound[pos]) / want[pos]))}"
            worst_abs = max(worst_abs, float((err / np.maximum(scale, 1.0)).max()))
            big = want >= scale * 2.0 ** -12
            if (big & (scale > 0)).any():
                worst = max(worst, float(np.max(err[big & (scale > 0)] / want[big & (scale > 0)])))
        want_b = tab[..., t] if t < T else np.zeros((E, n, m))
        err = np.abs(h["beta"][:, t].astype(np.float64) - want_b)
        assert (err <= bound + 2.0 ** -24 * np.abs(want_b)).all(), f"beta t={t}"
    # rewards on the host in float64 from the float64 table (mock :126-138)
    acts = h["actions"][:, :T, :, 0]
    ret = np.zeros(E)
    for t in range(T):
        a = acts[:, t]
        beta = np.take_along_axis(tab[..., t], a[..., None], axis=2)[..., 0]        # [E, n]
        pen = (a != prev).astype(np.float64) * (beta > 1e-12)
        bh = beta - 0.5 * pen
        cnt = np.stack([np.bincount(a[e], minlength=m)[a[e]] for e in range(E)])
        r = np.where(bh > 0, bh / cnt, bh)
        np.testing.assert_allclose(h["rewards"][:, t], r.astype(np.float32), rtol=2e-7, atol=0, err_msg=f"t={t}")
        ret += r.sum(1)
        prev = a
    np.testing.assert_allclose(env.get_returns().cpu().numpy(), ret, rtol=1e-12)
    print(f"float32 bump values vs float64: max error {worst_abs:.3g} of the task scale, max relative "
          f"{worst:.3g} where the value is >= 2^-12 of the scale")
    assert worst < 1e-6 and worst_abs <= 1.5 * 2.0 ** -23


def test_full_size_dense_256_episode_properties():
    """BASELINE configs[4] size (256 x 256 dense benefits, 2,048 envs, T=20): invariants on
    every env of a full episode plus an oracle replay of sampled envs (benefits from the
    exported bump parameters in float64).  Reference anchor: mock_constellation_env.py:228-274
    (beta_hat), :116-162 (step)."""
    from oracle.check import bump_table_from_params
    n, m, T, L, E = 256, 256, 20, 3, 2048
    env = AssignEnvBatch(n, m, T, L, 0.5, seed=4096, num_envs=E, device=DEV, benefits="dense")
    b = new_batch(env, E)
    env.reset(b, 0)
    prev0 = env.export_prev_assigns()
    idx = np.array([0, 1, 1000, 2047])
    params = env.export_bump_params()
    assert bool((params[..., 0] > 0).all())  # dense: every (i, j) pair has a bump
    params = params[idx].cpu().numpy()
    for t in range(T):
        env.random_actions(b, t)
        env.step(b, t)
    env.sync()
    obs, beta = b["obs"], b["beta"]
    for t in range(T):  # per row: keeps the int64 one-hot temporaries at ~1 GB
        a = b["actions"][:, t, :, 0]
        oh = torch.zeros((E, n, m), dtype=torch.int64, device=DEV).scatter_(-1, a.unsqueeze(-1), 1)
        assert torch.equal(obs[:, t + 1, :, :m].to(torch.int64), oh), t
        assert torch.equal(b["actions_onehot"][:, t], oh), t
        assert torch.equal(beta[:, t], obs[:, t, :, m:2 * m]), t
        if t + 1 < T:
            assert torch.equal(obs[:, t + 1, :, 2 * m:3 * m], obs[:, t + 2, :, m:2 * m]), t
        assert torch.equal(b["prev_assigns"][:, t + 1], a), t
        del oh
    assert (beta[:, T] == 0).all() and (obs[:, T, :, m:] == 0).all()
    assert b["avail_actions"].all() and (b["filled"] == 1).all()
    assert torch.equal(b["terminated"][:, :, 0].sum(1), torch.ones(E, dtype=torch.int64, device=DEV))
    assert torch.equal(b["prev_assigns"][:, 0], prev0)
    srt = prev0.sort(dim=1)[0]
    assert (srt[:, 1:] != srt[:, :-1]).all()
    r = env.get_returns()
    assert torch.allclose(b["rewards"][:, :T].double().sum((1, 2)), r, rtol=1e-5, atol=1e-3)
    table = bump_table_from_params(params, T)
    td = {k: v[idx].cpu().numpy() for k, v in b.data.transition_data.items()}
    replay_and_compare(n, m, T, L, 0.5, table, prev0[idx].cpu().numpy(), td, r[idx].cpu().numpy(),
                       philox=True, rtol_reward=2e-7)


def test_action_range_error():
    env = AssignEnvBatch(4, 4, 3, 1, 0.5, num_envs=2, device=DEV)
    b = new_batch(env, 2)
    env.reset(b, 0)
    b["actions"][1, 0, 2] = 4
    env.step(b, 0)
    with pytest.raises(ValueError, match="outside"):
        env.sync()
    env.sync()  # sticky error cleared once reported


def test_create_errors():
    with pytest.raises(ValueError, match="larger sample"):
        AssignEnvBatch(8, 4, 3, 1, 0.5, device=DEV)
    env = AssignEnvBatch(4, 4, 3, 1, 0.5, device=DEV)
    b = new_batch(env, 1)
    with pytest.raises(RuntimeError, match="before reset"):
        env.step(b, 0)


# ------------------------------------------------------------------------------ single-env plugin
def test_single_env_plugin_matches_golden(golden):
    g = golden("mock_reset")
    c = 5  # 16x16, seed 0
    n, m, T, L, s = [int(x) for x in g[f"c{c}_shape"]]
    env = MockConstellationEnv(n, m, T, L, 0.5, stream_seed=s)
    env.reset()
    np.testing.assert_array_equal(np.array(env._obs, dtype=np.float32), g[f"c{c}_obs"].astype(np.float32))
    np.testing.assert_array_equal(env.prev_assigns, g[f"c{c}_prev_assigns"])
    oe = ora.OracleMockEnv(n, m, T, L, 0.5, mt=ora.MT(s))
    oe.reset()
    rng = np.random.RandomState(0)
    for t in range(T):
        a = rng.randint(0, m, size=n)
        r, d, _ = env.step(a)
        r0, d0, _ = oe.step(a)
        np.testing.assert_array_equal(np.float32(r), np.float32(r0))
        assert d == d0
        pre = env.get_pretransition_data()
        np.testing.assert_array_equal(np.array(pre["obs"][0], np.float32), oe._obs.astype(np.float32))


# ------------------------------------------------------------------------------ fused epsilon-greedy
def _eg(eps, seed=0):
    from types import SimpleNamespace

    from marl_sap_amd.action_selectors.classic_selectors import EpsilonGreedyActionSelector
    return EpsilonGreedyActionSelector(SimpleNamespace(epsilon_start=eps, epsilon_finish=eps, epsilon_anneal_time=1,
                                                       evaluation_epsilon=0.0, seed=seed))


@pytest.mark.parametrize("B,n,m", [(512, 64, 64), (64, 7, 10), (32, 5, 100), (16, 9, 200), (1, 1, 1)])
def test_epsilon_greedy_greedy_matches_torch(B, n, m):
    g = torch.Generator(device=DEV).manual_seed(B + n + m)
    q = torch.randn((B, n, m), device=DEV, generator=g)
    avail = torch.rand((B, n, m), device=DEV, generator=g) > 0.3
    avail[..., 0] |= ~avail.any(-1)  # every row has an available action
    q[0, 0, :] = 1.0                  # ties: first maximal available index
    sel = _eg(0.0)
    a = sel.select_action(q, avail, 0)
    ref = q.masked_fill(~avail, -float("inf")).max(dim=2)[1]
    assert torch.equal(a, ref)
    if m > 1:
        q[1, 0, m // 2] = float("nan")  # an available NaN propagates like torch.max
        avail[1, 0, m // 2] = True
        a = sel.select_action(q, avail, 0)
        assert a[1, 0].item() == m // 2
    sel.flush()


def test_epsilon_greedy_exploration_distribution():
    B, n, m = 4096, 16, 10
    q = torch.randn((B, n, m), device=DEV)
    avail = torch.ones((B, n, m), dtype=torch.bool, device=DEV)
    avail[:, :, 7:] = False
    sel = _eg(1.0)
    a = sel.select_action(q, avail, 0)
    counts = torch.bincount(a.flatten(), minlength=m).cpu().numpy()
    assert counts[7:].sum() == 0
    expect = B * n / 7
    assert np.all(np.abs(counts[:7] - expect) < 5 * np.sqrt(expect))
    greedy = q.masked_fill(~avail, -float("inf")).max(2)[1]
    sel = _eg(0.3)
    frac = (sel.select_action(q, avail, 0) != greedy).float().mean().item()
    assert abs(frac - 0.3 * 6 / 7) < 0.01
    sel.flush()


def test_epsilon_greedy_writes_batch_row_in_place():
    E, n, m, T = 8, 6, 8, 4
    env = AssignEnvBatch(n, m, T, 2, 0.5, num_envs=E, device=DEV)
    b = new_batch(env, E)
    env.reset(b, 0)
    q = torch.randn((E, n, m), device=DEV)
    row = b["actions"][:, 1, :, 0]
    out = _eg(0.0).select_action(q, b["avail_actions"][:, 0], 0, out=row)
    assert out is row
    assert torch.equal(b["actions"][:, 1, :, 0], q.max(2)[1])
    assert (b["actions"][:, 0] == 0).all() and (b["actions"][:, 2:] == 0).all()


def test_philox_bump_parameter_distribution():
    """The Philox bump draws (one Philox call per four pairs, asg_device.h:philox_bump32x4)
    follow generate_benefits_over_time's distribution (mock_constellation_env.py:281-293):
    active with probability 1/4, center ~ U(0, T), width ~ U(wmin, wmax) -- and pairs of one
    call are independent."""
    n = m = 64
    T, E = 20, 64
    env = AssignEnvBatch(n, m, T, 3, 0.5, seed=11, num_envs=E, device=DEV)
    b = new_batch(env, E)
    env.reset(b, 0)
    p = env.export_bump_params().cpu().numpy().reshape(E, n * m, 3)
    scale, center, a = p[..., 0], p[..., 1], p[..., 2]
    act = scale > 0
    assert abs(act.mean() - 0.25) < 0.005
    assert set(np.unique(scale[act])) <= {1.0, 10.0}
    even, odd = act[:, 0::2], act[:, 1::2]
    assert abs((even & odd).mean() - 0.0625) < 0.004
    assert abs(np.corrcoef(even.ravel(), odd.ravel())[0, 1]) < 0.01
    assert center.min() >= 0.0 and center.max() < T and abs(center.mean() - T / 2) < 0.05
    spread = float.fromhex("0x1.c4035ap+1") / a.astype(np.float64)  # a = log2(e) sqrt(-2 ln 0.05) / spread
    lo, hi = spread.min(), spread.max()
    assert 2.99 < lo and hi < 8.01 and hi - lo > 2.9
    u = (spread - lo) / (hi - lo)
    assert abs(u.mean() - 0.5) < 0.01
    assert abs(np.corrcoef(u[:, 0::2].ravel(), u[:, 1::2].ravel())[0, 1]) < 0.01
    env.close()
