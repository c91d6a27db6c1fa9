"""Filtered selectors (filtered_sap_selectors.py:7-148, filtered_classic_selectors.py:6-103),
HAALSelector (non_rl_selectors.py:54-118) and ContinuousActionSelector (bet_selectors.py)
on the GPU, through the C-ABI:
  * against the reference's own outputs (tests/golden/filtered_selectors.npz, haal.npz) with
    the reference's recorded random draws fed in -- bit for bit;
  * against the oracle (oracle/selectors.py) on tie-heavy inputs (the lower-index tie rule);
  * a filtered_reda-shaped rollout (FlatConstAgent + the filtered selectors) through
    GpuVecRunner on the batched RealConstellationEnv, every step checked."""
from types import SimpleNamespace

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():
    pytest.skip("needs a ROCm GPU", allow_module_level=True)

from marl_sap_amd.action_selectors import REGISTRY as SEL  # noqa: E402
from marl_sap_amd.action_selectors.filtered_selectors import filtered_benefit_matrix, filtered_top_m  # noqa: E402
from marl_sap_amd.action_selectors.non_rl_selectors import REGISTRY as NONRL  # noqa: E402
from marl_sap_amd.components import EpisodeBatch  # noqa: E402
from marl_sap_amd.envs import RealAssignEnvBatch  # noqa: E402

DEV = torch.device("cuda", 0)
KIND = {"sap": "filtered_const_sap", "egsap": "filtered_const_epsgr_sap_test", "eg": "filtered_const_epsilon_greedy"}


def _args(eps, M, **kw):
    a = dict(epsilon_start=eps, epsilon_finish=eps, epsilon_anneal_time=1000, evaluation_epsilon=0.0,
             env_args={"M": M}, seed=3)
    a.update(kw)
    return SimpleNamespace(**a)


def test_filtered_selectors_match_reference(golden):
    g = golden("filtered_selectors")
    for c in g["cases"]:
        B, n, m, M, L, test_mode = [int(x) for x in g[f"{c}__cfg"]]
        kind = str(g[f"{c}__kind"])
        sel = SEL[KIND[kind]](_args(float(g[f"{c}__epsilon"]), M))
        q = torch.from_numpy(g[f"{c}__q"]).to(DEV)
        beta = torch.from_numpy(g[f"{c}__beta"]).to(DEV)
        avail = torch.ones((B, n, m), dtype=torch.bool, device=DEV)
        kw = {"tie_noise": torch.from_numpy(g[f"{c}__tie_noise"]).to(DEV).contiguous()}
        if kind == "sap" and f"{c}__gauss_noise" in g:
            kw["gauss_noise"] = torch.from_numpy(g[f"{c}__gauss_noise"]).to(DEV).contiguous()
        out = sel.select_action(q, avail, 0, test_mode=bool(test_mode), beta=beta, **kw)
        want = g[f"{c}__actions"]
        assert str(out.dtype) == str(g[f"{c}__actions_dtype"]), c
        np.testing.assert_array_equal(out.cpu().numpy(), want, err_msg=str(c))


@pytest.mark.parametrize("dtype", [torch.float16, torch.float32, torch.float64])
@pytest.mark.parametrize("B,n,m,L,M", [(3, 5, 24, 3, 4), (2, 7, 130, 2, 10), (1, 4, 450, 3, 10), (2, 3, 1000, 3, 64)])
def test_top_m_tie_rule_vs_oracle(dtype, B, n, m, L, M):
    """Tie-heavy totals (a coarse grid and all-zero tasks): the lower task index first."""
    from oracle.selectors import top_m
    rng = np.random.RandomState(m + M)
    beta = np.round(rng.uniform(0, 2, size=(B, n, m, L)) * 2) / 2
    beta[rng.uniform(size=(B, n, m)) < 0.5] = 0
    bt = torch.from_numpy(beta).to(dtype)
    got = filtered_top_m(bt.to(DEV), M).cpu().numpy()
    np.testing.assert_array_equal(got, top_m(bt.numpy(), M))


def test_top_m_strided_beta_view():
    """A batch-major EpisodeBatch's beta[:, t] (a strided view) is read in place."""
    from oracle.selectors import top_m
    rng = np.random.RandomState(1)
    full = torch.from_numpy(rng.uniform(size=(3, 4, 6, 20, 3))).to(torch.float16)  # [B, T+1, n, m, L]
    view = full.to(DEV)[:, 2]                                                          # [B, n, m, L]
    assert not view.is_contiguous()
    np.testing.assert_array_equal(filtered_top_m(view, 5).cpu().numpy(), top_m(view.cpu().numpy(), 5))


def test_benefit_matrix_philox_noise_properties():
    from oracle.selectors import top_m
    rng = np.random.RandomState(2)
    B, n, m, M, L = 4, 16, 200, 8, 3
    q = torch.from_numpy(rng.standard_normal((B, n, M + 1)).astype(np.float32) * 1e-3).to(DEV)
    beta = torch.from_numpy(rng.uniform(size=(B, n, m, L))).to(torch.float16).to(DEV)
    top = filtered_top_m(beta, M)
    mat = filtered_benefit_matrix(q, top, m, seed=11, counter=1).cpu().numpy()
    qn, tn = q.cpu().numpy(), top.cpu().numpy()
    np.testing.assert_array_equal(tn, top_m(beta.cpu().numpy(), M))
    bi, ii = np.indices((B, n))
    np.testing.assert_array_equal(mat[bi[..., None], ii[..., None], tn], qn[:, :, :M])
    mask = np.ones((B, n, m), bool)
    mask[bi[..., None], ii[..., None], tn] = False
    d = (mat - qn[:, :, M:M + 1])[mask]
    # u * 1e-8 plus the rounding of base + noise (half an ulp of |base| ~ 1e-3)
    assert d.min() >= 0 and d.max() <= 1.0e-8 + 2.5e-10 and np.unique(d).size > 100
    # the same key draws the same noise; another counter draws different noise
    again = filtered_benefit_matrix(q, top, m, seed=11, counter=1).cpu().numpy()
    other = filtered_benefit_matrix(q, top, m, seed=11, counter=2).cpu().numpy()
    assert np.array_equal(mat, again) and not np.array_equal(mat, other)
    # shard invariance: envs [2, 4) drawn by a rank with env_base 2 equal the 1-rank draw
    half = filtered_benefit_matrix(q[2:], top[2:], m, seed=11, counter=1, env_base=2).cpu().numpy()
    np.testing.assert_array_equal(half, mat[2:])


def test_filtered_sap_philox_noise_is_lsa_of_its_matrix(oracle):
    rng = np.random.RandomState(4)
    B, n, m, M, L = 3, 20, 40, 6, 3
    sel = SEL["filtered_const_sap"](_args(0.4, M))
    q = torch.from_numpy(rng.standard_normal((B, n, M + 1)).astype(np.float32)).to(DEV)
    beta = torch.from_numpy(rng.uniform(size=(B, n, m, L))).to(torch.float16).to(DEV)
    out = sel.select_action(q, torch.ones((B, n, m), dtype=torch.bool, device=DEV), 0, beta=beta)
    mat = sel.last_matrix.cpu().numpy().astype(np.float64)
    for b in range(B):
        np.testing.assert_array_equal(out[b].cpu().numpy(), oracle.lsa(mat[b], maximize=True)[1])
    # the exploration noise has the reference's scale: std 2 eps mean|mat| (here >> 1e-8)
    top = filtered_top_m(beta, M)
    clean = filtered_benefit_matrix(q, top, m, seed=sel.seed, counter=sel.calls).cpu().numpy()
    noise = sel.last_matrix.cpu().numpy() - clean
    want = 2 * 0.4 * np.abs(clean).mean(axis=(1, 2))
    np.testing.assert_allclose(noise.std(axis=(1, 2)), want, rtol=0.05)


def test_filtered_epsilon_greedy_exploration_and_soft_map():
    rng = np.random.RandomState(5)
    B, n, m, M, L = 64, 32, 50, 5, 2
    beta = torch.from_numpy(rng.uniform(size=(B, n, m, L))).to(torch.float16).to(DEV)
    avail = torch.from_numpy(rng.uniform(size=(B, n, m)) < 0.5).to(DEV)
    avail[..., 0] = True
    q = torch.from_numpy(rng.standard_normal((B, n, M + 1)).astype(np.float32)).to(DEV)
    sel = SEL["filtered_const_epsilon_greedy"](_args(1.0, M))
    a = sel.select_action(q, avail, 0, beta=beta)
    assert a.dtype == torch.int64
    assert bool(torch.gather(avail, 2, a.unsqueeze(-1)).all())  # exploring rows pick available tasks
    # eps = 0: the unmasked argmax of the matrix (availability ignored, as the reference)
    sel0 = SEL["filtered_const_epsilon_greedy"](_args(0.0, M))
    a0 = sel0.select_action(q, avail, 0, beta=beta)
    np.testing.assert_array_equal(a0.cpu().numpy(), sel0.last_matrix.argmax(-1).cpu().numpy())
    # soft policies: a one-hot policy on index p < M picks the p-th top task; p = M a task
    # outside the top M, uniformly
    soft = SEL["filtered_const_soft_policies"](_args(0.0, M))
    top = filtered_top_m(beta, M).cpu().numpy()
    p = rng.randint(0, M + 1, size=(B, n))
    pol = torch.nn.functional.one_hot(torch.from_numpy(p), M + 1).float().to(DEV)
    got = soft.select_action(pol, avail, 0, beta=beta).cpu().numpy()
    lo = p < M
    bi, ii = np.indices((B, n))
    np.testing.assert_array_equal(got[lo], top[bi[lo], ii[lo], p[lo]])
    hi = ~lo
    assert not np.any(got[hi][:, None] == top[hi])
    pol_m = torch.nn.functional.one_hot(torch.full((B, n), M), M + 1).float().to(DEV)
    draws = np.concatenate([soft.select_action(pol_m, avail, 0, beta=beta).cpu().numpy().ravel() for _ in range(20)])
    assert set(np.unique(draws)) <= set(range(m)) and np.unique(draws).size > (m - M) * 0.9


def test_continuous_selector():
    sel = SEL["continuous"](_args(0.5, 4))
    x = torch.randn((8, 4, 6), device=DEV)
    assert torch.equal(sel.select_action(x, None, 0, test_mode=True), x)  # evaluation_epsilon 0
    y = sel.select_action(x, None, 0)
    assert y.device == x.device and 0.4 < float((y - x).std()) < 0.6
    lp = sel.action_log_prob(y, x)
    assert lp.shape == x.shape


# ---------------------------------------------------------------------------------------
def _step_real(env, batch, t, actions):
    batch["actions"][:, t, :, 0] = torch.as_tensor(np.asarray(actions), dtype=torch.int16, device=DEV)
    env.step(batch, t)


def test_haal_matches_reference(golden):
    g = golden("haal")
    for c in range(int(g["n_cases"])):
        B, n, m, T, L, N, M, pre, k = [int(x) for x in g[f"h{c}_spec"]]
        env = RealAssignEnvBatch(1, n, m, T, N, M, L, float(g[f"h{c}_lambda"]), sat_prox_mat=g[f"h{c}_tables"],
                                 T_trans=g[f"h{c}_T_trans"], task_prios=g[f"h{c}_prios"], num_envs=B, device=DEV)
        batch = EpisodeBatch(env.scheme, {"agents": n}, B, T + 1, preprocess=env.preprocess, device=DEV,
                             time_major=True)
        env.reset(batch, 0)
        for t in range(pre):  # reach the fixture's state: step k with prev_assigns = prev
            _step_real(env, batch, t, g[f"h{c}_prev"])
        sel = NONRL["haal_selector"](SimpleNamespace())
        sel.envs = env
        out = sel.select_action(batch)
        sel.status.flush()
        np.testing.assert_array_equal(out.cpu().numpy(), g[f"h{c}_actions"])
        np.testing.assert_array_equal(sel.last_values.cpu().numpy(), g[f"h{c}_values"])
        best = np.array([int(np.argmax(v)) for v in g[f"h{c}_values"]])  # first maximum
        np.testing.assert_array_equal(sel.last_best.cpu().numpy(), best)
        env.close()


def _variant_env(kind, tables, N, M, L, lam, prios, E, bands, nbr, prev0=None, seed=0):
    from marl_sap_amd.envs import InterferenceAssignEnvBatch, RealPowerAssignEnvBatch
    n, m, T = tables.shape[-3:]
    if kind == "power":
        return RealPowerAssignEnvBatch(1, n, m, T, N, M, L, lam, sat_prox_mat=tables, graphs=[None] * T,
                                       task_prios=prios, num_envs=E, initial_assignments=prev0, seed=seed, device=DEV)
    return InterferenceAssignEnvBatch(1, n, None, T, N, M, L, lam, task_prios=prios, sat_freq_bands=bands,
                                      sat_prox_mat=tables, neighbor_matrix=nbr, num_envs=E, initial_assignments=prev0,
                                      seed=seed, device=DEV)


def test_haal_variants_match_reference(golden):
    """HAAL over the power / interference envs: the forks carry the power
    states (drained by their own steps, dead / below-1e-12 rows zeroed in beta_hat) -- actions,
    every sequence's value and the winning sequence bit-exact against the reference's selector
    (tests/golden/haal_variants.npz), after the fixture's own pre-selection steps."""
    g = golden("haal_variants")
    for c in range(int(g["n_cases"])):
        kind = str(g[f"h{c}_kind"])
        B, n, m, T, L, N, M, pre, k = [int(x) for x in g[f"h{c}_spec"]]
        env = _variant_env(kind, g[f"h{c}_tables"], N, M, L, float(g[f"h{c}_lambda"]), g[f"h{c}_prios"], B,
                           g[f"h{c}_bands"], g[f"h{c}_nbr"], prev0=g[f"h{c}_prev0"])
        batch = EpisodeBatch(env.scheme, {"agents": n}, B, T + 1, preprocess=env.preprocess, device=DEV,
                             time_major=True)
        env.reset(batch, 0)
        for t in range(pre):
            _step_real(env, batch, t, g[f"h{c}_pre_actions"][:, t])
        np.testing.assert_array_equal(batch["prev_assigns"][:, pre].cpu().numpy(), g[f"h{c}_prev"])
        assert torch.equal(batch["power_states"][:, pre].cpu(), torch.from_numpy(g[f"h{c}_power"]).to(torch.float16))
        sel = NONRL["haal_selector"](SimpleNamespace())
        sel.envs = env
        out = sel.select_action(batch)
        sel.status.flush()
        np.testing.assert_array_equal(out.cpu().numpy(), g[f"h{c}_actions"], err_msg=f"{kind} case {c}")
        np.testing.assert_array_equal(sel.last_values.cpu().numpy(), g[f"h{c}_values"], err_msg=f"{kind} case {c}")
        best = np.array([int(np.argmax(v)) for v in g[f"h{c}_values"]])
        np.testing.assert_array_equal(sel.last_best.cpu().numpy(), best)
        env.close()


@pytest.mark.parametrize("kind,n,m,T,L", [("power", 12, 20, 10, 4), ("power", 30, 45, 8, 3),
                                          ("interference", 14, 24, 9, 3)])
def test_haal_variants_vs_oracle_through_an_episode(oracle, kind, n, m, T, L):
    """HAAL on the power variants at every step of an episode driven by HAAL itself (satellites
    drain and die along the way), against the oracle restatement (pinned by the fixture above)."""
    from oracle.selectors import haal_variant
    E = 4
    rng = np.random.RandomState(n + m + T + len(kind))
    tables = rng.uniform(0.0, 1.0, size=(E, n, m, T))
    tables[rng.uniform(size=tables.shape) < 0.4] = 0.0
    prios = rng.choice([1.0, 1.0, 1.0, 5.0], size=m)
    bands = rng.randint(0, 3, size=n)
    nbr = (rng.uniform(size=(m, m)) > 0.75).astype(np.float64)
    nbr = np.maximum(nbr, nbr.T)
    np.fill_diagonal(nbr, 1.0)
    env = _variant_env(kind, tables, 2, 2, L, 0.4, prios, E, bands, nbr, seed=3)
    batch = EpisodeBatch(env.scheme, {"agents": n}, E, T + 1, preprocess=env.preprocess, device=DEV,
                         time_major=True)
    env.reset(batch, 0)
    prev = batch["prev_assigns"][:, 0].cpu().numpy().astype(np.int64)
    power = np.ones((E, n))
    tt = np.ones((m, m)) - np.eye(m)
    from oracle.selectors import power_update, real_beta
    dead_seen = 0
    for t in range(T):
        out, values, best, status = env.haal_select(return_values=True)
        assert int(status.abs().max()) == 0
        acts = out.cpu().numpy().astype(np.int64)
        for e in range(E):
            a, vals = haal_variant(kind, tables[e], prios, tt, 0.4, t, prev[e], power[e], env.L, T, bands=bands,
                                   nbr=nbr)
            np.testing.assert_array_equal(acts[e], a, err_msg=f"t={t} env {e}")
            np.testing.assert_array_equal(values[e].cpu().numpy(), vals, err_msg=f"t={t} env {e}")
            power[e] = power_update(real_beta(tables[e], prios, t, env.L, T), acts[e], power[e])
        _step_real(env, batch, t, acts)
        prev = acts
        dead_seen += int((power < 1e-12).sum())
    assert dead_seen > 0  # the episode exercised dead / drained satellites
    env.close()


@pytest.mark.parametrize("n,m,T,L", [(12, 20, 8, 4), (30, 45, 6, 3), (5, 8, 9, 5)])
def test_haal_vs_oracle_through_an_episode(oracle, n, m, T, L):
    """Sparse per-env tables (many zero benefits -> masked penalties, exact ties in the LSA),
    HAAL at every step of an episode driven by HAAL itself, against the oracle."""
    from oracle.selectors import haal
    E = 4
    rng = np.random.RandomState(n + m + T)
    tables = rng.uniform(0.0, 1.0, size=(E, n, m, T))
    tables[rng.uniform(size=tables.shape) < 0.5] = 0.0
    tables[:, :, : m // 4] = np.round(tables[:, :, : m // 4] * 2) / 2
    prios = rng.uniform(0.5, 2.0, size=m)
    tt = (rng.uniform(size=(m, m)) > 0.3).astype(np.float64)
    env = RealAssignEnvBatch(1, n, m, T, 2, 2, L, 0.4, sat_prox_mat=tables, task_prios=prios, T_trans=tt,
                             num_envs=E, device=DEV)
    batch = EpisodeBatch(env.scheme, {"agents": n}, E, T + 1, preprocess=env.preprocess, device=DEV,
                         time_major=True)
    env.reset(batch, 0)
    prev = np.tile(np.arange(n), (E, 1))
    for t in range(T):
        out, values, best, status = env.haal_select(return_values=True)
        assert int(status.abs().max()) == 0
        acts = out.cpu().numpy().astype(np.int64)
        for e in range(E):
            a, vals = haal(tables[e], prios, tt, 0.4, t, prev[e], env.L, T)
            np.testing.assert_array_equal(acts[e], a)
            np.testing.assert_array_equal(values[e].cpu().numpy(), vals)
        _step_real(env, batch, t, acts)
        prev = acts
    with pytest.raises(ValueError):
        env.haal_select()
    env.close()


def test_haal_nan_benefits_report_status_without_fault():
    """A NaN benefit makes the root LSA of that env fail (scipy: "matrix contains invalid
    numeric entries"); its -1 assignment rows must not be used as indices by the tree's
    child matrices or the sequence values (they are poisoned with NaN instead).  The failing
    env reports its status, the selector raises scipy's ValueError on flush, and the other
    envs' actions equal a NaN-free run."""
    E, n, m, T, L = 3, 6, 9, 5, 4
    rng = np.random.RandomState(5)
    tables = rng.uniform(0.0, 1.0, size=(E, n, m, T))
    bad = tables.copy()
    bad[1, 2, 4, 1] = np.nan    # seen by the root node's L-summed benefit
    bad[2, 0, :, 4] = -np.inf   # outside the root's window (times 0-3): a child node's LSA fails
    #                             (agent 0 has no finite task: infeasible) and its -1 rows feed
    #                             the grandchildren's matrices and the sequence values

    def run(tab):
        env = RealAssignEnvBatch(1, n, m, T, 2, 2, L, 0.4, sat_prox_mat=tab, num_envs=E, device=DEV)
        b = EpisodeBatch(env.scheme, {"agents": n}, E, T + 1, preprocess=env.preprocess, device=DEV,
                         time_major=True)
        env.reset(b, 0)
        out, values, best, status = env.haal_select(return_values=True)
        env.sync()
        res = out.cpu(), status.cpu(), values.cpu()
        env.close()
        return res

    out_ok, st_ok, _ = run(tables)
    out_bad, st_bad, val_bad = run(bad)
    assert int(st_ok.abs().max()) == 0
    assert int(st_bad[0]) == 0 and int(st_bad[1]) != 0 and int(st_bad[2]) != 0
    assert torch.equal(out_bad[0], out_ok[0])
    assert bool((out_bad[1] == -1).all())
    from marl_sap_amd.action_selectors.lsa import DeferredStatus
    ds = DeferredStatus()
    ds.add(st_bad[:2].to(DEV))
    with pytest.raises(ValueError, match="invalid numeric entries"):
        ds.flush()
    assert int(st_bad[2]) == -5  # ASG_E_LSA_INFEASIBLE


# ---------------------------------------------------------------------------------------
@pytest.mark.parametrize("selector,agent", [("filtered_const_epsgr_sap_test", "flat_const_agent_fused"),
                                            ("filtered_const_sap", "flat_const_agent"),
                                            ("filtered_const_epsilon_greedy", "flat_const_agent_fused")])
def test_filtered_reda_rollout_on_real_env(oracle, selector, agent):
    """filtered_reda-shaped rollout: BasicMAC + FlatConstAgent (M + 1 outputs) + a filtered
    selector over the batched RealConstellationEnv through GpuVecRunner.  Every step's
    actions are the selector's rule applied to its own matrix, whose top-M columns hold the
    agent's Q-values on the oracle's top-M tasks."""
    from marl_sap_amd.controllers import REGISTRY as MAC
    from marl_sap_amd.runners import REGISTRY as RUN
    from oracle.selectors import top_m
    n, m, T, N, M, L, E = 16, 40, 5, 3, 6, 3, 6
    rng = np.random.RandomState(7)
    table = rng.uniform(0.01, 1.0, size=(n, m, T))
    args = SimpleNamespace(batch_size_run=E, env="real_constellation_env", test_nepisode=E, runner_log_interval=10**9,
                           env_args=dict(num_planes=1, num_sats_per_plane=n, m=m, T=T, N=N, M=M, L=L, lambda_=0.5,
                                         sat_prox_mat=table, graphs=[None] * T, seed=5),
                           agent=agent, hidden_dim=64, use_rnn=True, obs_last_action=False, obs_agent_id=False,
                           agent_output_type="q", action_selector=selector, epsilon_start=0.3, epsilon_finish=0.3,
                           epsilon_anneal_time=1000, evaluation_epsilon=0.0, mac="basic_mac", seed=5,
                           runner="gpu", use_cuda=True, device="cuda")
    runner = RUN["gpu"](args, logger=None)
    env = runner.get_env()
    args.n, args.m, args.T = env.n, env.m, env.T
    mac = MAC["basic_mac"](env.scheme, {"agents": n}, args)
    mac.cuda()
    runner.setup(scheme=env.scheme, groups={"agents": n}, preprocess=env.preprocess, mac=mac)
    sel = mac.action_selector
    rec = []
    orig = sel.select_action

    def wrapped(q, avail, t_env, test_mode=False, beta=None, **kw):
        out = orig(q, avail, t_env, test_mode=test_mode, beta=beta, **kw)
        rec.append((q.detach().cpu().numpy(), beta.cpu().numpy(), sel.last_matrix.cpu().numpy(), out.cpu().numpy()))
        return out

    sel.select_action = wrapped
    test_mode = selector == "filtered_const_epsgr_sap_test"
    batch = runner.run(test_mode=test_mode)
    assert len(rec) == T
    for t, (q, beta, mat, out) in enumerate(rec):
        top = top_m(beta, M)
        bi, ii = np.indices((E, n))
        if selector != "filtered_const_sap":  # (SAP's matrix carries its Gaussian exploration noise)
            np.testing.assert_array_equal(mat[bi[..., None], ii[..., None], top], q[:, :, :M])
        if selector == "filtered_const_epsilon_greedy":
            assert out.dtype == np.int64  # eps 0.3: exploring rows anywhere, the rest the argmax
            greedy = mat.argmax(-1)
            assert 0.4 < np.mean(out == greedy) < 0.95
        else:
            for b in range(E):
                np.testing.assert_array_equal(out[b], oracle.lsa(mat[b].astype(np.float64), maximize=True)[1])
        np.testing.assert_array_equal(batch["actions"][:, t, :, 0].cpu().numpy(), out.astype(np.int64))
    env.close()
