"""Batched RealConstellationEnv on the GPU against
  * the reference's own reset/step outputs (tests/golden/real_env.npz, tie-free tables),
  * the C oracle (oracle/asg_real_oracle.c) on tie-heavy sparse tables, per env,
through the reference's float16 / int16 scheme (values cast float64 -> float32 -> float16
exactly as torch casts them in EpisodeBatch.update)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():
    pytest.skip("needs a ROCm GPU", allow_module_level=True)

from marl_sap_amd.components import EpisodeBatch  # noqa: E402
from marl_sap_amd.envs import RealAssignEnvBatch  # noqa: E402

DEV = torch.device("cuda", 0)


def f16(x):
    return torch.from_numpy(np.asarray(x, dtype=np.float64)).to(torch.float16)


def new_batch(env, E):
    return EpisodeBatch(env.scheme, {"agents": env.n}, E, env.T + 1, preprocess=env.preprocess, device=DEV,
                        time_major=True)


def check_row(b, e, t, obs, beta, prev):
    assert torch.equal(b["obs"][e, t].cpu(), f16(obs))
    assert torch.equal(b["beta"][e, t].cpu(), f16(beta))
    assert torch.equal(b["prev_assigns"][e, t].cpu(), torch.from_numpy(np.asarray(prev)).to(torch.int16))
    assert bool(b["avail_actions"][e, t].all()) and int(b["filled"][e, t, 0]) == 1


def test_real_env_matches_reference_fixture(golden):
    d = golden("real_env")
    for c in range(int(d["n_cases"])):
        n, m, T, L, N, M = (int(x) for x in d[f"r{c}_spec"])
        env = RealAssignEnvBatch(1, n, m, T, N, M, L, float(d[f"r{c}_lambda"]), sat_prox_mat=d[f"r{c}_table"],
                                 graphs=[None] * T, T_trans=d[f"r{c}_T_trans"], task_prios=d[f"r{c}_prios"],
                                 num_envs=2, device=DEV)
        assert env.obs_space_size == int(d[f"r{c}_obs_size"])
        b = new_batch(env, 2)
        env.reset(b, 0)
        for e in range(2):
            check_row(b, e, 0, d[f"r{c}_obs0"], d[f"r{c}_beta0"], d[f"r{c}_prev0"])
        ret = np.zeros(2)
        for t in range(T):
            a = torch.from_numpy(d[f"r{c}_actions"][t]).to(torch.int16)
            b["actions"][:, t, :, 0] = a.to(DEV)  # both envs take the reference's actions
            done = env.step(b, t)
            assert done == bool(d[f"r{c}_done"][t])
            for e in range(2):
                assert torch.equal(b["rewards"][e, t].cpu(), f16(d[f"r{c}_rewards"][t]))
                check_row(b, e, t + 1, d[f"r{c}_obs"][t], d[f"r{c}_beta"][t], d[f"r{c}_prev"][t])
                onehot = torch.zeros((n, m), dtype=torch.int16)
                onehot[torch.arange(n), a.long()] = 1
                assert torch.equal(b["actions_onehot"][e, t].cpu(), onehot)
                assert bool(b["terminated"][e, t, 0]) == (t + 1 >= T)
            ret += sum(d[f"r{c}_rewards"][t])
        env.sync()
        assert np.array_equal(env.get_returns().cpu().numpy(), ret)


@pytest.mark.parametrize("n,m,T,L,N,M,sparse", [(16, 24, 6, 3, 4, 6, True), (20, 20, 5, 2, 19, 4, False),
                                                (33, 70, 4, 3, 5, 10, True), (8, 9, 3, 5, 2, 2, True),
                                                (20, 30, 4, 3, 6, 6, "near"), (33, 70, 5, 3, 5, 10, "near"),
                                                (15, 27, 5, 3, 4, 6, True)])
def test_real_env_matches_oracle_per_env_tables(oracle, n, m, T, L, N, M, sparse):
    """Per-env tables, random actions; sparse tables make many equal totals, so this
    checks the stable tie rule the GPU and the oracle share.  "near": quarter-step values
    plus offsets of a few 2**-36 -- the competitors' best totals tie as float32 keys but not
    as float64, so the observation pass must take its exact float64 re-ranking.  Odd m with
    L = 3: agent rows of beta start at both 4-byte alignments (the strip's dword + short
    stores)."""
    E = 5
    rng = np.random.RandomState(n * 100 + m)
    tables = rng.uniform(0.0, 1.0, size=(E, n, m, T))
    if sparse == "near":
        tables = np.round(tables * 4) / 4 + rng.randint(0, 4, size=tables.shape) * 2.0 ** -36
    elif sparse:
        tables *= rng.uniform(size=(E, n, m, 1)) > 0.7
        tables[:, :, : m // 3] = np.round(tables[:, :, : m // 3] * 4) / 4  # exact ties among non-zeros
    prios = rng.uniform(0.5, 2.0, size=m)
    env = RealAssignEnvBatch(1, n, m, T, N, M, L, 0.5, sat_prox_mat=tables, task_prios=prios, num_envs=E,
                             device=DEV)
    refs = [oracle.OracleRealEnv(tables[e], N, M, L, 0.5, task_prios=prios) for e in range(E)]
    b = new_batch(env, E)
    env.reset(b, 0)
    for e, r in enumerate(refs):
        r.reset()
        check_row(b, e, 0, r.obs, r.beta, r.prev_assigns)
    for t in range(T):
        acts = rng.randint(0, m, size=(E, n))
        b["actions"][:, t, :, 0] = torch.from_numpy(acts).to(torch.int16).to(DEV)
        env.step(b, t)
        for e, r in enumerate(refs):
            rew, done, _ = r.step(acts[e])
            assert torch.equal(b["rewards"][e, t].cpu(), f16(rew))
            check_row(b, e, t + 1, r.obs, r.beta, r.prev_assigns)
    env.sync()


def test_real_env_nan_benefits_stay_in_bounds():
    """NaN entries in an injected benefit table (the reference's argsort would rank them
    last): every ranking pick must still be a valid task / agent index, so the observation
    pass reads in bounds and the rollout completes."""
    E, n, m, T, L, N, M = 3, 12, 20, 4, 2, 4, 4
    rng = np.random.RandomState(11)
    tables = rng.uniform(0.0, 1.0, size=(E, n, m, T))
    tables[:, :, ::3] = np.nan          # a third of the tasks NaN for every agent
    tables[1] = np.nan                  # one env entirely NaN
    env = RealAssignEnvBatch(1, n, m, T, N, M, L, 0.5, sat_prox_mat=tables, num_envs=E, device=DEV)
    b = new_batch(env, E)
    env.reset(b, 0)
    for t in range(T):
        b["actions"][:, t, :, 0] = torch.from_numpy(rng.randint(0, m, size=(E, n))).to(torch.int16).to(DEV)
        env.step(b, t)
    env.sync()
    assert b["obs"].shape[0] == E


def test_real_env_errors():
    tab = np.ones((4, 6, 3))
    with pytest.raises(ValueError):
        RealAssignEnvBatch(1, 4, 6, 3, 2, 3, 2, 0.5, sat_prox_mat=tab, device=DEV)  # odd M
    with pytest.raises(ValueError):
        RealAssignEnvBatch(1, 7, 6, 3, 2, 2, 2, 0.5, sat_prox_mat=np.ones((7, 6, 3)), device=DEV)  # n > m
    with pytest.raises(ValueError):
        RealAssignEnvBatch(1, 4, 6, 3, 2, 2, 2, 0.5, device=DEV)  # no sat_prox_mat
    env = RealAssignEnvBatch(1, 4, 6, 3, 2, 2, 2, 0.5, sat_prox_mat=tab, num_envs=2, device=DEV)
    b = new_batch(env, 2)
    env.reset(b, 0)
    b["actions"][:, 0, :, 0] = 9
    env.step(b, 0)
    with pytest.raises(ValueError, match="out of range"):
        env.sync()


def test_gpu_runner_drives_real_env():
    """The "gpu" runner + BasicMAC (PyTorch RNNAgent on the float16 obs) + epsilon-greedy
    over a batched RealConstellationEnv: int16 actions written through EpisodeBatch.update."""
    from types import SimpleNamespace
    from marl_sap_amd.controllers import REGISTRY as mac_REGISTRY
    from marl_sap_amd.runners import REGISTRY as r_REGISTRY
    n, m, T, E = 12, 20, 5, 8
    tab = np.random.RandomState(0).uniform(size=(n, m, T))
    args = SimpleNamespace(
        batch_size_run=E, env="real_constellation_env",
        env_args=dict(num_planes=3, num_sats_per_plane=4, m=m, T=T, N=3, M=4, L=3, lambda_=0.5,
                      sat_prox_mat=tab, graphs=[None] * T, seed=0),
        test_nepisode=1, runner_log_interval=10 ** 9, n=n, m=m, T=T, hidden_dim=64, use_rnn=True,
        obs_last_action=False, obs_agent_id=False, agent_output_type="q", action_selector="epsilon_greedy",
        agent="rnn", epsilon_start=0.3, epsilon_finish=0.3, epsilon_anneal_time=1, evaluation_epsilon=0.0,
        mac="basic_mac")
    runner = r_REGISTRY["gpu"](args, None)
    env = runner.get_env()
    mac = mac_REGISTRY["basic_mac"](env.scheme, {"agents": n}, args)
    mac.cuda()
    runner.setup(env.scheme, {"agents": n}, env.preprocess, mac)
    batch = runner.run(test_mode=False)
    assert batch["actions"].dtype == torch.int16 and batch["obs"].dtype == torch.float16
    a = batch["actions"][:, :T, :, 0]
    assert int(a.min()) >= 0 and int(a.max()) < m
    assert torch.equal(batch["actions_onehot"][:, :T].argmax(-1).to(torch.int16), a)
    assert runner.t_env == E * T
    ret = batch["rewards"][:, :T].double().sum((1, 2)).cpu()
    np.testing.assert_allclose(runner.last_returns.cpu().numpy(), ret.numpy(), rtol=5e-3, atol=5e-3)


def _variant_env(kind, table, N, M, L, lam, prios, E, bands=None, nbr=None, prev0=None, seed=0):
    from marl_sap_amd.envs import InterferenceAssignEnvBatch, RealPowerAssignEnvBatch
    n, m, T = table.shape[-3:]
    if kind == "power":
        return RealPowerAssignEnvBatch(1, n, m, T, N, M, L, lam, sat_prox_mat=table, graphs=[None] * T,
                                       task_prios=prios, num_envs=E, initial_assignments=prev0, seed=seed,
                                       device=DEV)
    return InterferenceAssignEnvBatch(1, n, None, T, N, M, L, lam, task_prios=prios, sat_freq_bands=bands,
                                      sat_prox_mat=table, neighbor_matrix=nbr, num_envs=E,
                                      initial_assignments=prev0, seed=seed, device=DEV)


def test_real_variants_match_reference_fixture(golden):
    """RealPowerConstellationEnv / InterferenceConstellationEnv outputs of the reference
    itself (power drain and death, band conflicts), float16 scheme incl. power_states."""
    d = golden("real_variants")
    for c in range(int(d["n_cases"])):
        n, m, T, L, N, M = (int(x) for x in d[f"v{c}_spec"])
        env = _variant_env(str(d[f"v{c}_kind"]), d[f"v{c}_table"], N, M, L, float(d[f"v{c}_lambda"]),
                           d[f"v{c}_prios"], 2, bands=d[f"v{c}_bands"], nbr=d[f"v{c}_nbr"], prev0=d[f"v{c}_prev0"])
        assert env.obs_space_size == int(d[f"v{c}_obs_size"]) and "power_states" in env.scheme
        b = new_batch(env, 2)
        env.reset(b, 0)
        for e in range(2):
            check_row(b, e, 0, d[f"v{c}_obs0"], d[f"v{c}_beta0"], d[f"v{c}_prev0"])
            assert torch.equal(b["power_states"][e, 0].cpu(), f16(np.ones(n)))
        for t in range(T):
            b["actions"][:, t, :, 0] = torch.from_numpy(d[f"v{c}_actions"][t]).to(torch.int16).to(DEV)
            env.step(b, t)
            for e in range(2):
                assert torch.equal(b["rewards"][e, t].cpu(), f16(d[f"v{c}_rewards"][t])), (c, t)
                check_row(b, e, t + 1, d[f"v{c}_obs"][t], d[f"v{c}_beta"][t], d[f"v{c}_prev"][t])
                assert torch.equal(b["power_states"][e, t + 1].cpu(), f16(d[f"v{c}_power"][t]))
        env.sync()


@pytest.mark.parametrize("kind,n,m,T,L,N,M", [("power", 14, 24, 9, 3, 4, 6), ("interference", 20, 30, 8, 2, 5, 4),
                                             ("interference", 33, 50, 7, 3, 6, 8)])
def test_real_variants_match_oracle(oracle, kind, n, m, T, L, N, M):
    """Per-env sparse tables (equal totals), Philox reset assignments read back from the
    batch and replayed on the oracle; integer-valued neighbour matrix with self loops."""
    E = 4
    rng = np.random.RandomState(n + m)
    tables = rng.uniform(0.0, 1.0, size=(E, n, m, T)) * (rng.uniform(size=(E, n, m, 1)) > 0.6)
    prios = rng.choice([1.0, 1.0, 1.0, 5.0], size=m)
    bands = rng.randint(0, 4, size=n)
    nbr = (rng.uniform(size=(m, m)) > 0.75).astype(np.float64)
    nbr = np.maximum(nbr, nbr.T)
    np.fill_diagonal(nbr, 1.0)
    env = _variant_env(kind, tables, N, M, L, 0.5, prios, E, bands=bands, nbr=nbr, seed=11)
    b = new_batch(env, E)
    env.reset(b, 0)
    prev0 = b["prev_assigns"][:, 0].cpu().numpy().astype(np.int64)
    assert all(len(set(p)) == n and p.min() >= 0 and p.max() < m for p in prev0)  # choice(m, n, replace=False)
    refs = [oracle.OracleRealVariantEnv(kind, tables[e], N, M, L, 0.5, prios, prev0[e], bands=bands,
                                        neighbor_matrix=nbr) for e in range(E)]
    for e, r in enumerate(refs):
        r.reset()
        check_row(b, e, 0, r.obs, r.beta, r.prev_assigns)
    for t in range(T):
        acts = np.where(rng.uniform(size=(E, n)) < 0.3, rng.randint(0, 3, size=(E, n)), rng.randint(0, m, size=(E, n)))
        b["actions"][:, t, :, 0] = torch.from_numpy(acts).to(torch.int16).to(DEV)
        env.step(b, t)
        for e, r in enumerate(refs):
            rew, _, _ = r.step(acts[e])
            assert torch.equal(b["rewards"][e, t].cpu(), f16(rew)), (e, t)
            check_row(b, e, t + 1, r.obs, r.beta, r.prev_assigns)
            assert torch.equal(b["power_states"][e, t + 1].cpu(), f16(r.power_states))
    env.sync()
    # a second episode draws new assignments
    env.reset(b, 0)
    assert not np.array_equal(b["prev_assigns"][:, 0].cpu().numpy(), prev0)


REAL_RUNNER_TAGS = ["real_eg_16", "real_sap_16", "real_eg_32"]


@pytest.mark.parametrize("agent", ["rnn", "rnn_fused"])
@pytest.mark.parametrize("tag", REAL_RUNNER_TAGS)
def test_runner_matches_reference_real_dump(golden, tag, agent):
    """The "episode" runner + BasicMAC over the batched RealConstellationEnv against the
    reference EpisodeRunner's EpisodeBatch (tests/golden/real_runner_dumps.npz): same
    weights, greedy epsilon-greedy / SAP actions, every scheme field and the return."""
    from types import SimpleNamespace
    from marl_sap_amd.controllers import REGISTRY as mac_REGISTRY
    from marl_sap_amd.runners import REGISTRY as r_REGISTRY
    g = golden("real_runner_dumps")
    n, m, T, N, M, L, use_rnn = [int(x) for x in g[f"{tag}__cfg"]]
    sel = str(g[f"{tag}__names"][0])
    args = SimpleNamespace(
        batch_size_run=1, env="real_constellation_env",
        env_args=dict(num_planes=1, num_sats_per_plane=n, m=m, T=T, N=N, M=M, L=L, lambda_=float(g[f"{tag}__lambda"]),
                      sat_prox_mat=g[f"{tag}__table"], graphs=[None] * T, task_prios=g[f"{tag}__prios"], seed=0),
        runner_protocol="episode", test_nepisode=1, runner_log_interval=10 ** 9, n=n, m=m, T=T, hidden_dim=64,
        use_rnn=bool(use_rnn), obs_last_action=False, obs_agent_id=False, agent_output_type="q",
        action_selector=sel, agent=agent, epsilon_start=0.0, epsilon_finish=0.0, epsilon_anneal_time=1000,
        evaluation_epsilon=0.0, mac="basic_mac")
    runner = r_REGISTRY["episode"](args, None)
    env = runner.get_env()
    mac = mac_REGISTRY["basic_mac"](env.scheme, {"agents": n}, args)
    mac.agent.load_state_dict({k[len(tag) + 5:]: torch.as_tensor(g[k]) for k in g.files
                               if k.startswith(f"{tag}__w__")})
    mac.to(DEV)
    runner.setup(env.scheme, {"agents": n}, env.preprocess, mac)
    batch = runner.run(test_mode=False)
    td = {k: v.cpu().numpy() for k, v in batch.data.transition_data.items()}
    for k in ["obs", "beta", "rewards", "actions", "actions_onehot", "avail_actions", "terminated", "filled",
              "prev_assigns"]:
        ref = g[f"{tag}__{k}"]
        assert td[k].dtype == ref.dtype, k
        np.testing.assert_array_equal(td[k], ref, err_msg=f"{tag}:{k}")
    np.testing.assert_allclose(np.array(runner.train_returns), g[f"{tag}__returns"], rtol=1e-5, atol=1e-6)
    assert runner.t_env == int(g[f"{tag}__t_env"])
