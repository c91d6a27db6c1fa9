"""bids_as_actions on the batched real-env family (VERDICT r5 "Next" item 4).

The reference's RealConstellationEnv, RealPowerConstellationEnv and InterferenceConstellationEnv
all accept bids: the actions row is a float32 [n, m] bid matrix per agent set and the step's
tasks are scipy's linear_sum_assignment(bids, maximize=True) (real_constellation_env.py:110-112,
140-142; real_power_constellation_env.py:112, 142; interference_constellation_env.py:121, 159).
Here asg_real_step solves every env's bids with the batched scipy-exact LSA (asg_lsa_batched,
rectangular n <= m) and feeds the assignments to the same transition.  Checked:
  * bit-exact against the reference's own outputs (tests/golden/real_bids.npz: tie-free bids);
  * against the C oracle (scipy LSA restatement + the real-env oracle) on per-env tables and
    bids, including the reference's 324 x 450 constellation shape;
  * NaN bids raise scipy's ValueError at sync; the GpuVecRunner drives it with the continuous
    selector (torch noise on the device) end to end."""
from types import SimpleNamespace

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():
    pytest.skip("needs a ROCm GPU", allow_module_level=True)

from marl_sap_amd.components import EpisodeBatch  # noqa: E402
from marl_sap_amd.envs import InterferenceAssignEnvBatch, RealAssignEnvBatch, RealPowerAssignEnvBatch  # noqa: E402

DEV = torch.device("cuda", 0)


def f16(x):
    return torch.from_numpy(np.asarray(x, dtype=np.float64)).to(torch.float16)


def new_batch(env, E):
    return EpisodeBatch(env.scheme, {"agents": env.n}, E, env.T + 1, preprocess=env.preprocess, device=DEV,
                        time_major=True)


def _env(kind, table, N, M, L, lam, prios, E, bands=None, nbr=None, prev0=None, seed=0):
    n, m, T = table.shape[-3:]
    if kind == "real":
        return RealAssignEnvBatch(1, n, m, T, N, M, L, lam, sat_prox_mat=table, graphs=[None] * T, task_prios=prios,
                                  num_envs=E, bids_as_actions=True, device=DEV)
    if kind == "power":
        return RealPowerAssignEnvBatch(1, n, m, T, N, M, L, lam, sat_prox_mat=table, graphs=[None] * T,
                                       task_prios=prios, num_envs=E, initial_assignments=prev0, seed=seed,
                                       bids_as_actions=True, device=DEV)
    return InterferenceAssignEnvBatch(1, n, None, T, N, M, L, lam, task_prios=prios, sat_freq_bands=bands,
                                      sat_prox_mat=table, neighbor_matrix=nbr, num_envs=E, initial_assignments=prev0,
                                      seed=seed, bids_as_actions=True, device=DEV)


def _row(b, e, t, obs, beta, prev):
    assert torch.equal(b["obs"][e, t].cpu(), f16(obs))
    assert torch.equal(b["beta"][e, t].cpu(), f16(beta))
    assert torch.equal(b["prev_assigns"][e, t].cpu(), torch.from_numpy(np.asarray(prev)).to(torch.int16))
    assert bool(b["avail_actions"][e, t].all()) and int(b["filled"][e, t, 0]) == 1


def test_real_bids_scheme():
    tab = np.random.RandomState(1).uniform(0.01, 1.0, size=(6, 10, 4))
    env = _env("real", tab, 2, 4, 3, 0.5, None, 2)
    assert env.scheme["actions"] == {"vshape": (10,), "group": "agents", "dtype": torch.float32}
    assert env.preprocess == {}  # no one-hot (real_constellation_env.py:110-112)
    b = new_batch(env, 2)
    assert "actions_onehot" not in b.data.transition_data
    env.reset(b, 0)
    b["actions"][:, 0] = torch.rand(2, 6, 10, device=DEV)
    env.step(b, 0)
    env.sync()
    env.close()


def test_real_bids_match_reference_fixture(golden):
    d = golden("real_bids")
    for c in range(int(d["n_cases"])):
        kind = str(d[f"b{c}_kind"])
        n, m, T, L, N, M = (int(x) for x in d[f"b{c}_spec"])
        env = _env(kind, d[f"b{c}_table"], N, M, L, float(d[f"b{c}_lambda"]),
                   d[f"b{c}_prios"] if kind != "real" else None, 2, bands=d[f"b{c}_bands"], nbr=d[f"b{c}_nbr"],
                   prev0=d[f"b{c}_prev0"])
        assert env.obs_space_size == int(d[f"b{c}_obs_size"])
        b = new_batch(env, 2)
        env.reset(b, 0)
        for e in range(2):
            _row(b, e, 0, d[f"b{c}_obs0"], d[f"b{c}_beta0"], d[f"b{c}_prev0"])
        ret = np.zeros(2)
        for t in range(T):
            b["actions"][:, t] = torch.from_numpy(d[f"b{c}_bids"][t]).to(DEV)  # both envs bid the same
            done = env.step(b, t)
            assert done == bool(d[f"b{c}_done"][t])
            for e in range(2):
                assert torch.equal(b["rewards"][e, t].cpu(), f16(d[f"b{c}_rewards"][t])), (kind, c, t)
                # prev_assigns row t + 1 = the step's assignments = scipy's LSA of the bids
                _row(b, e, t + 1, d[f"b{c}_obs"][t], d[f"b{c}_beta"][t], d[f"b{c}_prev"][t])
                if kind != "real":
                    assert torch.equal(b["power_states"][e, t + 1].cpu(), f16(d[f"b{c}_power"][t]))
                assert bool(b["terminated"][e, t, 0]) == (t + 1 >= T)
            ret += sum(d[f"b{c}_rewards"][t])
        env.sync()
        if kind == "real":
            assert np.array_equal(env.get_returns().cpu().numpy(), ret)
        env.close()


@pytest.mark.parametrize("kind,n,m,T,L,N,M,E", [("real", 40, 64, 5, 3, 4, 6, 6), ("power", 33, 50, 6, 3, 5, 4, 4),
                                                ("interference", 20, 30, 5, 2, 5, 4, 4),
                                                ("real", 324, 450, 3, 3, 10, 10, 2)])
def test_real_bids_match_oracle(oracle, kind, n, m, T, L, N, M, E):
    """Per-env tables and bids; the assignments are the oracle's scipy LSA of exactly the float32
    bids in the batch (ties impossible: continuous bids), then the oracle env steps them."""
    rng = np.random.RandomState(n * 7 + m)
    tables = rng.uniform(0.0, 1.0, size=(E, n, m, T)) * (rng.uniform(size=(E, n, m, 1)) > 0.5)
    prios = rng.choice([1.0, 1.0, 1.0, 5.0], size=m)
    bands = rng.randint(0, 4, size=n)
    nbr = (rng.uniform(size=(m, m)) > 0.75).astype(np.float64)
    nbr = np.maximum(nbr, nbr.T)
    np.fill_diagonal(nbr, 1.0)
    env = _env(kind, tables, N, M, L, 0.5, prios if kind != "real" else None, E, bands=bands, nbr=nbr, seed=5)
    b = new_batch(env, E)
    env.reset(b, 0)
    prev0 = b["prev_assigns"][:, 0].cpu().numpy().astype(np.int64)
    if kind == "real":
        refs = [oracle.OracleRealEnv(tables[e], N, M, L, 0.5) for e in range(E)]
    else:
        refs = [oracle.OracleRealVariantEnv(kind, tables[e], N, M, L, 0.5, prios, prev0[e], bands=bands,
                                            neighbor_matrix=nbr) for e in range(E)]
    for e, r in enumerate(refs):
        r.reset()
        _row(b, e, 0, r.obs, r.beta, r.prev_assigns)
    for t in range(T):
        bids = rng.uniform(0.0, 1.0, size=(E, n, m)).astype(np.float32)
        bids[:, :, : m // 8] += np.float32(0.5)  # contested columns
        b["actions"][:, t] = torch.from_numpy(bids).to(DEV)
        env.step(b, t)
        for e, r in enumerate(refs):
            _, col = oracle.lsa(bids[e].astype(np.float64), maximize=True)
            rew, _, _ = r.step(col)
            assert torch.equal(b["rewards"][e, t].cpu(), f16(rew)), (e, t)
            _row(b, e, t + 1, r.obs, r.beta, r.prev_assigns)
            assert np.array_equal(b["prev_assigns"][e, t + 1].cpu().numpy().astype(np.int64), col)
            if kind != "real":
                assert torch.equal(b["power_states"][e, t + 1].cpu(), f16(r.power_states))
    env.sync()
    env.close()


def test_real_bids_invalid_entries_raise():
    tab = np.random.RandomState(2).uniform(0.01, 1.0, size=(8, 12, 4))
    env = _env("real", tab, 2, 4, 3, 0.5, None, 3)
    b = new_batch(env, 3)
    env.reset(b, 0)
    bids = torch.rand(3, 8, 12, device=DEV)
    bids[1, 3, 4] = float("nan")
    b["actions"][:, 0] = bids
    env.step(b, 0)
    with pytest.raises(ValueError, match="invalid numeric entries"):
        env.sync()
    env.sync()  # the sticky error was cleared
    env.close()


def test_gpu_runner_real_bids_continuous_selector(oracle):
    """GpuVecRunner + BasicMAC (RNNAgent) + ContinuousActionSelector over a bids_as_actions real
    env (ippo_sap.yaml's env path on the real family): the bids rows are the selector's, every
    step's assignments are scipy's LSA of the stored bids."""
    from marl_sap_amd.controllers import REGISTRY as mac_REGISTRY
    from marl_sap_amd.runners import REGISTRY as r_REGISTRY
    n, m, T, E = 12, 20, 4, 6
    tab = np.random.RandomState(3).uniform(0.01, 1.0, size=(n, m, T))
    args = SimpleNamespace(
        batch_size_run=E, env="real_constellation_env",
        env_args=dict(num_planes=3, num_sats_per_plane=4, m=m, T=T, N=3, M=4, L=3, lambda_=0.5, sat_prox_mat=tab,
                      graphs=[None] * T, seed=0, bids_as_actions=True),
        test_nepisode=1, runner_log_interval=10 ** 9, n=n, m=m, T=T, hidden_dim=64, use_rnn=True,
        obs_last_action=False, obs_agent_id=False, agent_output_type="pi_logits", action_selector="continuous",
        agent="rnn", epsilon_start=0.3, epsilon_finish=0.3, epsilon_anneal_time=1, evaluation_epsilon=0.0,
        mac="basic_mac", softmax_agent_inputs=True)
    runner = r_REGISTRY["gpu"](args, None)
    env = runner.get_env()
    assert env.bids_as_actions
    mac = mac_REGISTRY["basic_mac"](env.scheme, {"agents": n}, args)
    mac.cuda()
    runner.setup(env.scheme, {"agents": n}, env.preprocess, mac)
    batch = runner.run(test_mode=False)
    bids = batch["actions"][:, :T].cpu().double().numpy()
    assert batch["actions"].dtype == torch.float32 and np.isfinite(bids).all() and np.abs(bids).sum() > 0
    for e in range(E):
        for t in range(T):
            _, col = oracle.lsa(bids[e, t], maximize=True)
            assert np.array_equal(batch["prev_assigns"][e, t + 1].cpu().numpy().astype(np.int64), col), (e, t)
    assert runner.t_env == E * T
