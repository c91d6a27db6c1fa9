"""The timed kernel at the timed size, against the oracle.

bench.py's headline runs GpuVecRunner with the fused rollout step (asg_step_select ->
rollout_h2_kernel: env transition t + RNNAgent forward + epsilon-greedy for t + 1 in one
launch) at BASELINE configs[2] (64 x 64, 16,384 envs, T = 20, eps = 0.05, Philox bumps), and
its configs[4] leg at 256 x 256 dense with 2,048 envs.  These tests build the runner exactly
as bench.make_args does, run one whole episode through runner.run(), and check:

  * every env: the size-independent invariants of the batch (one-hot block == actions,
    actions_onehot, lookahead window shift, beta == block 1, terminal zero rows, avail /
    filled / terminated / prev_assigns, returns == sum of rewards);
  * sampled envs (first, last, one inside each wave stride): a full replay of the env on
    the C oracle (mock_constellation_env.py:116-162 semantics: rewards, obs, beta, one-hots,
    returns) from the episode's exported bump parameters (numpy float64);
  * EVERY env: the same replay in C over all envs (oracle/asg_check.c, multi-threaded, env
    chunks) from the handle's float64 export of those parameters;
  * the same sampled envs' actions: the PyTorch RNNAgent module (the reference's
    rnn_agent.py:23-31, fp32, same weights) replayed over the batch's observation rows gives
    Q_t; rows whose Philox draw explores (oracle/philox.py, the kernel's draw restated) must
    hold the predicted task, every other row the argmax of Q_t (rows whose top-2 gap is
    below 1e-4 may pick either of the tied pair).

Reference anchors: runners/episode_runner.py:60-127 (the loop), envs/mock_constellation_env.py
:116-162 (step), :228-274 (beta_hat), action_selectors/classic_selectors.py:28-54.
"""
import gc
import os
import sys

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():
    pytest.skip("needs a ROCm GPU", allow_module_level=True)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from marl_sap_amd.controllers import REGISTRY as MAC  # noqa: E402
from marl_sap_amd.modules.agents import RNNAgent  # noqa: E402
from marl_sap_amd.runners import REGISTRY as RUN  # noqa: E402
from oracle.check import bump_table_from_params, replay_all, replay_and_compare  # noqa: E402
from oracle.philox import eps_greedy_draws  # noqa: E402

DEV = torch.device("cuda", 0)
GAP = 1e-4  # top-2 Q gap below which fp32 summation order may flip the greedy choice


def _bench_runner(config, args_over=None, **over):
    a = bench.parse(["--config", str(config)])
    for k, v in over.items():
        setattr(a, k, v)
    args = bench.make_args(a, a.envs, **(args_over or {}))
    runner = RUN["gpu"](args, bench.NullLogger())
    env = runner.get_env()
    torch.manual_seed(a.seed)
    mac = MAC["basic_mac"](env.scheme, {"agents": a.n}, args)
    mac.to(DEV)
    runner.setup(env.scheme, {"agents": a.n}, env.preprocess, mac)
    return a, args, runner, env, mac


def _sample(E):
    # first, last, and one env inside each wave's env stride (grid 256 WGs x 8 waves)
    idx = {0, 1, E // 2, E - 1}
    for s in (2048, 4096, 8192, 12288):
        if s + 3 < E:
            idx.add(s + 3)
    idx.add(min(E - 1, 777))
    return np.array(sorted(idx))


def _check_invariants(b, env, E, n, m, T, prev0):
    obs, beta = b["obs"], b["beta"]
    for t in range(T):  # per row: bounded temporaries at 256 x 256
        a = b["actions"][:, t, :, 0]
        assert bool(((a >= 0) & (a < m)).all()), t
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
    assert bool(b["terminated"][:, T - 1, 0].all())
    assert torch.equal(b["prev_assigns"][:, 0], prev0)
    srt = prev0.sort(dim=1)[0]
    assert (srt[:, 1:] != srt[:, :-1]).all()
    r = env.get_returns()
    assert torch.allclose(b["rewards"][:, :T].double().sum((1, 2)), r, rtol=1e-5, atol=1e-3)
    return r


def _check_actions(b, mac, idx, n, m, T, eps, seed, counter0):
    """Replay the PyTorch RNNAgent over the sampled envs' observation rows; predicted
    action = the Philox exploration draw or the greedy argmax (gap-tolerant)."""
    args = mac.args
    ref = RNNAgent(b["obs"].shape[-1], args).to(DEV)
    ref.load_state_dict(mac.selector_agent.state_dict())
    ix = torch.as_tensor(idx, device=DEV)
    h = torch.zeros((len(idx) * n, 64), device=DEV)
    rows = (idx[:, None] * n + np.arange(n)[None, :]).reshape(-1)
    n_explore = n_close = 0
    for t in range(T):
        x = b["obs"][ix, t].reshape(len(idx) * n, -1)
        with torch.no_grad():
            q, h = ref(x, h)
        q = q.double().cpu().numpy()
        got = b["actions"][ix, t, :, 0].reshape(-1).cpu().numpy()
        explore, target = eps_greedy_draws(seed, rows, counter0 + t + 1, eps, m)
        greedy = q.argmax(1)
        srt = np.sort(q, axis=1)
        close = (srt[:, -1] - srt[:, -2]) < GAP
        ok_greedy = (got == greedy) | (close & (q[np.arange(len(got)), got] >= srt[:, -1] - GAP))
        want_ok = np.where(explore, got == target, ok_greedy)
        bad = np.flatnonzero(~want_ok)
        assert bad.size == 0, (f"t={t}: {bad.size} rows differ, first row {rows[bad[0]]}: got {got[bad[0]]} "
                               f"explore={explore[bad[0]]} target={target[bad[0]]} greedy={greedy[bad[0]]}")
        n_explore += int(explore.sum())
        n_close += int((close & ~explore).sum())
    total = T * len(rows)
    print(f"actions checked: {total} rows, {n_explore} exploring, {n_close} near-ties")
    assert 0.3 * eps * total <= n_explore <= 3 * eps * total + 5
    assert n_close <= 0.01 * total


@pytest.mark.parametrize("config", [2, 4])
def test_bench_workload_episode_vs_oracle(config):
    a, args, runner, env, mac = _bench_runner(config)
    E, n, m, T, L = a.envs, a.n, a.m, a.T, a.L
    try:
        with torch.no_grad():
            assert mac.fused_step_ok(env, _shape_probe(runner)), \
                "the bench schedule must be the fused rollout kernel"
        b = runner.run(test_mode=False)
        assert runner.t_env == E * T
        # the reset ran inside the episode's launch (asg_reset_rollout): its permutation is the
        # batch's prev_assigns row 0 (no quirks here; checked to be a partial permutation below),
        # its Philox episode key the handle's until the next reset
        prev0 = b["prev_assigns"][:, 0].reshape(E, n).clone()
        pz = prev0.sort(dim=1).values
        assert bool(((pz >= 0) & (pz < m)).all()) and bool((pz[:, 1:] != pz[:, :-1]).all())
        params = env.export_bump_params()
        env.sync()
        r = _check_invariants(b, env, E, n, m, T, prev0)
        idx = _sample(E)
        table = bump_table_from_params(params[idx].cpu().numpy(), T)
        td = {k: v[idx].cpu().numpy() for k, v in b.data.transition_data.items()}
        replay_and_compare(n, m, T, L, 0.5, table, prev0[idx].cpu().numpy(), td, r[idx].cpu().numpy(),
                           philox=True, rtol_reward=2e-7 if m > 64 else 0.0)
        # the sampled envs' float64 tables from their bump parameters (numpy) equal the handle's
        # own export; then EVERY env replayed on the C oracle from that export (asg_check.c)
        full = env.export_benefits()
        np.testing.assert_allclose(full[torch.as_tensor(idx, device=DEV)].cpu().numpy(), table, rtol=4e-16, atol=0)
        envs, compared = replay_all(n, m, T, L, 0.5, b.data.transition_data, full, prev0, r, philox=True,
                                    rtol_reward=2e-7 if m > 64 else 0.0)
        print(f"exhaustive oracle replay: {envs} envs, {compared} values compared")
        del full
        sel = mac.action_selector
        _check_actions(b, mac, idx, n, m, T, float(sel.epsilon), sel.seed, sel.calls - T)
    finally:
        env.close()
        del runner, mac, env
        gc.collect()
        torch.cuda.empty_cache()


def _shape_probe(runner):
    """A 1-env batch of the runner's scheme (the fused-step check reads only its layout)."""
    from marl_sap_amd.components import EpisodeBatch
    return EpisodeBatch(runner.scheme, runner.groups, 1, runner.T + 1, preprocess=runner.preprocess,
                        device=runner.device, time_major=True)


def test_compat_mode_configs2_episode_vs_oracle():
    """configs[2] (64 x 64, 16,384 envs, T = 20, the bench's GRU RNNAgent + epsilon-greedy 0.05)
    in the same-seed mode: env e replays numpy's legacy MT19937 stream seeded with seed + e --
    the throwaway __init__ table, the reset's table and its choice(m, n, False) permutation that
    the reference draws after np.random.seed(seed + e) (mock_constellation_env.py:32-34, :99-105)
    -- on the episode kernel (fused_mode "episode": asg_reset, then one asg_rollout launch).
    Sampled envs are rebuilt by the C oracle from the seed alone and replayed row by row against
    the batch (float64 table: obs / beta / rewards bit-exact); every env's invariants hold; the
    actions are the PyTorch RNNAgent's."""
    from oracle import oracle as ora
    a, args, runner, env, mac = _bench_runner(2, args_over={"env_rng": "mt19937"})
    E, n, m, T, L = a.envs, a.n, a.m, a.T, a.L
    try:
        with torch.no_grad():
            assert mac.fused_mode(env, _shape_probe(runner)) == "episode"
        b = runner.run(test_mode=False)
        assert runner.t_env == E * T
        prev0 = b["prev_assigns"][:, 0].reshape(E, n).clone()
        env.sync()
        r = _check_invariants(b, env, E, n, m, T, prev0)
        idx = _sample(E)
        tables, prevs = [], []
        for e in idx:
            oe = ora.OracleMockEnv(n, m, T, L, 0.5, mt=ora.MT(a.seed + int(e)))
            oe.reset()
            tables.append(oe.sat_prox_mat)
            prevs.append(oe.prev_assigns.copy())
        np.testing.assert_array_equal(prev0[idx].cpu().numpy(), np.stack(prevs))  # the seed's permutation
        # the handle's tables are the seed's (the device's float64 exp vs libm's: within 1e-12
        # relative, as tests/test_gpu_parity.py:test_mt_multi_env_streams), and the batch is
        # their exact replay
        dev_tab = env.export_benefits()[torch.as_tensor(idx, device=DEV)].cpu().numpy()
        np.testing.assert_allclose(dev_tab, np.stack(tables), rtol=1e-12, atol=0)
        td = {k: v[idx].cpu().numpy() for k, v in b.data.transition_data.items()}
        replay_and_compare(n, m, T, L, 0.5, dev_tab, prev0[idx].cpu().numpy(), td, r[idx].cpu().numpy())
        # EVERY env: its table and permutation rebuilt from np.random.seed(seed + e) alone, and
        # every batch row replayed exactly (asg_check.c)
        envs, compared = replay_all(n, m, T, L, 0.5, b.data.transition_data, env.export_benefits(), prev0, r,
                                    seed=a.seed)
        print(f"exhaustive same-seed replay: {envs} envs, {compared} values compared")
        sel = mac.action_selector
        _check_actions(b, mac, idx, n, m, T, float(sel.epsilon), sel.seed, sel.calls - T)
    finally:
        env.close()
        del runner, mac, env
        gc.collect()
        torch.cuda.empty_cache()
