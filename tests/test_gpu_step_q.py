"""REDA's fused schedule ("step_q"): per step one asg_step_forward launch (env step t + the
RNNAgent forward of row t + 1, the observation row generated and consumed on chip, Q written)
and one asg_sap_select_into launch (noise + scipy-exact LSA, actions written into the batch
row).  A pure scheduling change: the batch, returns, hidden state, t_env and the numpy stream
equal the separate launches' (asg_step, the agent kernel, the SAP kernel) bit for bit -- the
GRU and the Linear agent, Philox and table benefit modes, ragged shapes, the jumpstart MAC of
mock_constellation_reda.yaml.  Reference: action_selectors/sap_selectors.py:52-98,
runners/episode_runner.py:60-127, controllers/jumpstart_controller.py:50-80."""
import ctypes
from types import SimpleNamespace

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():
    pytest.skip("needs a ROCm GPU", allow_module_level=True)

from marl_sap_amd import _lib  # noqa: E402
from marl_sap_amd.controllers import REGISTRY as MAC  # noqa: E402
from marl_sap_amd.runners import REGISTRY as RUN  # noqa: E402

DEV = torch.device("cuda", 0)


class _Logger:
    def log_stat(self, *a, **k):
        pass


def _table(n, m, T, seed=0):
    r = np.random.RandomState(seed)
    return r.rand(n, m, T) * (r.rand(n, m, 1) > 0.6) * r.choice([1.0, 10.0], size=(1, m, 1))


def _run(n, m, T, L, E, eps, benefits, fused, use_rnn=False, rng="philox", episodes=2, mac="basic_mac", **extra):
    env_args = dict(n=n, m=m, T=T, L=L, lambda_=0.5, bids_as_actions=False, seed=11, benefits=benefits)
    if benefits == "injected":
        env_args["sat_prox_mat"] = _table(n, m, T)
    args = SimpleNamespace(
        batch_size_run=E, env="mock_constellation_env", env_args=env_args, env_rng=rng, env_quirks=(),
        runner_protocol="episode", test_nepisode=1, runner_log_interval=10 ** 12, n=n, m=m, T=T, hidden_dim=64,
        use_rnn=use_rnn, obs_last_action=False, obs_agent_id=False, agent_output_type="q", action_selector="sap",
        agent="rnn", mac=mac, seed=5, epsilon_start=eps, epsilon_finish=eps, epsilon_anneal_time=1,
        evaluation_epsilon=0.0, fused_rollout=fused, **extra)
    runner = RUN["gpu"](args, _Logger())
    env = runner.get_env()
    torch.manual_seed(321)
    mac = MAC[mac](env.scheme, {"agents": n}, args)
    mac.to(DEV)
    runner.setup(env.scheme, {"agents": n}, env.preprocess, mac)
    with torch.no_grad():
        st = np.random.get_state()
        mode = mac.fused_mode(env, runner.new_batch())
        np.random.set_state(st)
    assert mode == ("step_q" if fused else None), mode
    out = []
    for _ in range(episodes):
        batch = runner.run(test_mode=False)
        out.append(({k: v.cpu().clone() for k, v in batch.data.transition_data.items()},
                    runner.last_returns.cpu().clone(), mac.hidden_states.detach().cpu().clone()))
    res = out, runner.t_env, list(runner.train_returns), np.random.rand()
    env.close()
    return res


def _same(a, b):
    (oa, ta, ra, na), (ob, tb, rb, nb) = a, b
    assert ta == tb and ra == rb and na == nb
    for (fa, reta, ha), (fb, retb, hb) in zip(oa, ob):
        for k in fa:
            assert torch.equal(fa[k], fb[k]), k
        assert torch.equal(reta, retb)
        assert torch.equal(ha, hb)


@pytest.mark.parametrize("n,m,T,L,E,eps,benefits,use_rnn,rng", [
    (64, 64, 6, 3, 24, 0.05, "bump", False, "philox"),   # configs[2]'s shape, mock_constellation_reda's agent
    (64, 64, 5, 3, 10, 0.3, "dense", True, "philox"),    # the GRU agent
    (20, 25, 5, 3, 9, 0.2, "bump", False, "philox"),     # the reference's default env: ragged tiles
    (16, 16, 4, 2, 12, 0.5, "bump", True, "philox"),     # configs[1]'s shape
    (33, 41, 4, 2, 6, 0.1, "injected", False, "mt19937"),  # odd m, an injected table, MT19937 draws
    (20, 25, 5, 3, 9, 0.2, "bump", False, "mt19937"),    # the same-seed mode (numpy's stream per env)
])
def test_step_q_is_bit_identical(n, m, T, L, E, eps, benefits, use_rnn, rng):
    # both runs start from the same numpy global state (the final draw checks that neither
    # schedule consumes more of it than the other)
    np.random.seed(3)
    b = _run(n, m, T, L, E, eps, benefits, fused=False, use_rnn=use_rnn, rng=rng)
    np.random.seed(3)
    _same(_run(n, m, T, L, E, eps, benefits, fused=True, use_rnn=use_rnn, rng=rng), b)


def test_step_q_jumpstart_reda():
    """mock_constellation_reda.yaml's MAC: JumpstartMAC (HAA jumpstart) + the SAP selector + the
    Linear agent; at jumpstart epsilon 0.5 HAA and RL steps interleave, the coin flips drawn
    from numpy's stream in the reference's order either way."""
    js = dict(jumpstart_action_selector="haa_selector", jumpstart_epsilon_start=0.5, jumpstart_epsilon_finish=0.5,
              jumpstart_epsilon_anneal_time=1, jumpstart_evaluation_epsilon=0.0)
    kw = dict(n=20, m=25, T=6, L=3, E=7, eps=0.1, benefits="bump", episodes=3, mac="jumpstart_mac", **js)
    np.random.seed(8)
    b = _run(fused=False, **kw)
    np.random.seed(8)
    _same(_run(fused=True, **kw), b)


def test_step_forward_equals_step_then_forward():
    """asg_step_forward's Q rows and hidden state equal asg_step followed by the agent kernel
    on the observation row it wrote (asg_rnn_agent_forward), bitwise; the batch too."""
    from marl_sap_amd.components import EpisodeBatch
    from marl_sap_amd.envs import AssignEnvBatch
    from marl_sap_amd.modules.agents import RNNFusedAgent
    for n, m, L, use_rnn in ((64, 64, 3, True), (20, 25, 3, False), (32, 256, 3, True)):
        T, E = 5, 6
        outs = []
        for fused in (True, False):
            env = AssignEnvBatch(n, m, T, L, 0.5, seed=2, num_envs=E, device=DEV)
            b = EpisodeBatch(env.scheme, {"agents": n}, E, T + 1, preprocess=env.preprocess, device=DEV,
                             time_major=True)
            torch.manual_seed(4)
            agent = RNNFusedAgent(m * (L + 1), SimpleNamespace(hidden_dim=64, use_rnn=use_rnn, m=m)).to(DEV)
            env.reset(b, 0)
            g = torch.Generator(device="cpu").manual_seed(1)
            h = torch.randn((E * n, 64), generator=g).to(DEV)
            qs, hs = [], []
            with torch.no_grad():
                for t in range(T - 1):
                    b["actions"][:, t, :, 0] = torch.randint(0, m, (E, n), generator=g).to(DEV)
                    if fused:
                        q, h = env.step_forward(b, t, agent, h)
                    else:
                        env.step(b, ts=t)
                        q, h = agent(b["obs"][:, t + 1].reshape(E * n, -1), h)
                    qs.append(q.cpu().clone())
                    hs.append(h.cpu().clone())
            env.sync()
            outs.append(({k: v.cpu() for k, v in b.data.transition_data.items()}, qs, hs, env.get_returns().cpu()))
            env.close()
        (fa, qa, ha, ra), (fb, qb, hb, rb) = outs
        for k in fa:
            assert torch.equal(fa[k], fb[k]), (n, m, k)
        for x, y in zip(qa + ha, qb + hb):
            assert torch.equal(x, y), (n, m)
        assert torch.equal(ra, rb)


def test_reset_forward_equals_reset_then_forward():
    """asg_reset_forward (the step_q schedule's reset + forward on the reset row, one launch):
    the batch, Q rows and hidden state of asg_reset followed by the agent kernel, bitwise --
    Philox bump / dense benefits and the MT19937 mode, two episodes (the second reset's key)."""
    from marl_sap_amd.components import EpisodeBatch
    from marl_sap_amd.envs import AssignEnvBatch
    from marl_sap_amd.modules.agents import RNNFusedAgent
    for n, m, L, use_rnn, benefits, rng in ((64, 64, 3, True, "bump", "philox"), (20, 25, 3, False, "bump", "philox"),
                                            (32, 48, 2, True, "dense", "philox"), (20, 25, 3, False, "bump", "mt19937")):
        T, E = 4, 6
        outs = []
        for fused in (True, False):
            env = AssignEnvBatch(n, m, T, L, 0.5, seed=2, num_envs=E, device=DEV, benefits=benefits, rng=rng)
            assert env.fused_reset_ok
            b = EpisodeBatch(env.scheme, {"agents": n}, E, T + 1, preprocess=env.preprocess, device=DEV,
                             time_major=True)
            torch.manual_seed(4)
            agent = RNNFusedAgent(m * (L + 1), SimpleNamespace(hidden_dim=64, use_rnn=use_rnn, m=m)).to(DEV)
            rec = []
            with torch.no_grad():
                for ep in range(2):
                    h = agent.init_hidden().unsqueeze(0).expand(E, n, -1)
                    if fused:
                        q, h = env.reset_forward(b, 0, agent, h)
                    else:
                        env.reset(b, ts=0)
                        q, h = agent(b["obs"][:, 0].reshape(E * n, -1), h)
                    rec.append((q.cpu().clone(), h.cpu().clone(),
                                {k: v.cpu().clone() for k, v in b.data.transition_data.items()}))
                    assert env.k == 0
                    # one step so the handle advances, then a new episode
                    b["actions"][:, 0, :, 0] = torch.arange(n, device=DEV).remainder(m).expand(E, n)
                    env.step(b, ts=0)
            env.sync()
            outs.append(rec)
            env.close()
        for (qa, ha, fa), (qb, hb, fb) in zip(*outs):
            assert torch.equal(qa, qb) and torch.equal(ha, hb), (n, m, benefits, rng)
            for k in fa:
                assert torch.equal(fa[k], fb[k]), (n, m, benefits, rng, k)


def test_sap_select_into_equals_float_output():
    """asg_sap_select_into: the int64 ids of asg_sap_select's float output, -1 rows for a NaN
    env, and its per-env status word min-accumulated over calls."""
    from marl_sap_amd.action_selectors.sap_selectors import SequentialAssignmentProblemSelector
    B, n, m = 300, 20, 25
    sel = SequentialAssignmentProblemSelector(SimpleNamespace(epsilon_start=0.3, epsilon_finish=0.3,
                                                              epsilon_anneal_time=1, evaluation_epsilon=0.0, seed=2))
    twin = SequentialAssignmentProblemSelector(sel.args)
    q = torch.randn((B, n, m), device=DEV)
    q[7, 3, 4] = float("nan")
    with torch.no_grad():
        f = twin.select_action(q, None, 0)
        out = torch.full((B, n), 99, dtype=torch.int64, device=DEV)
        r = sel.select_action(q, None, 0, out=out)
    assert r is out
    assert torch.equal(out.cpu(), f.cpu().to(torch.int64))
    assert bool((out[7] == -1).all())
    st = sel.status._sticky
    assert int(st[7]) == _lib.ASG_E_LSA_INVALID and int(st.abs().sum()) == abs(_lib.ASG_E_LSA_INVALID)
    q[7, 3, 4] = 0.0
    with torch.no_grad():
        sel.select_action(q, None, 0, out=out)
    assert int(sel.status._sticky[7]) == _lib.ASG_E_LSA_INVALID  # sticky until the flush
    with pytest.raises(ValueError, match="invalid numeric entries"):
        sel.status.flush()
    sel.status.flush()  # cleared
    # the ABI rejects what the fused kernel does not take
    L = _lib.lib()
    rc = L.asg_sap_select_into(ctypes.c_void_p(q.data_ptr()), _lib.i64arr(q.stride()), B, 30, m, 0.1, 1, 1, 0,
                               ctypes.c_void_p(out.data_ptr()), None, None, None)
    assert rc == _lib.ASG_E_INVALID_ARG
