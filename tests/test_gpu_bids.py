"""bids_as_actions on the fused schedule (config/algs/ippo_sap.yaml: ContinuousActionSelector,
softmax_agent_inputs, agent_output_type "pi_logits", the mock env solving LSA(bids, maximize)).

asg_bids_select turns the agent's raw outputs into the bids -- BasicMAC.forward's pi_logits
softmax (controllers/basic_controller.py:37-46), the selector's softmax over the agents and
th.normal(x, std) (action_selectors/bet_selectors.py:12-20) -- writes them as the batch's
actions row and solves their LSA (envs/mock_constellation_env.py:121-122) for the env's next
step.  Checked here: the transforms against torch fp32 (noise off), the assignments against the
scipy oracle on exactly the bids written, the noise's distribution / determinism / sharding,
and the runner's fused schedule (asg_step_forward + asg_bids_select per step) against the split
launches (asg_step + the agent kernel + asg_bids_select) bit for bit."""
from types import SimpleNamespace

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():
    pytest.skip("needs a ROCm GPU", allow_module_level=True)

from marl_sap_amd.components.episode_buffer import EpisodeBatch  # noqa: E402
from marl_sap_amd.controllers import REGISTRY as MAC  # noqa: E402
from marl_sap_amd.envs.assign_env import AssignEnvBatch  # noqa: E402
from marl_sap_amd.runners import REGISTRY as RUN  # noqa: E402
from oracle import oracle as ora  # noqa: E402

DEV = torch.device("cuda", 0)
SEED = (5 * 0x9E3779B97F4A7C15 + 0x2545F4914F6CDD1D) & 0xFFFFFFFFFFFFFFFF


class _Logger:
    def log_stat(self, *a, **k):
        pass


def _env(n, m, T=5, L=3, E=16, base=0, seed=7):
    env = AssignEnvBatch(n, m, T, L, 0.5, bids_as_actions=True, seed=seed, num_envs=E, env_index_base=base,
                         device=DEV)
    batch = EpisodeBatch(env.scheme, {"agents": n}, E, T + 1, preprocess=env.preprocess, device=DEV,
                         time_major=True)
    env.reset(batch, ts=0)
    return env, batch


def _torch_bids(q, row_sm, col_sm):
    x = q.double()
    if row_sm:
        x = torch.softmax(x, dim=-1)
    if col_sm:
        x = torch.softmax(x, dim=1)
    return x


@pytest.mark.parametrize("n,m,row_sm,col_sm", [(64, 64, 1, 1), (20, 25, 1, 1), (16, 16, 0, 1), (33, 41, 1, 0),
                                               (1, 7, 1, 1), (8, 64, 0, 0)])
def test_bids_transforms_vs_torch_and_assignments_vs_scipy(n, m, row_sm, col_sm):
    E = 48
    env, batch = _env(n, m, E=E)
    g = torch.Generator(device="cpu").manual_seed(n * 100 + m)
    q = (torch.randn(E, n, m, generator=g) * 3.0).to(DEV)
    out = batch["actions"][:, 0]
    env.bids_select(q, out, row_sm, col_sm, 0.0, SEED, 1)
    want = _torch_bids(q, row_sm, col_sm)
    # fp32 softmaxes (exp(x - max) / sum, torch's form) against a float64 evaluation
    assert torch.allclose(out.double(), want, rtol=2e-6, atol=1e-8), (out.double() - want).abs().max().item()
    bids = out.cpu().double().numpy()
    env.step(batch, 0)  # uses the assignments asg_bids_select left for row 0
    got = batch["prev_assigns"][:, 1].cpu().numpy()
    for e in range(E):
        _, col = ora.lsa(bids[e], maximize=True)
        assert np.array_equal(got[e], col), e
    env.sync()
    env.close()


def test_bids_tagged_step_equals_solving_the_row():
    """The step on a row asg_bids_select wrote uses its assignments; a row written by other means
    is solved by the step itself (bids_assign_kernel): the batches agree bit for bit."""
    n, m, E = 20, 25, 32
    a_env, a_batch = _env(n, m, E=E, seed=3)
    b_env, b_batch = _env(n, m, E=E, seed=3)
    q = torch.randn(E, n, m, device=DEV)
    for t in range(3):
        a_env.bids_select(q + t, a_batch["actions"][:, t], 1, 1, 0.2, SEED, t + 1)
        b_batch["actions"][:, t].copy_(a_batch["actions"][:, t])  # same bids, no tag
        a_env.step(a_batch, t)
        b_env.step(b_batch, t)
    for k, v in a_batch.data.transition_data.items():
        assert torch.equal(v, b_batch.data.transition_data[k]), k
    assert torch.equal(a_env.get_returns(), b_env.get_returns())
    a_env.close()
    b_env.close()


def test_bids_row_rewritten_after_select_is_solved_again():
    """a bids row rewritten after asg_bids_select (EpisodeBatch.update, a slice
    assignment, ...) must be solved as it is at the step, not stepped on the stale assignments.
    The env passes ASG_STEP_USE_SELECTED_BIDS only while the actions tensor's version is the one
    bids_select recorded; the raw C-ABI refuses the flag for a row bids_select did not write."""
    import ctypes

    from marl_sap_amd import _lib
    from marl_sap_amd.envs.assign_env import batch_view
    n, m, E = 16, 24, 32
    env, batch = _env(n, m, E=E, seed=5)
    g = torch.Generator(device="cpu").manual_seed(11)
    q = (torch.randn(E, n, m, generator=g) * 3.0).to(DEV)
    new_bids = (torch.randn(E, n, m, generator=g)).to(DEV)
    row = batch["actions"][:, 0]
    env.bids_select(q, row, 1, 1, 0.0, SEED, 1)
    assert env._bids_flags(batch, 0) == _lib.ASG_STEP_USE_SELECTED_BIDS
    env._bids_token = (row.data_ptr(), tuple(row.stride()), row._version)  # _bids_flags spent it
    batch.update({"actions": new_bids}, ts=0, mark_filled=False)  # rewrites the row in place
    assert env._bids_flags(batch, 0) == 0
    env._bids_token = None
    env.step(batch, 0)
    got = batch["prev_assigns"][:, 1].cpu().numpy()
    nb = batch["actions"][:, 0].cpu().double().numpy()
    assert np.array_equal(nb, new_bids.cpu().double().numpy())
    for e in range(E):
        _, col = ora.lsa(nb[e], maximize=True)
        assert np.array_equal(got[e], col), e
    env.sync()
    # the raw ABI: the flag on a row asg_bids_select did not write is refused (no silent reuse)
    L = _lib.lib()
    env.bids_select(q, batch["actions"][:, 1], 1, 1, 0.0, SEED, 2)
    with torch.cuda.device(env.device):
        rc = L.asg_step_ex(env._h, ctypes.byref(batch_view(batch)), 2, _lib.ASG_STEP_USE_SELECTED_BIDS)
    assert rc == _lib.ASG_E_STATE and "not the row" in _lib.last_error(env._h)
    env.close()


def test_bids_noise_distribution_determinism_sharding():
    n = m = 64
    E, std = 256, 0.3
    env, batch = _env(n, m, E=E)
    q = torch.zeros(E, n, m, device=DEV)
    out = batch["actions"][:, 0]
    env.bids_select(q, out, 1, 1, std, SEED, 9)
    z = (out.double() - 1.0 / n).flatten()  # softmaxes of zeros: 1/m then 1/n
    N = z.numel()
    assert abs(z.mean().item()) < 4 * std / N ** 0.5
    assert abs(z.std().item() / std - 1.0) < 0.01
    first = out.clone()
    env.bids_select(q, out, 1, 1, std, SEED, 9)
    assert torch.equal(out, first)  # same (seed, env, counter): same draws
    env.bids_select(q, out, 1, 1, std, SEED, 10)
    assert not torch.equal(out, first)
    # draws keyed by the global env index: envs 128..255 as their own shard
    h_env, h_batch = _env(n, m, E=128, base=128)
    h_env.bids_select(q[128:], h_batch["actions"][:, 0], 1, 1, std, SEED, 9)
    assert torch.equal(h_batch["actions"][:, 0], first[128:])
    env.close()
    h_env.close()


def test_bids_invalid_entries_raise():
    n, m, E = 16, 16, 8
    env, batch = _env(n, m, E=E)
    q = torch.randn(E, n, m, device=DEV)
    q[3, 2, 5] = float("nan")
    env.bids_select(q, batch["actions"][:, 0], 0, 0, 0.0, SEED, 1)
    env.step(batch, 0)
    with pytest.raises(ValueError, match="invalid numeric entries"):
        env.sync()
    env.close()


def _run(n, m, T, L, E, std, out_type, use_rnn, rng, benefits, fused, episodes=2):
    env_args = dict(n=n, m=m, T=T, L=L, lambda_=0.5, bids_as_actions=True, seed=11, benefits=benefits)
    args = SimpleNamespace(
        batch_size_run=E, env="mock_constellation_env", env_args=env_args, env_rng=rng, env_quirks=(),
        runner_protocol="episode", test_nepisode=1, runner_log_interval=10 ** 12, n=n, m=m, T=T, hidden_dim=64,
        use_rnn=use_rnn, obs_last_action=False, obs_agent_id=False, agent_output_type=out_type,
        action_selector="continuous", softmax_agent_inputs=True, agent="rnn", mac="basic_mac", seed=5,
        epsilon_start=std, epsilon_finish=std, epsilon_anneal_time=1, evaluation_epsilon=0.0, fused_rollout=fused)
    runner = RUN["gpu"](args, _Logger())
    env = runner.get_env()
    torch.manual_seed(321)
    mac = MAC["basic_mac"](env.scheme, {"agents": n}, args)
    mac.to(DEV)
    runner.setup(env.scheme, {"agents": n}, env.preprocess, mac)
    with torch.no_grad():
        mode = mac.fused_mode(env, runner.new_batch())
    assert mode == ("step_q" if fused else None), mode
    out = []
    for _ in range(episodes):
        batch = runner.run(test_mode=False)
        out.append(({k: v.cpu().clone() for k, v in batch.data.transition_data.items()},
                    runner.last_returns.cpu().clone(), mac.hidden_states.detach().cpu().clone()))
    res = out, runner.t_env, list(runner.train_returns)
    env.close()
    return res


@pytest.mark.parametrize("n,m,T,L,E,std,out_type,use_rnn,rng,benefits", [
    (64, 64, 5, 3, 12, 0.3, "pi_logits", False, "philox", "bump"),   # ippo_sap.yaml's agent at configs[2]'s shape
    (20, 25, 5, 3, 9, 0.05, "pi_logits", True, "philox", "bump"),    # the reference's default env, GRU agent
    (16, 16, 4, 2, 8, 0.0, "q", False, "philox", "dense"),           # no noise, no pi_logits softmax
    (20, 25, 4, 3, 6, 0.1, "pi_logits", False, "mt19937", "bump"),   # the same-seed mode's table
])
def test_bids_fused_schedule_is_bit_identical(n, m, T, L, E, std, out_type, use_rnn, rng, benefits):
    a = _run(n, m, T, L, E, std, out_type, use_rnn, rng, benefits, fused=False)
    b = _run(n, m, T, L, E, std, out_type, use_rnn, rng, benefits, fused=True)
    (oa, ta, ra), (ob, tb, rb) = a, b
    assert ta == tb and ra == rb
    for (fa, reta, ha), (fb, retb, hb) in zip(oa, ob):
        for k in fa:
            assert torch.equal(fa[k], fb[k]), k
        assert torch.equal(reta, retb)
        assert torch.equal(ha, hb)
    # the bids are the actions the batch stores: rows 0 .. T-1 filled, each a perturbed
    # probability matrix (softmax over the agents: columns sum to 1 before the noise)
    bids = oa[0][0]["actions"]
    assert bids.shape[-2:] == (n, m) and torch.isfinite(bids).all()
    if std == 0.0:
        assert torch.allclose(bids[:, :T].sum(dim=2), torch.ones(E, T, m), atol=1e-5)
