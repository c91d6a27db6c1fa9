"""Fused RNNAgent inference kernel (asg_rnn_agent_forward, f32 MFMA) against the PyTorch
RNNAgent with the same weights (the reference module, modules/agents/rnn_agent.py:7-31):
fp32 on both sides, only the summation order differs -> agreement to ~1e-6."""
from types import SimpleNamespace

import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():
    pytest.skip("needs a ROCm GPU", allow_module_level=True)

from marl_sap_amd.modules.agents import RNNAgent, RNNFusedAgent  # noqa: E402

DEV = torch.device("cuda", 0)


@pytest.mark.parametrize("R,K,m,use_rnn,hidden", [
    (64 * 256, 256, 64, True, "zero"), (4096 + 37, 256, 64, True, "dense"), (1000, 68, 16, True, "dense"),
    (513, 256, 48, False, "zero"), (2048, 128, 32, False, "dense"), (31, 20, 64, True, "dense"),
    (2000 + 5, 1024, 256, True, "dense"), (777, 512, 128, False, "dense"), (96, 1024, 256, True, "zero"),
    # any input size / n_out: the real envs' obs sizes (70, 490) and m (20, 450), n_out > 256
    (1000, 70, 16, True, "dense"), (517, 490, 450, True, "dense"), (300, 37, 20, False, "dense"),
    (129, 132, 500, True, "zero"), (65, 3, 1, True, "dense"), (200, 130, 512, False, "dense")])
def test_fused_agent_matches_pytorch(R, K, m, use_rnn, hidden):
    torch.manual_seed(R + K)
    args = SimpleNamespace(hidden_dim=64, use_rnn=use_rnn, m=m)
    ref = RNNAgent(K, args).to(DEV)
    fused = RNNFusedAgent(K, args).to(DEV)
    fused.load_state_dict(ref.state_dict())
    x = torch.randn((R, K), device=DEV)
    if hidden == "zero":  # BasicMAC.init_hidden: one zero row expanded over (batch, agents)
        h = ref.init_hidden().unsqueeze(0).expand(R // 64 if R % 64 == 0 else 1, R if R % 64 else 64, -1)
        h = h if h.shape[0] * h.shape[1] == R else torch.zeros((R, 64), device=DEV)
    else:
        h = torch.randn((R, 64), device=DEV) * 0.5
    with torch.no_grad():
        q0, h0 = ref(x, h)
        q1, h1 = fused(x, h)
    torch.testing.assert_close(h1, h0, rtol=1e-5, atol=2e-5)
    torch.testing.assert_close(q1, q0, rtol=1e-5, atol=2e-5)
    # autograd path of the fused module is the PyTorch module itself
    q2, _ = fused(x, h)
    assert q2.requires_grad and torch.equal(q2.detach(), q0)


@pytest.mark.parametrize("R,m,L,use_rnn,mode", [
    (64 * 300, 64, 3, True, "onehot"), (64 * 300 + 40, 64, 3, True, "mixed"), (4096, 64, 3, False, "zeros"),
    (2048 + 17, 256, 3, True, "onehot"), (1500, 128, 2, True, "mixed"), (999, 32, 4, True, "onehot"),
    (800, 64, 3, True, "twos")])
def test_fused_agent_onehot_prefix(R, m, L, use_rnn, mode):
    """Inputs whose first m entries are onehot(previous task) (the mock env's obs): tiles
    verified one-hot add W1[:, a] instead of running the prefix MFMAs; tiles with any other
    prefix (a second 1, a 2, ...) take the full MFMA loop.  Both agree with the PyTorch
    RNNAgent (ragged row counts, zero rows, the L2-read W1^T at m = 256)."""
    torch.manual_seed(R + m)
    K = m * (L + 1)
    args = SimpleNamespace(hidden_dim=64, use_rnn=use_rnn, m=m)
    ref = RNNAgent(K, args).to(DEV)
    fused = RNNFusedAgent(K, args).to(DEV)
    fused.load_state_dict(ref.state_dict())
    x = torch.rand((R, K), device=DEV)
    x[torch.rand((R, K), device=DEV) < 0.7] = 0.0
    a = torch.randint(0, m, (R,), device=DEV)
    x[:, :m] = torch.nn.functional.one_hot(a, m).float()
    if mode == "zeros":
        x[:, :m] = 0.0
    elif mode == "mixed":  # every 7th row is zero, rows 5 and 300 carry a second one, row 77 a 0.5
        x[::7, :m] = 0.0
        x[5, (a[5] + 1) % m] = 1.0
        x[min(300, R - 1), (a[min(300, R - 1)] + 3) % m] = 1.0
        x[77, (a[77] + 2) % m] = 0.5
    elif mode == "twos":
        x[::3, :m] *= 2.0
    h = torch.randn((R, 64), device=DEV) * 0.5
    with torch.no_grad():
        q0, h0 = ref(x, h)
        q1, h1 = fused(x, h)
    torch.testing.assert_close(h1, h0, rtol=1e-5, atol=2e-5)
    torch.testing.assert_close(q1, q0, rtol=1e-5, atol=2e-5)


def test_fused_agent_reads_time_major_obs_slab():
    from marl_sap_amd.components import EpisodeBatch
    from marl_sap_amd.envs import AssignEnvBatch
    E, n, m, T, L = 96, 64, 64, 4, 3
    env = AssignEnvBatch(n, m, T, L, 0.5, num_envs=E, device=DEV)
    b = EpisodeBatch(env.scheme, {"agents": n}, E, T + 1, preprocess=env.preprocess, device=DEV, time_major=True)
    env.reset(b, 0)
    args = SimpleNamespace(hidden_dim=64, use_rnn=True, m=m)
    ref = RNNAgent(m * (L + 1), args).to(DEV)
    fused = RNNFusedAgent(m * (L + 1), args).to(DEV)
    fused.load_state_dict(ref.state_dict())
    x = b["obs"][:, 0].reshape(E * n, -1)
    assert x.data_ptr() == b["obs"][:, 0].data_ptr()  # a view of the slab, no copy
    h = ref.init_hidden().unsqueeze(0).expand(E, n, -1)
    with torch.no_grad():
        q0, _ = ref(x, h)
        q1, _ = fused(x, h)
    torch.testing.assert_close(q1, q0, rtol=1e-5, atol=2e-5)
    assert torch.equal(q1.view(E, n, m).max(2)[1], q0.view(E, n, m).max(2)[1])


@pytest.mark.parametrize("eps,B,n,m,K,use_rnn", [
    (0.0, 300, 64, 64, 256, True), (0.3, 300, 64, 64, 256, True), (0.5, 37, 5, 48, 192, False),
    (0.4, 50, 8, 256, 1024, True), (1.0, 21, 3, 16, 64, True), (0.3, 40, 7, 144, 576, True),
    (0.3, 20, 12, 450, 490, True), (0.5, 30, 9, 20, 70, True), (0.0, 16, 20, 500, 132, False),
    (1.0, 25, 6, 300, 33, True), (0.2, 9, 11, 512, 64, True)])
def test_fused_select_equals_forward_then_selector(eps, B, n, m, K, use_rnn):
    """asg_rnn_agent_select == asg_rnn_agent_forward followed by asg_epsilon_greedy with
    the same Philox (seed, counter): same actions, same hidden state (ragged row counts,
    n_out beyond one 64-task window, random availability)."""
    from marl_sap_amd.action_selectors.classic_selectors import EpsilonGreedyActionSelector
    torch.manual_seed(1)
    args = SimpleNamespace(hidden_dim=64, use_rnn=use_rnn, m=m, epsilon_start=eps, epsilon_finish=eps,
                           epsilon_anneal_time=1, evaluation_epsilon=0.0, seed=5)
    agent = RNNFusedAgent(K, args).to(DEV)
    x = torch.randn((B * n, K), device=DEV)
    h = torch.randn((B * n, 64), device=DEV)
    avail = torch.rand((B, n, m), device=DEV) > (0.2 if m <= 64 else 0.7)
    avail[..., 3] = True
    sel = EpsilonGreedyActionSelector(args)
    with torch.no_grad():
        q, h1 = agent(x, h)
        a1 = sel.select_action(q.view(B, n, m), avail, 0)
        sel2 = EpsilonGreedyActionSelector(args)
        e, seed, counter, status, base = sel2.fused_params(0, False, DEV)
        assert (seed, counter, base) == (sel.seed, sel.calls, 0)
        out = torch.full((B, n), -7, dtype=torch.int64, device=DEV)
        h2 = agent.forward_select(x, h, avail, n, e, seed, counter, out, status)
    assert torch.equal(h2, h1)
    assert torch.equal(out, a1)
    assert int(status.item()) == 0


@pytest.mark.parametrize("fused", [True, False])
def test_select_draws_are_shard_invariant(fused):
    """epsilon > 0: the exploration draws are keyed by global (env, agent) row, so two
    shards (envs [0, B/2) and [B/2, B), env_index_base = 0 and B/2) pick exactly the actions
    of one call over all B envs -- fused agent + selection and the standalone selector."""
    from marl_sap_amd.action_selectors.classic_selectors import EpsilonGreedyActionSelector
    torch.manual_seed(3)
    B, n, m, K, eps = 64, 16, 64, 256, 0.5
    args = SimpleNamespace(hidden_dim=64, use_rnn=True, m=m, epsilon_start=eps, epsilon_finish=eps,
                           epsilon_anneal_time=1, evaluation_epsilon=0.0, seed=11)
    agent = RNNFusedAgent(K, args).to(DEV)
    x = torch.randn((B * n, K), device=DEV)
    h = torch.randn((B * n, 64), device=DEV)
    avail = torch.rand((B, n, m), device=DEV) > 0.3
    avail[..., 0] = True
    half = B // 2

    def run(lo, hi):
        sel = EpsilonGreedyActionSelector(args)
        sel.envs = SimpleNamespace(env_index_base=lo)
        out = torch.full((hi - lo, n), -7, dtype=torch.int64, device=DEV)
        with torch.no_grad():
            if fused:
                e, seed, counter, status, base = sel.fused_params(0, False, DEV)
                agent.forward_select(x[lo * n:hi * n], h[lo * n:hi * n], avail[lo:hi], n, e, seed, counter, out,
                                     status, env_index_base=base)
            else:
                q, _ = agent(x[lo * n:hi * n], h[lo * n:hi * n])
                out = sel.select_action(q.view(hi - lo, n, m), avail[lo:hi], 0)
        return out

    full = run(0, B)
    shards = torch.cat([run(0, half), run(half, B)])
    assert torch.equal(shards, full)
    greedy = torch.zeros_like(full)
    with torch.no_grad():
        q, _ = agent(x, h)
        greedy = q.view(B, n, m).masked_fill(~avail, -float("inf")).max(2)[1]
    frac = (full != greedy).float().mean().item()
    assert 0.2 < frac < 0.6, frac  # about eps * (1 - 1/available) of the rows explore off the argmax


@pytest.mark.parametrize("use_rnn", [True])
def test_split_bf16_gru_is_fp32_accurate(use_rnn):
    """The GRU's products run on three-way-split bf16 MFMAs (asg_rnn_agent_mfma_mode bit 0):
    against a float64 evaluation of the same module, the fused kernel's error is of the
    same size as PyTorch's own fp32 error (not bf16's ~4e-3), for h' and Q."""
    from marl_sap_amd import _lib
    assert _lib.lib().asg_rnn_agent_mfma_mode() & 1
    torch.manual_seed(11)
    R, m, K = 64 * 128, 64, 256
    args = SimpleNamespace(hidden_dim=64, use_rnn=use_rnn, m=m)
    ref = RNNAgent(K, args).to(DEV)
    fused = RNNFusedAgent(K, args).to(DEV)
    fused.load_state_dict(ref.state_dict())
    ref64 = RNNAgent(K, args).to(DEV).double()
    ref64.load_state_dict({k: v.double() for k, v in ref.state_dict().items()})
    x = torch.randn((R, K), device=DEV)
    h = torch.randn((R, 64), device=DEV) * 0.5
    with torch.no_grad():
        q64, h64 = ref64(x.double(), h.double())
        q32, h32 = ref(x, h)
        qf, hf = fused(x, h)
    for got, want, base in ((hf, h64, h32), (qf, q64, q32)):
        err_fused = (got.double() - want).abs().max().item()
        err_torch = (base.double() - want).abs().max().item()
        print(f"max |err| vs float64: fused {err_fused:.3e}, torch fp32 {err_torch:.3e}")
        assert err_fused <= 4 * err_torch + 1e-7, (err_fused, err_torch)
        assert err_fused < 1e-5
