"""SequentialAssignmentProblemSelector on the GPU (reference: action_selectors/
sap_selectors.py:52-98): the fused asg_sap_select kernel (n <= m <= 64) and the torch-noise
+ asg_lsa_batched path for larger problems.

At epsilon = 0 the reference adds exactly zero noise, so the selection is LSA(Q, maximize)
and must match the scipy oracle bit-exactly.  At epsilon > 0 the noise cannot match the
reference's CPU torch stream; its distribution is checked instead: on Q = a*I (2x2) the
assignment flips iff the four N(0, (2*eps*mean|Q|)^2) = N(0, (a*eps)^2) draws sum below
-2a, i.e. with probability Phi(-1/eps).
"""
import math
from types import SimpleNamespace

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # collected on CPU, but never run there
    pytest.skip("needs a ROCm GPU", allow_module_level=True)

from marl_sap_amd.action_selectors.sap_selectors import SequentialAssignmentProblemSelector  # noqa: E402
from oracle import oracle as ora  # noqa: E402

DEV = torch.device("cuda", 0)


def selector(eps, seed=0, base=0):
    args = SimpleNamespace(epsilon_start=eps, epsilon_finish=eps, epsilon_anneal_time=1, evaluation_epsilon=0.0,
                           seed=seed)
    sel = SequentialAssignmentProblemSelector(args)
    sel.envs = SimpleNamespace(env_index_base=base)
    return sel


def sap_like_q(rng, B, n, m):
    """shared per-task profile + small per-agent term: long augmenting paths, many ties"""
    return (rng.normal(size=(B, 1, m)) + 0.05 * rng.normal(size=(B, n, m))).astype(np.float32)


@pytest.mark.parametrize("B,n,m", [(256, 64, 64), (128, 40, 64), (64, 16, 16), (32, 1, 7), (8, 70, 70)])
def test_eps0_is_scipy_lsa(B, n, m):
    rng = np.random.RandomState(n * 100 + m)
    q = sap_like_q(rng, B, n, m)
    sel = selector(0.0)
    out = sel.select_action(torch.as_tensor(q, device=DEV), None, t_env=0).cpu().numpy()
    sel.status.flush()
    assert out.dtype == np.float32 and out.shape == (B, n)
    for b in range(B):
        assert np.array_equal(out[b], ora.lsa(q[b].astype(np.float64), maximize=True)[1].astype(np.float32)), b


def test_test_mode_uses_evaluation_epsilon():
    rng = np.random.RandomState(1)
    q = torch.as_tensor(sap_like_q(rng, 64, 32, 48), device=DEV)
    sel = selector(0.9)
    out = sel.select_action(q, None, t_env=0, test_mode=True).cpu().numpy()
    for b in range(64):
        assert np.array_equal(out[b], ora.lsa(q[b].cpu().numpy().astype(np.float64), maximize=True)[1]), b


def test_noise_is_keyed_and_a_valid_assignment():
    rng = np.random.RandomState(2)
    q = torch.as_tensor(sap_like_q(rng, 512, 64, 64), device=DEV)
    a, b = selector(0.5, seed=7), selector(0.5, seed=7)
    o1, o2 = a.select_action(q, None, 0), b.select_action(q, None, 0)
    assert torch.equal(o1, o2)                      # same (seed, env, call) -> same draws
    o3 = a.select_action(q, None, 0)                # next call: fresh noise
    assert not torch.equal(o1, o3)
    s = torch.sort(o1.long(), dim=1)[0]
    assert torch.equal(s, torch.arange(64, device=DEV).expand(512, 64))  # a permutation per env
    # sharding: envs 256..511 of a base-0 call == a base-256 call on those rows alone
    c, d = selector(0.5, seed=7), selector(0.5, seed=7, base=256)
    full, half = c.select_action(q, None, 0), d.select_action(q[256:], None, 0)
    assert torch.equal(full[256:], half)


@pytest.mark.parametrize("eps", [0.5, 1.0])
def test_noise_scale_flip_probability(eps):
    B, a = 200_000, 3.0
    q = torch.zeros((B, 2, 2), device=DEV)
    q[:, 0, 0] = a
    q[:, 1, 1] = a
    out = selector(eps, seed=11).select_action(q, None, 0)
    p = (out[:, 0] == 1).float().mean().item()
    expect = 0.5 * math.erfc(1.0 / eps / math.sqrt(2.0))   # Phi(-1/eps)
    sd = math.sqrt(expect * (1 - expect) / B)
    assert abs(p - expect) < 6 * sd, (p, expect)


def test_invalid_entries_raise_on_flush():
    q = torch.randn((4, 8, 8), device=DEV)
    q[1, 3, 3] = float("nan")
    q[2, 0, 5] = float("inf")                        # -inf once negated for maximize
    sel = selector(0.0)
    out = sel.select_action(q, None, 0)
    assert (out[1] == -1).all() and (out[2] == -1).all() and (out[0] >= 0).all()
    with pytest.raises(ValueError, match="invalid numeric entries"):
        sel.status.flush()


def _sap_raw(q, eps, seed, counter, base=0):
    """asg_sap_select through the C-ABI: (actions, status, augmenting-path steps)"""
    import ctypes
    from marl_sap_amd import _lib
    B, n, m = q.shape
    out = torch.empty((B, n), dtype=torch.float32, device=DEV)
    st = torch.empty((B,), dtype=torch.int32, device=DEV)
    steps = torch.zeros((B,), dtype=torch.int32, device=DEV)
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    _lib.check(_lib.lib().asg_sap_select(p(q), _lib.i64arr(q.stride()), B, n, m, float(eps), seed, counter, base,
                                         p(out), p(st), p(steps), _lib.stream_ptr(DEV)))
    torch.cuda.synchronize()
    return out, st, steps


def _noisy(q, eps, seed, counter, base=0):
    """asg_sap_noise: the matrix the selector solves for these arguments"""
    import ctypes
    from marl_sap_amd import _lib
    B, n, m = q.shape
    out = torch.empty((B, n, m), dtype=torch.float32, device=DEV)
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    _lib.check(_lib.lib().asg_sap_noise(p(q), _lib.i64arr(q.stride()), B, n, m, float(eps), seed, counter, base,
                                        p(out), None, _lib.stream_ptr(DEV)))
    return out


@pytest.mark.parametrize("B,n,m,eps,kind", [
    (2048, 64, 64, 0.05, "sap"),     # configs[2]'s SAP selection: the certified fast path
    (2048, 64, 64, 0.0, "sap"),
    (1024, 64, 64, 1.0, "sap"),
    (1024, 64, 64, 0.05, "uniform"),
    (1024, 16, 16, 0.3, "sap"),      # configs[1]'s shape
    (1024, 33, 33, 0.2, "uniform"),  # odd square size (padding lanes)
    (1024, 20, 25, 0.2, "sap"),      # rectangular: the scipy-exact solver alone
])
def test_sap_noisy_selection_is_scipy(B, n, m, eps, kind):
    """At epsilon > 0 the selection equals scipy's LSA(maximize) of exactly the noisy matrix
    the kernel formed (asg_sap_noise), env by env -- whichever solver ran (the certified fast
    path for square problems, the scipy-exact one otherwise)."""
    rng = np.random.RandomState(B + n + m)
    q = sap_like_q(rng, B, n, m) if kind == "sap" else rng.rand(B, n, m).astype(np.float32)
    qd = torch.as_tensor(q, device=DEV)
    out, st, steps = _sap_raw(qd, eps, 5, 3, base=100)
    noisy = _noisy(qd, eps, 5, 3, base=100).cpu().numpy()
    out, st, steps = out.cpu().numpy(), st.cpu().numpy(), steps.cpu().numpy()
    assert (st == 0).all()
    for b in range(B):
        assert np.array_equal(out[b], ora.lsa(noisy[b].astype(np.float64), maximize=True)[1].astype(np.float32)), b
    fast, exact = steps & 0xFFFF, steps >> 16
    if n == m:
        assert (fast > 0).all()
        assert (exact == 0).mean() > 0.95, (exact > 0).mean()  # almost every problem certified
    else:
        assert (fast == 0).all() and (exact > 0).all()


def test_sap_fast_path_falls_back_on_ties():
    """Square problems with exact ties (integer Q: several optimal assignments) fail the
    uniqueness certificate and take the scipy-exact solver: scipy's tie rule is kept."""
    rng = np.random.RandomState(9)
    B, n = 512, 64
    q = rng.randint(0, 4, size=(B, n, n)).astype(np.float32)
    q[: B // 2] += rng.randint(0, 3, size=(B // 2, 1, n)).astype(np.float32)
    out, st, steps = _sap_raw(torch.as_tensor(q, device=DEV), 0.0, 1, 1)
    out, steps = out.cpu().numpy(), steps.cpu().numpy()
    for b in range(B):
        assert np.array_equal(out[b], ora.lsa(q[b].astype(np.float64), maximize=True)[1].astype(np.float32)), b
    assert ((steps >> 16) > 0).mean() > 0.9  # ties: the exact solver ran


def test_sap_fast_path_full_size():
    """configs[2]'s selection size, 16,384 envs of 64 x 64 at epsilon 0.05: every env equals
    scipy on its noisy matrix (oracle, C), and the fast path's step count is reported."""
    rng = np.random.RandomState(77)
    B = 16384
    q = torch.as_tensor(sap_like_q(rng, B, 64, 64), device=DEV)
    out, st, steps = _sap_raw(q, 0.05, 2, 7)
    noisy = _noisy(q, 0.05, 2, 7).cpu().numpy()
    out, steps = out.cpu().numpy(), steps.cpu().numpy()
    assert (st.cpu().numpy() == 0).all()
    for b in range(B):
        col = ora.lsa(noisy[b].astype(np.float64), maximize=True)[1]
        assert np.array_equal(out[b], col.astype(np.float32)), b
    assert ((steps >> 16) == 0).mean() > 0.99


@pytest.mark.parametrize("gap_log2,expect", [(-40, "fallback"), (-30, "fallback"), (-23, "any"), (-20, "certified")])
def test_sap_fast_path_planted_near_tie(gap_log2, expect):
    """A second assignment planted at a small cost gap from the unique optimum: rows i1, i2 can
    only take columns i1, i2 (every other entry of theirs is -10; every other row prefers its
    own diagonal by ~9), and Q[i2, i1] = base - gap makes the swap worse by exactly `gap`
    (base = 2^-22: ulp 2^-45, so the gap is exact in float32).  With S (max|c| + max|u| +
    max|v|) of order 2^4..2^5, gaps 2^-40 (~S 2^-45) and 2^-30 (~S 2^-35) leave both swap
    edges near-tight (<= S 2^-30): the certificate must refuse and the scipy-exact solver run;
    2^-20 (~S 2^-25) must certify; 2^-23 sits just above the threshold band.  Every problem
    equals scipy's assignment (the C oracle)."""
    rng = np.random.RandomState(1000 - gap_log2)
    B, n = 256, 64
    q = (rng.uniform(-1.0, 1.0, size=(B, n, n)) + 10.0 * np.eye(n)).astype(np.float32)
    base, gap = np.float32(2.0 ** -22), 2.0 ** gap_log2
    for b in range(B):
        i1, i2 = rng.choice(n, 2, replace=False)
        q[b, [i1, i2], :] = -10.0
        q[b, :, [i1, i2]] = np.minimum(q[b, :, [i1, i2]], -10.0)
        q[b, i1, i1] = q[b, i2, i2] = q[b, i1, i2] = base
        q[b, i2, i1] = np.float32(float(base) - gap)
        assert float(q[b, i1, i1]) + float(q[b, i2, i2]) - float(q[b, i1, i2]) - float(q[b, i2, i1]) == gap
    out, st, steps = _sap_raw(torch.as_tensor(q, device=DEV), 0.0, 1, 1)
    out, st, steps = out.cpu().numpy(), st.cpu().numpy(), steps.cpu().numpy()
    assert (st == 0).all()
    for b in range(B):
        assert np.array_equal(out[b], ora.lsa(q[b].astype(np.float64), maximize=True)[1].astype(np.float32)), b
    exact = steps >> 16
    if expect == "fallback":
        assert (exact > 0).all(), (exact == 0).sum()
    elif expect == "certified":
        assert (exact == 0).all(), (exact > 0).sum()


def _sap_warm(q, eps, seed, counter, duals, warm):
    """asg_sap_select_warm through the C-ABI: (int64 actions, status, steps)"""
    import ctypes
    from marl_sap_amd import _lib
    B, n, m = q.shape
    out = torch.empty((B, n), dtype=torch.int64, device=DEV)
    st = torch.zeros((B,), dtype=torch.int32, device=DEV)
    steps = torch.zeros((B,), dtype=torch.int32, device=DEV)
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    _lib.check(_lib.lib().asg_sap_select_warm(p(q), _lib.i64arr(q.stride()), B, n, m, float(eps), seed, counter, 0,
                                              p(out), p(st), p(steps), p(duals), int(warm), _lib.stream_ptr(DEV)))
    torch.cuda.synchronize()
    return out, st, steps


@pytest.mark.parametrize("eps,n", [(0.0, 64), (0.05, 64), (0.3, 64), (0.05, 33)])
def test_sap_warm_start_episodes_are_scipy(eps, n):
    """Whole warm-started episodes: T = 20 consecutive selections per env on SAP-like Q that
    changes a little from step to step (each selection starting from the env's previous column
    duals) equal scipy's LSA of exactly the noisy matrix the kernel formed, step by step (and the
    cold selection's assignment); at small epsilon the warm start takes fewer augmenting-path
    steps than the cold one on the same calls."""
    rng = np.random.RandomState(int(eps * 100) + n)
    B, T = 512, 20
    base = sap_like_q(rng, B, n, n)
    duals = torch.empty((B, 64), dtype=torch.float64, device=DEV)
    warm_steps = cold_steps = 0
    for t in range(T):
        q = (base + 0.01 * rng.normal(size=(B, n, n))).astype(np.float32)  # the next step's Q: a small change
        qd = torch.as_tensor(q, device=DEV)
        out, st, steps = _sap_warm(qd, eps, 4, t + 1, duals, warm=t > 0)
        ref_out, _, ref_steps = _sap_raw(qd, eps, 4, t + 1)
        noisy = _noisy(qd, eps, 4, t + 1).cpu().numpy()
        out, st = out.cpu().numpy(), st.cpu().numpy()
        assert (st == 0).all()
        np.testing.assert_array_equal(out, ref_out.cpu().numpy().astype(np.int64))
        for b in range(0, B, 7):
            assert np.array_equal(out[b], ora.lsa(noisy[b].astype(np.float64), maximize=True)[1]), (t, b)
        if t > 0:
            warm_steps += int((steps & 0xFFFF).sum().item()) + int((steps >> 16).sum().item())
            cold_steps += int((ref_steps & 0xFFFF).sum().item()) + int((ref_steps >> 16).sum().item())
        assert torch.isfinite(duals[:, :n]).all()  # the next call's warm start
    if eps <= 0.05:  # small changes between calls: fewer augmenting-path steps (0.47x at eps 0 on GPU)
        assert warm_steps < cold_steps, (warm_steps, cold_steps)


def test_sap_warm_start_ignores_garbage_duals():
    """Any duals -- NaN (cold start), huge, or another problem's -- give scipy's assignment."""
    rng = np.random.RandomState(5)
    B, n = 256, 64
    qd = torch.as_tensor(sap_like_q(rng, B, n, n), device=DEV)
    ref = _sap_raw(qd, 0.05, 9, 2)[0].cpu().numpy().astype(np.int64)
    for fill in (float("nan"), 1e30, -3.0):
        duals = torch.full((B, 64), fill, dtype=torch.float64, device=DEV)
        duals[::2] = torch.as_tensor(rng.normal(size=(B // 2, 64)) * 5, device=DEV)
        out, st, _ = _sap_warm(qd, 0.05, 9, 2, duals, warm=1)
        assert (st.cpu().numpy() == 0).all()
        np.testing.assert_array_equal(out.cpu().numpy(), ref)
