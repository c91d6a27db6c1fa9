"""Parity checker: replays a GPU rollout on the CPU oracle (TEST INFRASTRUCTURE ONLY).

Given what the HIP env produced for E envs (the benefit table it used, its initial
prev_assigns, the actions it stepped and the EpisodeBatch rows it wrote), re-run every
env through OracleMockEnv (mock_constellation_env.py semantics) and compare:
  integer fields (actions_onehot, avail_actions, filled, terminated, prev_assigns) exact,
  float32 fields (obs, beta, rewards) exact against float32(oracle float64) -- the GPU
  computes the same float64 expressions -- and float64 returns within 1e-9 relative.
"""
import numpy as np

from . import oracle as ora

# Philox mode: float32 bump values vs float32 of their float64 evaluation: the
# kernel's error is <= 1.5 2^-23 of the bump's task scale (<= 10) at every time, plus the float32
# rounding of the value itself; v_exp_f32 flushes results below FLT_MIN (2^-126) to 0
PHILOX_RTOL = 2.0 ** -22
PHILOX_ATOL = 10.0 * 2.0 ** -22


def replay_and_compare(n, m, T, L, lam, table, prev0, td, returns, T_trans=None, quirks=(),
                       rtol_reward=0.0, obs_atol=0.0, philox=False):
    """table [E,n,m,T] f64, prev0 [E,n] i64, td: dict of numpy arrays [E, T+1, ...] read
    back from the GPU batch, returns [E] f64.  Raises AssertionError on any mismatch.

    philox=True (native Philox mode): `table` is the float64 evaluation of the episode's
    bump parameters (asg_export_benefits) while obs / beta hold the kernel's float32
    evaluation of the same bumps, checked within 2^-22 of the largest task scale plus 2^-22
    relative (csrc/asg_device.h bump32_at); rewards, masks, one-hots and returns stay exact."""
    E = table.shape[0]
    obs_rtol = PHILOX_RTOL if philox else 0.0
    if philox:
        obs_atol = max(obs_atol, PHILOX_ATOL)
    for e in range(E):
        env = ora.OracleMockEnv(n, m, T, L, lam, sat_prox_mat=table[e], T_trans=T_trans, mt=ora.MT(0))
        env.reset()
        env.prev_assigns[:] = prev0[e]
        _cmp(td["obs"][e, 0], env._obs.astype(np.float32), f"env {e} obs row 0", obs_atol, obs_rtol)
        _cmp(td["beta"][e, 0], env.beta.astype(np.float32), f"env {e} beta row 0", obs_atol, obs_rtol)
        ret = 0.0
        for t in range(T):
            a = td["actions"][e, t].reshape(n).astype(np.int64)
            r, done, _ = env.step(a)
            ret += sum(r)
            _cmp(td["rewards"][e, t], np.asarray(r).astype(np.float32), f"env {e} rewards t={t}",
                 rtol=rtol_reward)
            _cmp(td["obs"][e, t + 1], env._obs.astype(np.float32), f"env {e} obs t={t + 1}", obs_atol, obs_rtol)
            _cmp(td["beta"][e, t + 1], env.beta.astype(np.float32), f"env {e} beta t={t + 1}", obs_atol, obs_rtol)
            onehot = np.zeros((n, m), dtype=np.int64)
            onehot[np.arange(n), a] = 1
            if "actions_onehot" in td:
                _cmp(td["actions_onehot"][e, t], onehot, f"env {e} onehot t={t}")
            term = bool(done) if "parallel_terminated" not in quirks else (e != 0)
            assert bool(td["terminated"][e, t, 0]) == term, f"env {e} terminated t={t}"
            pa = np.zeros(n, np.int64) if "prev_assigns_zero" in quirks else a
            _cmp(td["prev_assigns"][e, t + 1], pa, f"env {e} prev_assigns t={t + 1}")
        assert td["avail_actions"][e].all(), f"env {e} avail_actions"
        assert (td["filled"][e] == 1).all(), f"env {e} filled"
        assert abs(returns[e] - ret) <= 1e-9 * max(1.0, abs(ret)), f"env {e} return {returns[e]} vs {ret}"


def bump_table_from_params(params, T):
    """float64 benefit table [E, n, m, T] from Philox bump parameters [E, n, m, 3]
    (scale, center, a2) as asg_export_bump_params returns them: the reference's
    scale * exp(-(t - c)^2 / sigma_2 / 2) (mock_constellation_env.py:293) evaluated in
    float64 on those parameters, written scale * 2^(-(t - c)^2 a2), a2 = log2(e) / (2 sigma_2)."""
    p = np.asarray(params, dtype=np.float64)
    x = np.arange(T, dtype=np.float64)[None, None, None, :] - p[..., 1:2]
    return p[..., 0:1] * np.exp2(-(x * x) * p[..., 2:3])


def _cmp(got, want, what, atol=0.0, rtol=0.0):
    got = np.asarray(got).reshape(np.asarray(want).shape)
    if atol == 0.0 and rtol == 0.0:
        if not np.array_equal(got, want):
            bad = np.argwhere(got != want)
            i = tuple(bad[0])
            raise AssertionError(f"{what}: {len(bad)} mismatches, first at {i}: {got[i]!r} vs {want[i]!r}")
    else:
        np.testing.assert_allclose(got, want, rtol=rtol, atol=atol, err_msg=what)


# ---- exhaustive replay (oracle/asg_check.c): every env of a GPU batch -------------------------
import ctypes  # noqa: E402


class _CheckCfg(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int), ("m", ctypes.c_int), ("T", ctypes.c_int), ("L", ctypes.c_int),
                ("lambda_", ctypes.c_double), ("quirks", ctypes.c_int), ("obs_atol", ctypes.c_double),
                ("obs_rtol", ctypes.c_double), ("reward_rtol", ctypes.c_double), ("env_index0", ctypes.c_int64),
                ("seed_check", ctypes.c_int), ("seed", ctypes.c_uint32), ("seed_rtol", ctypes.c_double)]


def _check_lib():
    L = ora.lib()
    if not hasattr(L, "_chk_ready"):
        vp = ctypes.c_void_p
        L.ora_check_rollout.argtypes = [ctypes.POINTER(_CheckCfg), ctypes.c_int] + [vp] * 12 + \
            [ctypes.c_int, ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(ctypes.c_longlong)]
        L.ora_check_rollout.restype = ctypes.c_int
        L._chk_ready = True
    return L


def check_threads():
    """Worker threads for the checker: the box's CPU share (16 per GPU), not os.cpu_count()."""
    import os
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    return max(1, min(16, avail))


def replay_all(n, m, T, L, lam, td, table, prev0, returns, quirks=(), philox=False, rtol_reward=0.0,
               seed=None, env_chunk=None, threads=None):
    """Replay EVERY env of a GPU batch on the oracle in C (asg_check.c), chunk by chunk.

    td: the batch's transition tensors ({name: torch tensor [E, T+1, ...]} on the GPU, any layout);
    table: torch float64 [E, n, m, T] (asg_export_benefits: the values the kernel used; in the Philox
    mode its float64 evaluation of the bump parameters); prev0 [E, n] int64; returns [E] float64.
    philox: obs / beta within the Philox float32 bump tolerance (PHILOX_ATOL / RTOL), else exact.
    seed: the MT19937 same-seed mode -- every env's table (rtol 1e-12) and reset permutation are
    also rebuilt from np.random.seed(seed + env).  Returns (envs checked, values compared); raises
    AssertionError naming the first mismatch."""
    import numpy as _np
    E = int(table.shape[0])
    W = m * (L + 1)
    if env_chunk is None:  # ~3 GiB of float32 obs per chunk
        env_chunk = max(1, min(E, (3 << 30) // (4 * (T + 1) * n * W)))
    cfg = _CheckCfg(n, m, T, L, float(lam),
                    (1 if "prev_assigns_zero" in quirks else 0) | (2 if "parallel_terminated" in quirks else 0),
                    PHILOX_ATOL if philox else 0.0, PHILOX_RTOL if philox else 0.0, float(rtol_reward), 0,
                    1 if seed is not None else 0, 0 if seed is None else int(seed) & 0xFFFFFFFF, 1e-12)
    lib_ = _check_lib()
    threads = threads or check_threads()
    compared = 0

    def host(t, dtype):
        return _np.ascontiguousarray(t.contiguous().cpu().numpy(), dtype=dtype)

    for e0 in range(0, E, env_chunk):
        e1 = min(E, e0 + env_chunk)
        cfg.env_index0 = e0
        arr = {
            "table": host(table[e0:e1], _np.float64), "prev0": host(prev0[e0:e1], _np.int64),
            "obs": host(td["obs"][e0:e1], _np.float32), "beta": host(td["beta"][e0:e1], _np.float32),
            "actions": host(td["actions"][e0:e1], _np.int64), "rewards": host(td["rewards"][e0:e1], _np.float32),
            "onehot": host(td["actions_onehot"][e0:e1], _np.int64) if "actions_onehot" in td else None,
            "term": host(td["terminated"][e0:e1], _np.uint8), "prevb": host(td["prev_assigns"][e0:e1], _np.int64),
            "avail": host(td["avail_actions"][e0:e1], _np.uint8), "filled": host(td["filled"][e0:e1], _np.int64),
            "returns": host(returns[e0:e1], _np.float64)}
        msg = ctypes.create_string_buffer(512)
        cnt = ctypes.c_longlong(0)
        ptr = lambda a: None if a is None else a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
        fails = lib_.ora_check_rollout(
            ctypes.byref(cfg), e1 - e0, ptr(arr["table"]), ptr(arr["prev0"]), ptr(arr["obs"]), ptr(arr["beta"]),
            ptr(arr["actions"]), ptr(arr["rewards"]), ptr(arr["onehot"]), ptr(arr["term"]), ptr(arr["prevb"]),
            ptr(arr["avail"]), ptr(arr["filled"]), ptr(arr["returns"]), threads, msg, 512, ctypes.byref(cnt))
        assert fails == 0, f"{fails} of envs {e0}..{e1 - 1} differ from the oracle replay; first: {msg.value.decode()}"
        compared += cnt.value
        del arr
    return E, compared
