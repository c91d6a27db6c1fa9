"""ctypes front-end of the CPU ORACLE (test infrastructure only).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this
module.  The product (marl_sap_amd) never does: its HIP path must stand on its own and
fails loudly without its extension.

`OracleMockEnv` follows MockConstellationEnv (src/envs/mock_constellation_env.py:13-274)
call for call, with the arithmetic done by asg_oracle.c; `lsa` follows scipy's
linear_sum_assignment including its error messages.
Pinned by tests/test_oracle_golden.py against tests/golden/*.npz.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libasg_oracle.so")
_lib = None

_dp = ctypes.POINTER(ctypes.c_double)
_i64p = ctypes.POINTER(ctypes.c_int64)


def build():
    """Compile the oracle (gcc; used by __graft_entry__.build and the test fixtures)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.ora_mt_sizeof.restype = ctypes.c_size_t
        L.ora_mt_seed.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
        L.ora_mt_next.argtypes = [ctypes.c_void_p]
        L.ora_mt_next.restype = ctypes.c_uint32
        L.ora_mt_double.argtypes = [ctypes.c_void_p]
        L.ora_mt_double.restype = ctypes.c_double
        L.ora_mt_uniform.argtypes = [ctypes.c_void_p, ctypes.c_double, ctypes.c_double]
        L.ora_mt_uniform.restype = ctypes.c_double
        L.ora_mt_permutation.argtypes = [ctypes.c_void_p, ctypes.c_int, _i64p]
        L.ora_mt_drawn.argtypes = [ctypes.c_void_p]
        L.ora_mt_drawn.restype = ctypes.c_uint64
        L.ora_mt_get_state.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint32),
                                       ctypes.POINTER(ctypes.c_int)]
        L.ora_generate.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                   ctypes.c_double, ctypes.c_double, _dp]
        L.ora_beta_hat.argtypes = [_dp, _i64p, ctypes.c_int, ctypes.c_int, _dp, ctypes.c_double, _dp]
        L.ora_lsa.argtypes = [_dp, ctypes.c_int, ctypes.c_int, ctypes.c_int, _i64p, _i64p]
        L.ora_lsa.restype = ctypes.c_int
        L.ora_env_construct_reset.argtypes = [ctypes.c_void_p] + [ctypes.c_int] * 5 + \
            [_dp, _dp, _i64p, _dp, _dp]
        L.ora_env_construct_reset.restype = ctypes.c_int
        L.ora_env_reset.argtypes = [ctypes.c_void_p] + [ctypes.c_int] * 5 + [_dp, _i64p, _dp, _dp]
        L.ora_env_reset.restype = ctypes.c_int
        L.ora_env_step.argtypes = [ctypes.c_int] * 4 + [ctypes.c_double, _dp, _dp,
                                                        ctypes.POINTER(ctypes.c_int), _dp, _i64p,
                                                        _i64p, _dp, _dp, _dp]
        L.ora_env_step.restype = ctypes.c_int
        L.ora_rollout_random.argtypes = [ctypes.c_int] * 5 + [ctypes.c_double, ctypes.c_uint32,
                                                              ctypes.c_int, ctypes.c_int, _dp]
        L.ora_rollout_random.restype = ctypes.c_double
        ci = ctypes.c_int
        L.ora_real_obs_size.argtypes = [ci, ci, ci]
        L.ora_real_obs_size.restype = ci
        L.ora_real_beta.argtypes = [_dp, _dp, ci, ci, ci, ci, ci, _dp]
        L.ora_real_obs.argtypes = [_dp, ci, ci, ci, ci, ci, _i64p, ci, _dp]
        L.ora_real_reset.argtypes = [_dp, _dp, ci, ci, ci, ci, ci, ci, _dp, _i64p, _dp]
        L.ora_real_step.argtypes = [_dp, _dp, _dp, ci, ci, ci, ci, ci, ci, ctypes.c_double,
                                    ctypes.POINTER(ci), _dp, _i64p, _i64p, _dp, ctypes.POINTER(ci), _dp]
        L.ora_realx_obs_size.argtypes = [ci, ci, ci, ci]
        L.ora_realx_obs_size.restype = ci
        L.ora_realx_reset.argtypes = [ci, _dp, _dp, ci, ci, ci, ci, ci, ci, _i64p, _dp, _i64p, _dp, _dp]
        L.ora_realx_step.argtypes = [ci, _dp, _dp, _dp, ctypes.POINTER(ci), _dp, ci, ci, ci, ci, ci, ci,
                                     ctypes.c_double, ctypes.POINTER(ci), _dp, _i64p, _dp, _i64p, _dp,
                                     ctypes.POINTER(ci), _dp]
        _lib = L
    return _lib


def _p(a, t):
    return None if a is None else a.ctypes.data_as(t)


class MT:
    """numpy legacy RandomState stream (np.random.seed(s) then draws)."""

    def __init__(self, seed):
        self._buf = ctypes.create_string_buffer(lib().ora_mt_sizeof())
        lib().ora_mt_seed(self._buf, ctypes.c_uint32(seed))

    @property
    def ptr(self):
        return self._buf

    def next32(self, k=1):
        return np.array([lib().ora_mt_next(self._buf) for _ in range(k)], dtype=np.uint32)

    def rand(self):
        return lib().ora_mt_double(self._buf)

    def uniform(self, lo, hi):
        return lib().ora_mt_uniform(self._buf, lo, hi)

    def permutation(self, m):
        out = np.empty(m, dtype=np.int64)
        lib().ora_mt_permutation(self._buf, m, _p(out, _i64p))
        return out

    def drawn(self):
        """32-bit words consumed since seeding."""
        return int(lib().ora_mt_drawn(self._buf))

    def state(self):
        key = (ctypes.c_uint32 * 624)()
        pos = ctypes.c_int()
        lib().ora_mt_get_state(self._buf, key, ctypes.byref(pos))
        return np.frombuffer(key, dtype=np.uint32).copy(), pos.value


def generate(mt, n, m, T, wmin, wmax):
    """generate_benefits_over_time (mock_constellation_env.py:276-299)."""
    out = np.empty((n, m, T), dtype=np.float64)
    lib().ora_generate(mt.ptr, n, m, T, wmin, wmax, _p(out, _dp))
    return out


def beta_hat(beta, prev, lam, T_trans=None):
    """MockConstellationEnv.beta_hat for [n,m] or [t,n,m] beta (mock :228-274)."""
    beta = np.ascontiguousarray(beta, dtype=np.float64)
    prev = np.ascontiguousarray(prev, dtype=np.int64)
    squeeze = beta.ndim == 2
    if squeeze:
        beta, prev = beta[None], prev[None]
    t, n, m = beta.shape
    tt = None if T_trans is None else np.ascontiguousarray(T_trans, dtype=np.float64)
    out = np.empty_like(beta)
    for k in range(t):
        lib().ora_beta_hat(_p(beta[k], _dp), _p(prev[k], _i64p), n, m, _p(tt, _dp), lam,
                           _p(out[k], _dp))
    return out[0] if squeeze else out


def lsa(C, maximize=False):
    """scipy.optimize.linear_sum_assignment restatement -> (row_ind, col_ind)."""
    C = np.asarray(C)
    if C.ndim != 2:
        raise ValueError("expected a matrix (2-D array), got a %r array" % (C.shape,))
    C = np.ascontiguousarray(C, dtype=np.float64)
    nr, nc = C.shape
    k = min(nr, nc)
    row = np.empty(k, dtype=np.int64)
    col = np.empty(k, dtype=np.int64)
    st = lib().ora_lsa(_p(C, _dp), nr, nc, int(bool(maximize)), _p(row, _i64p), _p(col, _i64p))
    if st == -1:
        raise ValueError("matrix contains invalid numeric entries")
    if st == -2:
        raise ValueError("cost matrix is infeasible")
    return row, col


class OracleMockEnv:
    """MockConstellationEnv on the C oracle.  `mt` plays numpy's global stream."""

    def __init__(self, n, m, T, L, lambda_, bids_as_actions=False, seed=None,
                 sat_prox_mat=None, T_trans=None, mt=None):
        self.n, self.m, self.T, self.L, self.lambda_ = n, m, T, L, lambda_
        self.bids_as_actions = bool(bids_as_actions)
        self.mt = mt if mt is not None else MT(0 if seed is None else seed)
        self.constant_benefits = sat_prox_mat is not None
        if self.constant_benefits:
            self.sat_prox_mat = np.ascontiguousarray(sat_prox_mat, dtype=np.float64)
        else:
            self.sat_prox_mat = generate(self.mt, n, m, T, 5.0, 8.0)          # :34
        self.T_trans = None if T_trans is None else np.ascontiguousarray(T_trans, np.float64)
        self.k = 0

    def reset(self):
        n, m, T, L = self.n, self.m, self.T, self.L
        self.prev_assigns = np.empty(n, dtype=np.int64)
        self._obs = np.empty((n, m * (L + 1)), dtype=np.float64)
        self.beta = np.empty((n, m), dtype=np.float64)
        if not self.constant_benefits:
            self.sat_prox_mat = np.empty((n, m, T), dtype=np.float64)
        st = lib().ora_env_reset(self.mt.ptr, n, m, T, L, int(self.constant_benefits),
                                 _p(self.sat_prox_mat, _dp), _p(self.prev_assigns, _i64p),
                                 _p(self._obs, _dp), _p(self.beta, _dp))
        if st != 0:
            raise ValueError("Cannot take a larger sample than population when 'replace=False'")
        self.k = 0
        return self._obs

    def step(self, actions):
        n, m = self.n, self.m
        rewards = np.empty(n, dtype=np.float64)
        k = ctypes.c_int(self.k)
        if self.bids_as_actions:
            bids = np.ascontiguousarray(actions, dtype=np.float64).reshape(n, m)
            acts = None
        else:
            acts = np.ascontiguousarray(np.asarray(actions, dtype=np.int64).reshape(n))
            bids = None
        obs = np.empty_like(self._obs)
        st = lib().ora_env_step(n, m, self.T, self.L, self.lambda_, _p(self.sat_prox_mat, _dp),
                                _p(self.T_trans, _dp), ctypes.byref(k), _p(self.beta, _dp),
                                _p(self.prev_assigns, _i64p), _p(acts, _i64p), _p(bids, _dp),
                                _p(rewards, _dp), _p(obs, _dp))
        if st < 0:
            raise ValueError("matrix contains invalid numeric entries" if st == -1
                             else "cost matrix is infeasible")
        self.k = k.value
        self._obs = obs
        return list(rewards), bool(st), {}

    def get_pretransition_data(self):
        return {"obs": [self._obs], "avail_actions": [[[1] * self.m] * self.n],
                "beta": [self.beta]}

    def beta_hat(self, beta, prev_assigns):
        return beta_hat(np.asarray(beta), np.asarray(prev_assigns), self.lambda_, self.T_trans)


class OracleRealEnv:
    """RealConstellationEnv with injected benefits (src/envs/real_constellation_env.py,
    constant-benefit path), arithmetic in asg_real_oracle.c; argsort ties resolved in the
    stable (lower index first) order."""

    def __init__(self, sat_prox_mat, N, M, L, lambda_, T_trans=None, task_prios=None):
        self.table = np.ascontiguousarray(sat_prox_mat, dtype=np.float64)
        self.n, self.m, self.T = self.table.shape
        self.N, self.M, self.L, self.lambda_ = N, M, min(L, self.T), float(lambda_)
        self.T_trans = np.ascontiguousarray(
            T_trans if T_trans is not None else np.ones((self.m, self.m)) - np.eye(self.m), dtype=np.float64)
        self.prios = np.ascontiguousarray(task_prios if task_prios is not None else np.ones(self.m),
                                          dtype=np.float64)
        self.obs_size = lib().ora_real_obs_size(N, M, self.L)

    def reset(self):
        self.k = 0
        self.done = False
        self.beta = np.empty((self.n, self.m, self.L))
        self.prev_assigns = np.empty(self.n, dtype=np.int64)
        self.obs = np.empty((self.n, self.obs_size))
        lib().ora_real_reset(_p(self.table, _dp), _p(self.prios, _dp), self.n, self.m, self.T, self.L, self.N,
                             self.M, _p(self.beta, _dp), _p(self.prev_assigns, _i64p), _p(self.obs, _dp))
        return self.obs

    def step(self, actions):
        a = np.ascontiguousarray(actions, dtype=np.int64)
        rewards = np.empty(self.n)
        k, done = ctypes.c_int(self.k), ctypes.c_int(0)
        lib().ora_real_step(_p(self.table, _dp), _p(self.prios, _dp), _p(self.T_trans, _dp), self.n, self.m,
                            self.T, self.L, self.N, self.M, self.lambda_, ctypes.byref(k), _p(self.beta, _dp),
                            _p(self.prev_assigns, _i64p), _p(a, _i64p), _p(rewards, _dp), ctypes.byref(done),
                            _p(self.obs, _dp))
        self.k, self.done = k.value, bool(done.value)
        return rewards, self.done, {}


class OracleRealVariantEnv(OracleRealEnv):
    """RealPowerConstellationEnv (kind "power", real_power_constellation_env.py) and
    InterferenceConstellationEnv (kind "interference", interference_constellation_env.py)
    with constant setup; `prev0` plays the reset's np.random.choice(m, n, replace=False)."""

    VARIANTS = {"real": 0, "power": 1, "interference": 2}

    def __init__(self, kind, sat_prox_mat, N, M, L, lambda_, task_prios, prev0, bands=None, neighbor_matrix=None,
                 T_trans=None):
        super().__init__(sat_prox_mat, N, M, L, lambda_, T_trans=T_trans, task_prios=task_prios)
        self.variant = self.VARIANTS[kind]
        self.prev0 = np.ascontiguousarray(prev0, dtype=np.int64)
        self.bands = np.ascontiguousarray(bands if bands is not None else np.zeros(self.n), dtype=np.int32)
        self.nbr = np.ascontiguousarray(neighbor_matrix if neighbor_matrix is not None else np.eye(self.m),
                                        dtype=np.float64)
        self.obs_size = lib().ora_realx_obs_size(self.variant, N, M, self.L)

    def reset(self):
        self.k = 0
        self.done = False
        self.beta = np.empty((self.n, self.m, self.L))
        self.prev_assigns = np.empty(self.n, dtype=np.int64)
        self.power_states = np.empty(self.n)
        self.obs = np.empty((self.n, self.obs_size))
        lib().ora_realx_reset(self.variant, _p(self.table, _dp), _p(self.prios, _dp), self.n, self.m, self.T, self.L,
                              self.N, self.M, _p(self.prev0, _i64p), _p(self.beta, _dp), _p(self.prev_assigns, _i64p),
                              _p(self.power_states, _dp), _p(self.obs, _dp))
        return self.obs

    def step(self, actions):
        a = np.ascontiguousarray(actions, dtype=np.int64)
        rewards = np.empty(self.n)
        k, done = ctypes.c_int(self.k), ctypes.c_int(0)
        lib().ora_realx_step(self.variant, _p(self.table, _dp), _p(self.prios, _dp), _p(self.T_trans, _dp),
                             self.bands.ctypes.data_as(ctypes.POINTER(ctypes.c_int)), _p(self.nbr, _dp), self.n,
                             self.m, self.T, self.L, self.N, self.M, self.lambda_, ctypes.byref(k), _p(self.beta, _dp),
                             _p(self.prev_assigns, _i64p), _p(self.power_states, _dp), _p(a, _i64p),
                             _p(rewards, _dp), ctypes.byref(done), _p(self.obs, _dp))
        self.k, self.done = k.value, bool(done.value)
        return rewards, self.done, {}


def rollout_random(E, n, m, T, L, lam, seed, threads, episodes=1):
    """Multi-threaded C rollout (asg_rollout.c); returns (seconds, returns[E])."""
    ret = np.empty(E, dtype=np.float64)
    secs = lib().ora_rollout_random(E, n, m, T, L, lam, seed, threads, episodes, _p(ret, _dp))
    return secs, ret
