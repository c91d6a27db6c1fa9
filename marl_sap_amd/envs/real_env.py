"""Batched RealConstellationEnv family on MI355X.

`RealAssignEnvBatch` owns E RealConstellationEnv episodes (src/envs/real_constellation_env.py)
on one GPU behind one `asg_real_*` C-ABI handle (include/asg.h): reset / step / the
top-M / top-N observation builder run as HIP kernels writing straight into an
EpisodeBatch with the reference's float16 / int16 scheme.  `RealPowerAssignEnvBatch`
(real_power_constellation_env.py) adds per-satellite power states;
`InterferenceAssignEnvBatch` (interference_constellation_env.py) adds the beam
interference reward over satellites sharing a frequency band.

Benefits: the constant-benefit path of the reference (sat_prox_mat + graphs injected,
:55-61) — the orbital simulator that would draw new tasks per reset
(HighPerformanceConstellationSim) is out of scope (astropy / poliastro are not part of
the rollout path).  `sat_prox_mat` is [n, m, T] (shared by every env, as the reference
reuses it every episode) or [E, n, m, T] (one table per env).
"""
import ctypes

import numpy as np
import torch

from .. import _lib
from ..components.transforms import OneHot
from .assign_env import batch_view
from .multiagentenv import MultiAgentEnv


def obs_size(N, M, L, power=False):
    """get_obs_size (real_constellation_env.py:251-253; + N + 1 power observations in
    real_power_constellation_env.py:286-290)."""
    return M * L + N * M * L + (N * M // 2) * L + M + ((N + 1) if power else 0)


def make_real_scheme(n, m, L, N, M, power=False, bids_as_actions=False):
    """Scheme + preprocess (real_constellation_env.py:74-97, real_power_constellation_env.py:
    95-116): half precision; the power variants add power_states; bids_as_actions: float32
    bids [m] per agent and no one-hot preprocess (real_constellation_env.py:110-112)."""
    scheme = {
        "obs": {"vshape": obs_size(N, M, L, power), "group": "agents", "dtype": torch.float16},
        "actions": {"vshape": (1,), "group": "agents", "dtype": torch.int16},
        "avail_actions": {"vshape": (m,), "group": "agents", "dtype": torch.bool},
        "rewards": {"vshape": (n,), "dtype": torch.float16},
        "terminated": {"vshape": (1,), "dtype": torch.bool},
        "prev_assigns": {"vshape": (n,), "dtype": torch.int16, "part_of_state": True},
        "beta": {"vshape": (n, m, L), "dtype": torch.float16, "part_of_state": True},
    }
    if power:
        scheme["power_states"] = {"vshape": (n,), "dtype": torch.float16, "part_of_state": True}
    preprocess = {"actions": ("actions_onehot", [OneHot(out_dim=m)])}
    if bids_as_actions:
        scheme["actions"] = {"vshape": (m,), "group": "agents", "dtype": torch.float32}
        preprocess = {}
    return scheme, preprocess


def real_batch_view(data):
    """asg_real_batch_view over an EpisodeBatch (or a dict of its transition tensors)."""
    td = data.data.transition_data if hasattr(data, "data") else data
    v = _lib.AsgRealBatchView()
    v.base = batch_view(td)
    v.power_states = _lib.field(td.get("power_states"))
    return v


class RealAssignEnvBatch(MultiAgentEnv):
    """E RealConstellationEnv episodes on one GPU, stepped in lockstep by HIP kernels."""

    VARIANT = _lib.ASG_REAL_PLAIN

    def __init__(self, num_planes, num_sats_per_plane, m, T, N, M, L, lambda_, sat_prox_mat=None, graphs=None,
                 bids_as_actions=False, seed=None, T_trans=None, task_prios=None, num_envs=1, env_index_base=0,
                 device=None, rng=None, quirks=(), sat_freq_bands=None, neighbor_matrix=None,
                 initial_assignments=None):
        if not torch.cuda.is_available():
            raise RuntimeError("RealAssignEnvBatch needs a ROCm GPU (HIP path only, no CPU fallback)")
        if sat_prox_mat is None:
            raise ValueError("RealAssignEnvBatch needs sat_prox_mat (constant-benefit path); the orbital "
                             "simulator is not part of this build")
        table = torch.as_tensor(np.asarray(sat_prox_mat, dtype=np.float64) if not torch.is_tensor(sat_prox_mat)
                                else sat_prox_mat, dtype=torch.float64)
        if table.dim() == 3:
            table = table.unsqueeze(0)
        self.num_envs = int(num_envs)
        if table.shape[0] not in (1, self.num_envs):
            raise ValueError("sat_prox_mat must be [n, m, T] or [num_envs, n, m, T]")
        # the table's shape wins over the constellation arguments (:56-61)
        self.n, self.m, self.T = int(table.shape[1]), int(table.shape[2]), int(table.shape[3])
        self.N, self.M, self.L = int(N), int(M), min(int(L), int(T))
        self.lambda_ = float(lambda_)
        # bids_as_actions: each step solves LSA(bids, maximize) per env on the GPU (asg_lsa_batched's
        # scipy-exact solver inside asg_real_step) -- real_constellation_env.py:140-142
        self.bids_as_actions = bool(bids_as_actions)
        self.env_index_base = int(env_index_base)
        self._seed = seed
        self.device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
        self.T_trans = (np.ones((self.m, self.m)) - np.eye(self.m) if T_trans is None
                        else np.ascontiguousarray(T_trans, dtype=np.float64))
        power = self.VARIANT != _lib.ASG_REAL_PLAIN
        if task_prios is None and power:
            # the reference draws choice([1, 1, 1, 5], m) from numpy's global stream
            task_prios = np.random.RandomState(0 if seed is None else int(seed)).choice([1, 1, 1, 5], size=self.m)
        self.task_prios = (np.ones(self.m) if task_prios is None
                           else np.ascontiguousarray(task_prios, dtype=np.float64))
        self.sat_freq_bands = None if sat_freq_bands is None else np.ascontiguousarray(sat_freq_bands, dtype=np.int32)
        self.neighbor_matrix = (None if neighbor_matrix is None
                                else np.ascontiguousarray(neighbor_matrix, dtype=np.float64))
        self.obs_space_size = obs_size(self.N, self.M, self.L, power)
        self.scheme, self.preprocess = make_real_scheme(self.n, self.m, self.L, self.N, self.M, power,
                                                        self.bids_as_actions)
        self.k = 0
        cfg = _lib.AsgRealConfig()
        cfg.num_envs, cfg.n, cfg.m, cfg.T, cfg.L = self.num_envs, self.n, self.m, self.T, int(L)
        cfg.N, cfg.M, cfg.lambda_ = self.N, self.M, self.lambda_
        dp = ctypes.POINTER(ctypes.c_double)
        cfg.T_trans = self.T_trans.ctypes.data_as(dp)
        cfg.task_prios = self.task_prios.ctypes.data_as(dp)
        cfg.variant = self.VARIANT
        cfg.bids_as_actions = int(self.bids_as_actions)
        cfg.seed = (0 if seed is None else int(seed)) & 0xFFFFFFFFFFFFFFFF
        cfg.env_index_base = self.env_index_base
        if self.sat_freq_bands is not None:
            cfg.sat_freq_bands = self.sat_freq_bands.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))
        if self.neighbor_matrix is not None:
            cfg.neighbor_matrix = self.neighbor_matrix.ctypes.data_as(dp)
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            _lib.check(_lib.lib().asg_real_create(ctypes.byref(cfg), self.device.index,
                                                  _lib.stream_ptr(self.device), ctypes.byref(h)))
        self._h = h
        t = table.to(self.device).contiguous()
        self._call("asg_real_set_benefits", ctypes.c_void_p(t.data_ptr()), t.shape[0], 1)
        if initial_assignments is not None:
            self.set_initial_assignments(initial_assignments)

    def set_initial_assignments(self, prev0):
        """Power variants: use these reset assignments ([n] or [E, n]) instead of Philox
        draws -- the reference's np.random.choice(m, n, replace=False); None: Philox."""
        if prev0 is None:
            self._call("asg_real_set_initial_assignments", None, 0, 0)
            return
        p = np.ascontiguousarray(prev0, dtype=np.int64)
        p2 = p.reshape(1 if p.ndim == 1 else p.shape[0], self.n)
        self._call("asg_real_set_initial_assignments", p2.ctypes.data_as(ctypes.c_void_p), p2.shape[0], 0)

    def _call(self, fn, *args):
        L = _lib.lib()
        with torch.cuda.device(self.device):
            L.asg_real_set_stream(self._h, _lib.stream_ptr(self.device))
            _lib.check(getattr(L, fn)(self._h, *args))

    def close(self):
        if getattr(self, "_h", None):
            _lib.lib().asg_real_destroy(self._h)
            self._h = None
        return True

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------------ hot path
    def reset(self, batch, ts=0):
        """New episode for every env (k = 0, prev_assigns = arange(n)); writes row ts."""
        self._call("asg_real_reset", ctypes.byref(real_batch_view(batch)), int(ts))
        self.k = 0

    def step(self, batch, ts):
        """Reads actions at row ts; writes rewards / terminated / actions_onehot at ts and
        the next pre-transition row (obs, beta, avail, prev_assigns, filled) at ts + 1.
        bids_as_actions: the actions row holds float32 bids [E, n, m] and the step's tasks are
        LSA(bids, maximize) per env (a NaN / -inf bid raises scipy's ValueError at sync())."""
        self._call("asg_real_step", ctypes.byref(real_batch_view(batch)), int(ts))
        self.k += 1
        return self.k >= self.T

    def sync(self):
        self._call("asg_real_sync_status")

    def get_returns(self):
        out = torch.empty(self.num_envs, dtype=torch.float64, device=self.device)
        self._call("asg_real_get_returns", ctypes.c_void_p(out.data_ptr()))
        return out

    def haal_select(self, return_values=False):
        """HAALSelector.select_action (non_rl_selectors.py:54-118) for every env at the
        current step, on the handle's own state (asg_real_haal_select): float32 [E, n] task
        ids; with return_values also the float64 [E, S] value of every time-interval
        sequence (the reference's order) and the int32 [E] index of the winning one.
        Raises ValueError with scipy's message when an LSA fails (deferred: a status tensor
        is returned for the runner to flush)."""
        S = int(_lib.lib().asg_real_haal_num_sequences(self._h))
        if S <= 0:
            raise ValueError("HAAL selection after the episode's last step")
        out = torch.empty((self.num_envs, self.n), dtype=torch.float32, device=self.device)
        values = torch.empty((self.num_envs, S), dtype=torch.float64, device=self.device)
        best = torch.empty((self.num_envs,), dtype=torch.int32, device=self.device)
        status = torch.empty((self.num_envs,), dtype=torch.int32, device=self.device)
        p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        self._call("asg_real_haal_select", p(out), p(values), p(best), p(status))
        if return_values:
            return out, values, best, status
        return out, status

    # ------------------------------------------------------------------ env surface
    def beta_hat(self, beta, prev_assigns):
        """RealConstellationEnv.beta_hat (:259-327): penalty on the l = 0 slice where the
        L-summed benefit is meaningful; [.., n, m, L] in, float64 out."""
        beta = torch.as_tensor(beta, device=self.device).to(torch.float64)
        prev = torch.as_tensor(prev_assigns, device=self.device).to(torch.int64)
        tt = torch.as_tensor(self.T_trans, device=self.device)
        pen = tt[prev] * (beta.sum(-1) > 1e-12)
        out = beta.clone()
        out[..., 0] = out[..., 0] - self.lambda_ * pen
        return out

    def get_obs_size(self):
        return self.obs_space_size

    def get_state_size(self):
        return self.n * self.obs_space_size

    def get_total_actions(self):
        return self.m

    def get_stats(self):
        return {}

    def get_env_info(self):
        return {"state_shape": self.get_state_size(), "obs_shape": self.get_obs_size(),
                "m": self.get_total_actions(), "n": self.n, "T": self.T}

    def save_replay(self):
        pass

    def render(self):
        pass


class RealPowerAssignEnvBatch(RealAssignEnvBatch):
    """RealPowerConstellationEnv (real_power_constellation_env.py) batched: power states
    drained 0.2 per meaningful task, recharged 0.1 otherwise (capped at 1), dead at <= 0;
    beta_hat zeroed below 1e-12 power; reset assignments are choice(m, n, replace=False)
    (Philox per global env, or `initial_assignments` for exact parity)."""

    VARIANT = _lib.ASG_REAL_POWER

    def beta_hat(self, beta, prev_assigns, power_states=None):
        out = super().beta_hat(beta, prev_assigns)
        if power_states is not None:
            dead = torch.as_tensor(power_states, device=self.device) < 1e-12
            out = torch.where(dead[..., None, None], torch.zeros_like(out), out)
        return out


class InterferenceAssignEnvBatch(RealPowerAssignEnvBatch):
    """InterferenceConstellationEnv (interference_constellation_env.py) batched: the power
    dynamics plus reward = beta[i, a_i, 0] * 0.5 ** conflicts with the conflicts counted
    over satellites of the same frequency band through the task neighbour matrix
    (:309-353).  The orbital simulator that produces sat_prox_mat / neighbor_matrix for
    coverage tasks is not part of this build: pass them in (constant setup)."""

    VARIANT = _lib.ASG_REAL_INTERFERENCE

    def __init__(self, num_planes, num_sats_per_plane, res=None, T=None, N=None, M=None, L=None, lambda_=None,
                 task_prios=None, sat_freq_bands=None, bids_as_actions=False, seed=None, sat_prox_mat=None,
                 neighbor_matrix=None, **kw):
        if sat_prox_mat is None or neighbor_matrix is None or sat_freq_bands is None:
            raise ValueError("InterferenceAssignEnvBatch needs sat_prox_mat, neighbor_matrix and sat_freq_bands")
        tab = np.asarray(sat_prox_mat) if not torch.is_tensor(sat_prox_mat) else sat_prox_mat
        super().__init__(num_planes, num_sats_per_plane, tab.shape[-2], T, N, M, L, lambda_, sat_prox_mat=sat_prox_mat,
                         bids_as_actions=bids_as_actions, seed=seed, task_prios=task_prios,
                         sat_freq_bands=sat_freq_bands, neighbor_matrix=neighbor_matrix, **kw)
        self.res = res
