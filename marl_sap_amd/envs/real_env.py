"""Batched RealConstellationEnv on MI355X.

`RealAssignEnvBatch` owns E RealConstellationEnv episodes (src/envs/real_constellation_env.py)
on one GPU behind one `asg_real_*` C-ABI handle (include/asg.h): reset / step / the
top-M / top-N observation builder run as HIP kernels writing straight into an
EpisodeBatch with the reference's float16 / int16 scheme.

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


def obs_size(N, M, L):
    """RealConstellationEnv.get_obs_size (:251-253)."""
    return M * L + N * M * L + (N * M // 2) * L + M


def make_real_scheme(n, m, L, N, M):
    """Scheme + preprocess (real_constellation_env.py:74-97): half precision."""
    scheme = {
        "obs": {"vshape": obs_size(N, M, L), "group": "agents", "dtype": torch.float16},
        "actions": {"vshape": (1,), "group": "agents", "dtype": torch.int16},
        "avail_actions": {"vshape": (m,), "group": "agents", "dtype": torch.bool},
        "rewards": {"vshape": (n,), "dtype": torch.float16},
        "terminated": {"vshape": (1,), "dtype": torch.bool},
        "prev_assigns": {"vshape": (n,), "dtype": torch.int16, "part_of_state": True},
        "beta": {"vshape": (n, m, L), "dtype": torch.float16, "part_of_state": True},
    }
    preprocess = {"actions": ("actions_onehot", [OneHot(out_dim=m)])}
    return scheme, preprocess


class RealAssignEnvBatch(MultiAgentEnv):
    """E RealConstellationEnv episodes on one GPU, stepped in lockstep by HIP kernels."""

    def __init__(self, num_planes, num_sats_per_plane, m, T, N, M, L, lambda_, sat_prox_mat=None, graphs=None,
                 bids_as_actions=False, seed=None, T_trans=None, task_prios=None, num_envs=1, env_index_base=0,
                 device=None, rng=None, quirks=()):
        if not torch.cuda.is_available():
            raise RuntimeError("RealAssignEnvBatch needs a ROCm GPU (HIP path only, no CPU fallback)")
        if sat_prox_mat is None:
            raise ValueError("RealAssignEnvBatch needs sat_prox_mat (constant-benefit path); the orbital "
                             "simulator is not part of this build")
        if bids_as_actions:
            raise ValueError("bids_as_actions is not supported by the batched RealConstellationEnv")
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
        self.bids_as_actions = False
        self.env_index_base = int(env_index_base)
        self._seed = seed
        self.device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
        self.T_trans = (np.ones((self.m, self.m)) - np.eye(self.m) if T_trans is None
                        else np.ascontiguousarray(T_trans, dtype=np.float64))
        self.task_prios = (np.ones(self.m) if task_prios is None
                           else np.ascontiguousarray(task_prios, dtype=np.float64))
        self.obs_space_size = obs_size(self.N, self.M, self.L)
        self.scheme, self.preprocess = make_real_scheme(self.n, self.m, self.L, self.N, self.M)
        self.k = 0
        cfg = _lib.AsgRealConfig()
        cfg.num_envs, cfg.n, cfg.m, cfg.T, cfg.L = self.num_envs, self.n, self.m, self.T, int(L)
        cfg.N, cfg.M, cfg.lambda_ = self.N, self.M, self.lambda_
        dp = ctypes.POINTER(ctypes.c_double)
        cfg.T_trans = self.T_trans.ctypes.data_as(dp)
        cfg.task_prios = self.task_prios.ctypes.data_as(dp)
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            _lib.check(_lib.lib().asg_real_create(ctypes.byref(cfg), self.device.index,
                                                  _lib.stream_ptr(self.device), ctypes.byref(h)))
        self._h = h
        t = table.to(self.device).contiguous()
        self._call("asg_real_set_benefits", ctypes.c_void_p(t.data_ptr()), t.shape[0], 1)

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
        self._call("asg_real_reset", ctypes.byref(batch_view(batch)), int(ts))
        self.k = 0

    def step(self, batch, ts):
        """Reads actions at row ts; writes rewards / terminated / actions_onehot at ts and
        the next pre-transition row (obs, beta, avail, prev_assigns, filled) at ts + 1."""
        self._call("asg_real_step", ctypes.byref(batch_view(batch)), int(ts))
        self.k += 1
        return self.k >= self.T

    def sync(self):
        self._call("asg_real_sync_status")

    def get_returns(self):
        out = torch.empty(self.num_envs, dtype=torch.float64, device=self.device)
        self._call("asg_real_get_returns", ctypes.c_void_p(out.data_ptr()))
        return out

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
