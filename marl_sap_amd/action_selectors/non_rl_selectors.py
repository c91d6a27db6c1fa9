"""Non-RL selectors (reference: action_selectors/non_rl_selectors.py:10-50).

HAASelector: per env, LSA(maximize) of beta_hat(beta, prev_assigns) taken from the
batch's part_of_state fields -- fused into one HIP kernel over all envs
(asg_haa_select: beta_hat formed on the fly, scipy-exact LSA per wave)."""
import ctypes

import torch

from .. import _lib
from .lsa import DeferredStatus, raise_on_status

REGISTRY = {}


class HAASelector:
    def __init__(self, args):
        self.args = args
        self.envs = None
        self.status = DeferredStatus()

    def _env_params(self):
        env = self.envs[0] if self.envs is not None else None
        lam = env.lambda_ if env is not None else self.args.env_args["lambda_"]
        tt = getattr(env, "T_trans", None)
        m = self.args.m
        if tt is not None and not (torch.is_tensor(tt) and tt.numel() == 0):
            tt = torch.as_tensor(tt, dtype=torch.float64)
            eye = torch.ones((m, m), dtype=torch.float64) - torch.eye(m, dtype=torch.float64)
            if tt.shape == (m, m) and torch.equal(tt, eye):
                tt = None  # the default 1 - I is computed in-kernel
        return float(lam), tt

    def select_action(self, batch):
        beta = batch["beta"][:, 0]
        prev = batch["prev_assigns"][:, 0]
        if beta.dim() == 4:  # L-deep beta of the real env: use the current step only
            beta = beta[..., 0]
        lam, tt = self._env_params()
        out, status = haa_select_batched(beta, prev, lam, tt, return_status=True)
        self.status.add(status)
        return out


def haa_select_batched(beta, prev, lambda_, T_trans=None, return_status=False):
    """float32 [B, n] task ids = LSA(beta_hat(beta[b], prev[b]), maximize)[1] for every env
    (non_rl_selectors.py:36-47), one asg_haa_select launch.  beta: [B, n, m] CUDA tensor,
    prev: [B, n] int64, T_trans: None (the default 1 - I) or [m, m]."""
    B, n, m = beta.shape
    if beta.dtype != torch.float32:
        beta = beta.float()
    if prev.dtype != torch.int64:
        prev = prev.long()
    tt_dev = None
    if T_trans is not None:
        tt_dev = torch.as_tensor(T_trans, dtype=torch.float64).to(beta.device).contiguous()
        if tt_dev.shape != (m, m):
            raise ValueError(f"T_trans must be [{m}, {m}], got {list(tt_dev.shape)}")
        if not bool(torch.isfinite(tt_dev).all()):
            # beta_hat would hold NaN / inf entries: scipy's error for the LSA on it
            raise ValueError("matrix contains invalid numeric entries")
    out = torch.empty((B, n), dtype=torch.float32, device=beta.device)
    status = torch.empty((B,), dtype=torch.int32, device=beta.device)
    with torch.cuda.device(beta.device):
        _lib.check(_lib.lib().asg_haa_select(
            ctypes.c_void_p(beta.data_ptr()), _lib.i64arr(beta.stride()), ctypes.c_void_p(prev.data_ptr()),
            _lib.i64arr(prev.stride()), B, n, m,
            ctypes.c_void_p(tt_dev.data_ptr()) if tt_dev is not None else None, float(lambda_),
            ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(status.data_ptr()), _lib.stream_ptr(beta.device)))
    if return_status:
        return out, status
    raise_on_status(status)
    return out


class HAALSelector:
    """HAAL: HAA with an L-step lookahead over time-interval sequences (reference:
    non_rl_selectors.py:54-118).  The reference deep-copies each env once per sequence and
    steps the copies on the CPU; here the batched real env evaluates every sequence of every
    env on the GPU from its own state (asg_real_haal_select: one batched LSA per level of
    the sequences' decision tree, the rewards in the reference's order).  Returns float32
    task ids [B, n].  The reference requires the episode runner (its envs must be in
    lockstep with the batch); the batched env always is, so any protocol works."""

    def __init__(self, args):
        self.args = args
        self.envs = None
        self.status = DeferredStatus()
        self.last_values = None  # [B, S] float64 sequence values of the last call
        self.last_best = None    # [B] index of the winning sequence

    def select_action(self, batch):
        env = self.envs
        if env is None or not hasattr(env, "haal_select"):
            raise ValueError("HAALSelector needs the batched RealConstellationEnv (selector.envs)")
        out, values, best, status = env.haal_select(return_values=True)
        self.last_values, self.last_best = values, best
        self.status.add(status)
        return out


REGISTRY["haa_selector"] = HAASelector
REGISTRY["haal_selector"] = HAALSelector
