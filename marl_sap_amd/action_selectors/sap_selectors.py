"""Sequential-assignment selectors (reference: action_selectors/sap_selectors.py:7-98).
The per-env scipy loop becomes one batched HIP LSA over all envs (lsa.py)."""
import ctypes

import numpy as np
import torch

from .. import _lib
from ..components.epsilon_schedules import DecayThenFlatSchedule
from .classic_selectors import env_index_base, selector_seed
from .lsa import DeferredStatus, linear_sum_assignment_batched


def _lsa_actions(q, status_sink):
    """float32 [B, n] task ids = LSA(q[b], maximize)[1] for every env (n <= m)."""
    _, col, status = linear_sum_assignment_batched(q, maximize=True, return_status=True)
    status_sink.add(status)
    return col.to(torch.float32)


class SequentialAssignmentProblemSelector:
    """REDA selector: Gaussian noise of std 2*eps*mean|Q| per env, then LSA(maximize).

    n <= m <= 64: one fused HIP kernel (asg_sap_select: noise drawn in registers from
    Philox keyed by (seed, global env index, call counter), register-resident LSA); writing
    into the batch's actions row (the runner's step_q schedule) with n == m, the certified
    fast path starts from each env's previous column duals (asg_sap_select_warm).
    Larger problems: the noise from torch, then asg_lsa_batched."""

    def __init__(self, args):
        self.args = args
        self.schedule = DecayThenFlatSchedule(args.epsilon_start, args.epsilon_finish, args.epsilon_anneal_time,
                                              decay="linear")
        self.epsilon = self.schedule.eval(0)
        self.status = DeferredStatus()
        self.seed = selector_seed(args)
        self.calls = 0
        self.envs = None  # set by the runner (reference: run.py sets action_selector.envs)
        # instrumentation (bench.py): an int32 [B] device tensor receives every env's count of
        # augmenting-path steps of the next fused call
        self.count_steps = None
        # the fast path's warm start (asg_sap_select_warm): each env's column duals from its
        # previous selection, [B, 64] float64 on the device; args.sap_warm_start = False opts out.
        # Assignments do not depend on it (certified or solved by scipy's algorithm).
        self.warm_start = bool(getattr(args, "sap_warm_start", True))
        self._duals = None
        # an episode's first selection solves a new env's Q: by default it still starts from the
        # previous episode's last duals (measured faster than a cold start: 1.20 vs 1.43 ms for
        # the reset + forward + first selection at configs[2], profiles/r6_reda_cold_warm_s23.txt);
        # args.sap_warm_across_episodes = False starts it cold
        self.warm_across_episodes = bool(getattr(args, "sap_warm_across_episodes", True))
        self._cold_next = False

    def episode_start(self):
        """The next selection is the first of an episode (called by the MAC at t_ep = 0)."""
        self._cold_next = not self.warm_across_episodes

    def _env_index_base(self):
        return env_index_base(self)

    def select_action(self, agent_inputs, avail_actions, t_env, test_mode=False, beta=None, out=None):
        """Returns the float32 task ids (the reference's picked_actions); with `out` (an int64
        [B, n] contiguous view, e.g. the EpisodeBatch actions row the runner would cast them
        into) the ids are written there as int64 and `out` is returned."""
        self.epsilon = self.schedule.eval(t_env)
        if test_mode:
            self.epsilon = self.args.evaluation_epsilon
        q = agent_inputs.detach()
        B, n, m = q.shape
        if n <= m <= 64 and q.is_cuda:
            if q.dtype != torch.float32:
                q = q.float()
            into = (out is not None and out.dtype == torch.int64 and tuple(out.shape) == (B, n)
                    and out.is_contiguous() and out.device == q.device)
            self.calls += 1
            steps = ctypes.c_void_p(self.count_steps.data_ptr()) if self.count_steps is not None else None
            common = (ctypes.c_void_p(q.data_ptr()), _lib.i64arr(q.stride()), B, n, m, float(self.epsilon),
                      self.seed & 0xFFFFFFFFFFFFFFFF, self.calls, self._env_index_base())
            with torch.cuda.device(q.device):
                if into:
                    status = self.status.sticky(B, q.device)  # min-accumulated by the kernel
                    if self.warm_start and n == m:
                        d = self._duals
                        warm = int(d is not None and d.shape[0] == B and d.device == q.device and not self._cold_next)
                        self._cold_next = False
                        if d is None or d.shape[0] != B or d.device != q.device:
                            d = self._duals = torch.empty((B, 64), dtype=torch.float64, device=q.device)
                        _lib.check(_lib.lib().asg_sap_select_warm(
                            *common, ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(status.data_ptr()), steps,
                            ctypes.c_void_p(d.data_ptr()), warm, _lib.stream_ptr(q.device)))
                        return out
                    _lib.check(_lib.lib().asg_sap_select_into(
                        *common, ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(status.data_ptr()), steps,
                        _lib.stream_ptr(q.device)))
                    return out
                res = torch.empty((B, n), dtype=torch.float32, device=q.device)
                status = torch.empty((B,), dtype=torch.int32, device=q.device)
                _lib.check(_lib.lib().asg_sap_select(
                    *common, ctypes.c_void_p(res.data_ptr()), ctypes.c_void_p(status.data_ptr()), steps,
                    _lib.stream_ptr(q.device)))
            self.status.add(status)
            return res
        if self.epsilon > 0:
            avg = q.abs().mean(dim=(1, 2), keepdim=True)
            q = q + torch.randn_like(q) * (avg * self.epsilon * 2)
        return _lsa_actions(q, self.status)


class EpsilonGreedySAPTestActionSelector:
    """epsilon-greedy while training, LSA on the Q-values in test mode."""

    def __init__(self, args):
        self.args = args
        self.schedule = DecayThenFlatSchedule(args.epsilon_start, args.epsilon_finish, args.epsilon_anneal_time,
                                              decay="linear")
        self.epsilon = self.schedule.eval(0)
        self.status = DeferredStatus()

    def select_action(self, agent_inputs, avail_actions, t_env, test_mode=False, beta=None):
        self.epsilon = self.schedule.eval(t_env)
        B, n, m = agent_inputs.shape
        if test_mode:
            return _lsa_actions(agent_inputs.detach(), self.status)
        if np.random.rand() < self.epsilon:
            return torch.randperm(n, device=agent_inputs.device)  # reference quirk: one permutation
        masked_q = agent_inputs.masked_fill(avail_actions == 0, -float("inf"))
        pick_random = (torch.rand_like(agent_inputs[:, :, 0]) < self.epsilon).long()
        random_actions = torch.multinomial(avail_actions.reshape(B * n, m).float(), 1).view(B, n)
        return pick_random * random_actions + (1 - pick_random) * masked_q.max(dim=2)[1]
