"""Filtered selectors of the real-env algorithms (reference:
action_selectors/filtered_sap_selectors.py:7-148, filtered_classic_selectors.py:6-103).

The agent emits M + 1 values per agent -- one per task of its top M (by the L-summed
benefit in `beta`) and a baseline for every other task.  Each selector maps them onto the m
tasks and picks: LSA per env (SAP), epsilon-greedy argmax per row, or a sampled index.  The
reference builds the [n, m] matrix env by env on the CPU (topk, fancy indexing, scipy);
here it is asg_filtered_topm + asg_filtered_benefits over all envs at once, then the batched
scipy-exact LSA or the epsilon-greedy kernel (include/asg.h).

Randomness: the reference's torch.rand_like tie noise and torch.normal exploration noise are
Philox draws keyed by (args.seed, global env, call counter) here -- shard-invariant, not the
CPU torch stream.  Parity tests pass the reference's recorded draws through `tie_noise=` /
`gauss_noise=` and get its actions bit for bit.  torch.topk's order among equal totals is
unspecified; here ties go to the lower task index.
"""
import ctypes

import torch

from .. import _lib
from ..components.epsilon_schedules import DecayThenFlatSchedule
from .classic_selectors import env_index_base, selector_seed
from .lsa import DeferredStatus, linear_sum_assignment_batched


def _p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def filtered_top_m(beta, M):
    """th.topk(beta.sum(-1), k=M).indices for beta [B, n, m, L] (float16 / float32 /
    float64 CUDA tensor): int64 [B, n, M], descending, ties to the lower index."""
    if beta.dim() != 4:
        raise ValueError("beta must be [B, n, m, L]")
    if beta.dtype not in (torch.float16, torch.float32, torch.float64):
        beta = beta.float()
    B, n, m, L = beta.shape
    out = torch.empty((B, n, M), dtype=torch.int64, device=beta.device)
    with torch.cuda.device(beta.device):
        _lib.check(_lib.lib().asg_filtered_topm(_p(beta), _lib.dtype_code(beta.dtype), _lib.i64arr(beta.stride()), B,
                                                n, m, L, M, _p(out), _lib.stream_ptr(beta.device)))
    return out


def filtered_benefit_matrix(q, topm, m, tie_noise=None, gauss_epsilon=0.0, gauss_noise=None, seed=0, counter=0,
                            env_base=0):
    """The [B, n, m] float32 matrix of the filtered selectors (filtered_sap_selectors.py:37-55):
    baseline q[..., M] + u * 1e-8 everywhere, q[..., s] on the s-th top task; optionally the
    SAP selector's Gaussian noise (std 2 eps mean|mat[b]|) added per env."""
    if q.dtype != torch.float32:
        q = q.float()
    B, n, M1 = q.shape
    M = topm.shape[-1]
    if M1 != M + 1:
        raise ValueError(f"agent outputs must be [B, n, M + 1] = [.., .., {M + 1}], got {list(q.shape)}")
    out = torch.empty((B, n, m), dtype=torch.float32, device=q.device)
    for t in (tie_noise, gauss_noise):
        if t is not None and (t.shape != out.shape or t.dtype != torch.float32 or not t.is_contiguous()):
            raise ValueError("injected noise must be a contiguous float32 [B, n, m] tensor")
    topm = topm.contiguous()
    with torch.cuda.device(q.device):
        _lib.check(_lib.lib().asg_filtered_benefits(
            _p(q), _lib.i64arr(q.stride()), _p(topm), B, n, m, M, _p(tie_noise), float(gauss_epsilon),
            _p(gauss_noise), seed & 0xFFFFFFFFFFFFFFFF, counter, env_base, _p(out), _lib.stream_ptr(q.device)))
    return out


class _FilteredBase:
    def __init__(self, args):
        self.args = args
        self.seed = selector_seed(args)
        self.calls = 0
        self.envs = None  # set by the runner (env_index_base for shard-invariant draws)
        self.last_matrix = None  # the benefit matrix of the last call (debugging / tests)
        self.status = None

    def _M(self):
        return int(self.args.env_args["M"])

    def _matrix(self, agent_inputs, beta, tie_noise, gauss_epsilon=0.0, gauss_noise=None):
        assert beta is not None, "Need beta to figure out which are the top M tasks for each agent."
        self.calls += 1
        topm = filtered_top_m(beta, self._M())
        mat = filtered_benefit_matrix(agent_inputs.detach(), topm, beta.shape[2], tie_noise, gauss_epsilon,
                                      gauss_noise, self.seed, self.calls, env_index_base(self))
        self.last_matrix = mat
        return mat

    def _greedy(self, mat, avail_actions, epsilon):
        """pick_random * Categorical(avail) + (1 - pick_random) * mat.max(dim=2)[1]"""
        B, n, m = mat.shape
        av = avail_actions if avail_actions.dtype == torch.bool else avail_actions != 0
        out = torch.empty((B, n), dtype=torch.int64, device=mat.device)
        if self.status is None or self.status.device != mat.device:
            self.status = torch.zeros(1, dtype=torch.int32, device=mat.device)
        with torch.cuda.device(mat.device):
            _lib.check(_lib.lib().asg_filtered_epsilon_greedy(
                _p(mat), _lib.i64arr(mat.stride()), _p(av), _lib.i64arr(av.stride()), B, n, m, float(epsilon),
                self.seed & 0xFFFFFFFFFFFFFFFF, self.calls, env_index_base(self), _p(out), _lib.i64arr(out.stride()),
                _p(self.status), _lib.stream_ptr(mat.device)))
        return out

    # the message of this selector's device status word (ASG_E_INVALID_ARG)
    status_message = "epsilon-greedy exploration over a row with no available action"

    def flush(self):
        """Raise (once per episode, from the runner) on a deferred device error."""
        if isinstance(getattr(self, "lsa_status", None), DeferredStatus):
            self.lsa_status.flush()
        if self.status is not None and int(self.status.item()) != 0:
            self.status.zero_()
            raise ValueError(self.status_message)


class FilteredSAPActionSelector(_FilteredBase):
    """filtered_sap_selectors.py:7-66: Gaussian noise of std 2 eps mean|mat| per env, then
    LSA(maximize); float32 task ids."""

    def __init__(self, args):
        super().__init__(args)
        self.schedule = DecayThenFlatSchedule(args.epsilon_start, args.epsilon_finish, args.epsilon_anneal_time,
                                              decay="linear")
        self.epsilon = self.schedule.eval(0)
        self.lsa_status = DeferredStatus()

    def select_action(self, agent_inputs, avail_actions, t_env, test_mode=False, beta=None, tie_noise=None,
                      gauss_noise=None):
        self.epsilon = self.schedule.eval(t_env)
        if test_mode:
            self.epsilon = self.args.evaluation_epsilon
        mat = self._matrix(agent_inputs, beta, tie_noise, float(self.epsilon), gauss_noise)
        _, col, status = linear_sum_assignment_batched(mat, maximize=True, return_status=True)
        self.lsa_status.add(status)
        return col.to(torch.float32)


class FilteredEpsGrSAPTestActionSelector(_FilteredBase):
    """filtered_sap_selectors.py:68-148: LSA on the (noise-free) matrix in test mode (float32
    task ids), epsilon-greedy on it while training (int64)."""

    def __init__(self, args):
        super().__init__(args)
        self.schedule = DecayThenFlatSchedule(args.epsilon_start, args.epsilon_finish, args.epsilon_anneal_time,
                                              decay="linear")
        self.epsilon = self.schedule.eval(0)
        self.lsa_status = DeferredStatus()

    def select_action(self, agent_inputs, avail_actions, t_env, test_mode=False, beta=None, tie_noise=None):
        self.epsilon = self.schedule.eval(t_env)
        mat = self._matrix(agent_inputs, beta, tie_noise)
        if test_mode:
            _, col, status = linear_sum_assignment_batched(mat, maximize=True, return_status=True)
            self.lsa_status.add(status)
            return col.to(torch.float32)
        return self._greedy(mat, avail_actions, self.epsilon)


class FilteredEpsilonGreedyActionSelector(_FilteredBase):
    """filtered_classic_selectors.py:6-67: epsilon-greedy over the filtered matrix (int64)."""

    def __init__(self, args):
        super().__init__(args)
        self.schedule = DecayThenFlatSchedule(args.epsilon_start, args.epsilon_finish, args.epsilon_anneal_time,
                                              decay="linear")
        self.epsilon = self.schedule.eval(0)

    def select_action(self, agent_inputs, avail_actions, t_env, test_mode=False, beta=None, tie_noise=None):
        self.epsilon = self.schedule.eval(t_env)
        if test_mode:
            self.epsilon = self.args.evaluation_epsilon
        mat = self._matrix(agent_inputs, beta, tie_noise)
        return self._greedy(mat, avail_actions, self.epsilon)


class FilteredSoftPoliciesSelector(_FilteredBase):
    """filtered_classic_selectors.py:69-103: sample an index from the M + 1 policy values
    (Categorical), then map it to a task: the index-th top task, or for index M a uniformly
    random task outside the top M (int64)."""

    status_message = "soft-policies selection picked an index outside [0, M] (policy over M + 1 outputs expected)"

    def select_action(self, agent_inputs, avail_actions, t_env, test_mode=False, beta=None):
        assert beta is not None, "Need beta to figure out which are the top M tasks for each agent."
        B, n, M1 = agent_inputs.shape
        M = self._M()
        picked = torch.distributions.Categorical(agent_inputs).sample().long().contiguous()
        topm = filtered_top_m(beta, M)
        self.calls += 1
        out = torch.empty((B, n), dtype=torch.int64, device=agent_inputs.device)
        if self.status is None or self.status.device != out.device:
            self.status = torch.zeros(1, dtype=torch.int32, device=out.device)
        with torch.cuda.device(out.device):
            _lib.check(_lib.lib().asg_filtered_soft_map(
                _p(picked), _p(topm), B, n, beta.shape[2], M, self.seed & 0xFFFFFFFFFFFFFFFF, self.calls,
                env_index_base(self), _p(out), _p(self.status), _lib.stream_ptr(out.device)))
        return out
