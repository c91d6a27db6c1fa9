"""Classic selectors (reference: action_selectors/classic_selectors.py:7-54) on the GPU.
Epsilon-greedy is one fused HIP pass (asg_epsilon_greedy) over the Q-values."""
import ctypes

import torch
from torch.distributions import Categorical

from .. import _lib
from ..components.epsilon_schedules import DecayThenFlatSchedule


def selector_seed(args):
    """64-bit Philox key of a selector: a function of args.seed alone."""
    return (int(getattr(args, "seed", 0) or 0) * 0x9E3779B97F4A7C15 + 0x2545F4914F6CDD1D) & 0xFFFFFFFFFFFFFFFF


def env_index_base(selector):
    """Global index of this rank's env 0 (the runner's env_index_base), for draws keyed by
    global env."""
    envs = getattr(selector, "envs", None)
    return int(getattr(envs, "env_index_base", getattr(selector.args, "env_index_base", 0)) or 0)


class MultinomialActionSelector:
    def __init__(self, args):
        self.args = args
        self.schedule = DecayThenFlatSchedule(args.epsilon_start, args.epsilon_finish, args.epsilon_anneal_time,
                                              decay="linear")
        self.epsilon = self.schedule.eval(0)
        self.test_greedy = getattr(args, "test_greedy", True)

    def select_action(self, agent_inputs, avail_actions, t_env, test_mode=False, beta=None):
        masked = agent_inputs.clone()
        masked[avail_actions == 0.0] = 0.0
        self.epsilon = self.schedule.eval(t_env)
        if test_mode and self.test_greedy:
            return masked.max(dim=2)[1]
        return Categorical(masked).sample().long()


class EpsilonGreedyActionSelector:
    """With prob. epsilon a uniformly random AVAILABLE action, else argmax over available
    actions (first maximal index) -- one HIP kernel per call; `out` (an int64 [B, n] view,
    e.g. the EpisodeBatch actions row) receives the actions in place."""

    def __init__(self, args):
        self.args = args
        self.schedule = DecayThenFlatSchedule(args.epsilon_start, args.epsilon_finish, args.epsilon_anneal_time,
                                              decay="linear")
        self.epsilon = self.schedule.eval(0)
        # the Philox key depends on args.seed only (not on the process's torch seed), and the
        # draws are keyed by global (env, agent) row: every rank of a sharded rollout draws
        # what a 1-GPU run draws for the same global envs
        self.seed = selector_seed(args)
        self.calls = 0
        self.status = None
        self.envs = None  # set by the runner (reference: run.py sets action_selector.envs)

    def env_index_base(self):
        return env_index_base(self)

    def fused_params(self, t_env, test_mode, device, calls=1):
        """Epsilon / seed / call counter / status word / global env base for a kernel that
        fuses this selector into the agent forward (asg_rnn_agent_select, asg_rollout); same
        state updates as `calls` select_action calls (their counters are the returned one,
        + 1, ...)."""
        self.epsilon = self.schedule.eval(t_env)
        if test_mode:
            self.epsilon = self.args.evaluation_epsilon
        if self.status is None or self.status.device != device:
            self.status = torch.zeros(1, dtype=torch.int32, device=device)
        first = self.calls + 1
        self.calls += int(calls)
        return self.epsilon, self.seed, first, self.status, self.env_index_base()

    def select_action(self, agent_inputs, avail_actions, t_env, test_mode=False, beta=None, out=None):
        self.epsilon = self.schedule.eval(t_env)
        if test_mode:
            self.epsilon = self.args.evaluation_epsilon
        q = agent_inputs if agent_inputs.dtype == torch.float32 else agent_inputs.float()
        B, n, m = q.shape
        if out is None or out.dtype != torch.int64:
            out = torch.empty((B, n), dtype=torch.int64, device=q.device)
        av = avail_actions if avail_actions.dtype == torch.bool else avail_actions != 0
        if self.status is None or self.status.device != q.device:
            self.status = torch.zeros(1, dtype=torch.int32, device=q.device)
        self.calls += 1
        with torch.cuda.device(q.device):
            _lib.check(_lib.lib().asg_epsilon_greedy(
                ctypes.c_void_p(q.data_ptr()), _lib.i64arr(q.stride()), ctypes.c_void_p(av.data_ptr()),
                _lib.i64arr(av.stride()), B, n, m, float(self.epsilon), self.seed & 0xFFFFFFFFFFFFFFFF, self.calls,
                self.env_index_base(), ctypes.c_void_p(out.data_ptr()), _lib.i64arr(out.stride()), ctypes.c_void_p(self.status.data_ptr()),
                _lib.stream_ptr(q.device)))
        return out

    def flush(self):
        """Raise (once per episode, from the runner) if a row had nothing to explore."""
        if self.status is not None and int(self.status.item()) != 0:
            self.status.zero_()
            raise ValueError("epsilon-greedy exploration over a row with no available action")


class SoftPoliciesSelector:
    def __init__(self, args):
        self.args = args

    def select_action(self, agent_inputs, avail_actions, t_env, test_mode=False, beta=None):
        return Categorical(agent_inputs).sample().long()
