"""Sequential-assignment selectors (reference: action_selectors/sap_selectors.py:7-98).
The per-env scipy loop becomes one batched HIP LSA over all envs (lsa.py)."""
import numpy as np
import torch

from ..components.epsilon_schedules import DecayThenFlatSchedule
from .lsa import DeferredStatus, linear_sum_assignment_batched


def _lsa_actions(q, status_sink):
    """float32 [B, n] task ids = LSA(q[b], maximize)[1] for every env (n <= m)."""
    _, col, status = linear_sum_assignment_batched(q, maximize=True, return_status=True)
    status_sink.add(status)
    return col.to(torch.float32)


class SequentialAssignmentProblemSelector:
    """REDA selector: Gaussian noise of std 2*eps*mean|Q| per env, then LSA(maximize)."""

    def __init__(self, args):
        self.args = args
        self.schedule = DecayThenFlatSchedule(args.epsilon_start, args.epsilon_finish, args.epsilon_anneal_time,
                                              decay="linear")
        self.epsilon = self.schedule.eval(0)
        self.status = DeferredStatus()

    def select_action(self, agent_inputs, avail_actions, t_env, test_mode=False, beta=None):
        self.epsilon = self.schedule.eval(t_env)
        if test_mode:
            self.epsilon = self.args.evaluation_epsilon
        q = agent_inputs.detach()
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
