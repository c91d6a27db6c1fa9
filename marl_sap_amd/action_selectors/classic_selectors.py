"""Classic selectors (reference: action_selectors/classic_selectors.py:7-54), batched
torch ops on the GPU."""
import torch
from torch.distributions import Categorical

from ..components.epsilon_schedules import DecayThenFlatSchedule


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
    actions (first maximal index)."""

    def __init__(self, args):
        self.args = args
        self.schedule = DecayThenFlatSchedule(args.epsilon_start, args.epsilon_finish, args.epsilon_anneal_time,
                                              decay="linear")
        self.epsilon = self.schedule.eval(0)

    def select_action(self, agent_inputs, avail_actions, t_env, test_mode=False, beta=None):
        self.epsilon = self.schedule.eval(t_env)
        if test_mode:
            self.epsilon = self.args.evaluation_epsilon
        masked_q = agent_inputs.masked_fill(avail_actions == 0, -float("inf"))
        greedy = masked_q.max(dim=2)[1]
        if self.epsilon <= 0.0:
            return greedy
        pick_random = torch.rand_like(agent_inputs[:, :, 0]) < self.epsilon
        B, n, m = agent_inputs.shape
        random_actions = torch.multinomial(avail_actions.reshape(B * n, m).float(), 1).view(B, n)
        return torch.where(pick_random, random_actions, greedy)


class SoftPoliciesSelector:
    def __init__(self, args):
        self.args = args

    def select_action(self, agent_inputs, avail_actions, t_env, test_mode=False, beta=None):
        return Categorical(agent_inputs).sample().long()
