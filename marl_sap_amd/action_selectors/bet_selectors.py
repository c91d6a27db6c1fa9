"""Bids-as-actions selector (reference: action_selectors/bet_selectors.py:4-24).

ContinuousActionSelector perturbs the agent's bid vector with Gaussian noise whose scale
follows the epsilon schedule (the reference calls it a variance and passes it to
torch.normal as the standard deviation; kept as is).  The draw happens on the agent
outputs' device (the GPU here), so the bids never leave HBM before the env's batched LSA
(asg_step with bids_as_actions).
"""
import torch

from ..components.epsilon_schedules import DecayThenFlatSchedule


class ContinuousActionSelector:
    def __init__(self, args):
        self.args = args
        self.schedule = DecayThenFlatSchedule(args.epsilon_start, args.epsilon_finish, args.epsilon_anneal_time,
                                              decay="linear")
        self.variance = self.schedule.eval(0)

    def select_action(self, agent_inputs, avail_actions, t_env, test_mode=False, state=None, beta=None):
        if getattr(self.args, "softmax_agent_inputs", False):
            agent_inputs = torch.softmax(agent_inputs, dim=1)
        self.variance = self.args.evaluation_epsilon if test_mode else self.schedule.eval(t_env)
        if self.variance == 0:
            return agent_inputs.detach().clone()  # torch.normal(x, 0) == x
        return torch.normal(agent_inputs, self.variance).detach()

    def action_log_prob(self, actions, old_agent_inputs):
        return torch.distributions.Normal(old_agent_inputs, self.variance).log_prob(actions)
