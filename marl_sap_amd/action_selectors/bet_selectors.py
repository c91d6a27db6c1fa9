"""Bids-as-actions selector (reference: action_selectors/bet_selectors.py:4-24).

ContinuousActionSelector perturbs the agent's bid vector with Gaussian noise whose scale
follows the epsilon schedule (the reference calls it a variance and passes it to
torch.normal as the standard deviation; kept as is).  The draw happens on the agent
outputs' device (the GPU here), so the bids never leave HBM before the env's batched LSA
(asg_step with bids_as_actions).

With the batched env (bids_as_actions, n <= m <= 64) the MAC takes `fused_bids` instead: one
kernel per step (asg_bids_select) applies the MAC's pi_logits softmax, this selector's softmax
over the agents and its noise (Philox keyed by (seed, global env index, call)), writes the bids
into the batch's actions row and solves their LSA for the env's next step.
"""
import torch

from ..components.epsilon_schedules import DecayThenFlatSchedule
from .classic_selectors import selector_seed


class ContinuousActionSelector:
    def __init__(self, args):
        self.args = args
        self.schedule = DecayThenFlatSchedule(args.epsilon_start, args.epsilon_finish, args.epsilon_anneal_time,
                                              decay="linear")
        self.variance = self.schedule.eval(0)
        self.seed = selector_seed(args)
        self.calls = 0
        self.envs = None  # set by the runner (the batched env: fused_bids)
        # instrumentation (bench.py): an int32 [B] device tensor receives every env's augmenting-path
        # steps of the next fused_bids call (the counting kernel instance), then is left as is
        self.count_steps = None

    def fused_bids(self, q, out, t_env, test_mode=False, row_softmax=False):
        """The bids of every env from the agent's raw outputs q [B, n, m] (row_softmax: the
        MAC's pi_logits softmax first) into `out` [B, n, m] float32 (the batch's actions row),
        and their LSA assignments into the env handle -- select_action's bids (up to the noise
        draws) in one asg_bids_select launch.  Returns out."""
        self.variance = self.args.evaluation_epsilon if test_mode else self.schedule.eval(t_env)
        self.calls += 1
        self.envs.bids_select(q, out, row_softmax, bool(getattr(self.args, "softmax_agent_inputs", False)),
                              float(self.variance), self.seed, self.calls, count_steps=self.count_steps)
        return out

    def select_action(self, agent_inputs, avail_actions, t_env, test_mode=False, state=None, beta=None):
        if getattr(self.args, "softmax_agent_inputs", False):
            agent_inputs = torch.softmax(agent_inputs, dim=1)
        self.variance = self.args.evaluation_epsilon if test_mode else self.schedule.eval(t_env)
        if self.variance == 0:
            return agent_inputs.detach().clone()  # torch.normal(x, 0) == x
        return torch.normal(agent_inputs, self.variance).detach()

    def action_log_prob(self, actions, old_agent_inputs):
        return torch.distributions.Normal(old_agent_inputs, self.variance).log_prob(actions)
