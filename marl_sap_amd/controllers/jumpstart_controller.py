"""Jumpstart controller (reference: controllers/jumpstart_controller.py:10-121): with
probability jumpstart_epsilon (one numpy coin flip per step for the whole batch, drawn
from numpy's global stream like the reference) the non-RL selector (HAA) acts."""
import numpy as np

from ..action_selectors.non_rl_selectors import REGISTRY as non_rl_REGISTRY
from ..components.epsilon_schedules import DecayThenFlatSchedule
from .basic_controller import BasicMAC


class JumpstartMAC(BasicMAC):
    def __init__(self, scheme, groups, args):
        super().__init__(scheme, groups, args)
        self.jumpstart_action_selector = non_rl_REGISTRY[args.jumpstart_action_selector](args)
        self.jumpstart_eps_schedule = DecayThenFlatSchedule(args.jumpstart_epsilon_start,
                                                            args.jumpstart_epsilon_finish,
                                                            args.jumpstart_epsilon_anneal_time, decay="linear")
        self.jumpstart_epsilon = self.jumpstart_eps_schedule.eval(0)

    def select_actions(self, ep_batch, t_ep, t_env, bs=slice(None), test_mode=False, out=None):
        self.jumpstart_epsilon = self.jumpstart_eps_schedule.eval(t_env)
        if test_mode:
            self.jumpstart_epsilon = self.args.jumpstart_evaluation_epsilon
        if np.random.rand() < self.jumpstart_epsilon:
            return self.jumpstart_action_selector.select_action(ep_batch[bs, t_ep])
        return super().select_actions(ep_batch, t_ep, t_env, bs=bs, test_mode=test_mode, out=out)

    def forward(self, ep_batch, t, test_mode=False, action_selection_mode=False):
        agent_inputs = self._build_inputs(ep_batch, t)
        net = self.selector_agent if action_selection_mode else self.agent
        agent_outs, self.hidden_states = net(agent_inputs, self.hidden_states)
        if self.agent_output_type == "pi_logits":
            if getattr(self.args, "mask_before_softmax", True):
                avail = ep_batch["avail_actions"][:, t].reshape(ep_batch.batch_size * self.n, -1)
                agent_outs = agent_outs.masked_fill(avail == 0, -1e10)
            agent_outs = agent_outs.softmax(dim=-1)
        return agent_outs.view(ep_batch.batch_size, self.n, -1)
