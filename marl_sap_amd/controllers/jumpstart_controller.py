"""Jumpstart controller (reference: controllers/jumpstart_controller.py:10-121): with
probability jumpstart_epsilon (one numpy coin flip per selection for the whole batch, drawn
from numpy's global stream like the reference) the non-RL selector (HAA) acts.

When the RL MAC fuses (the RNNAgent + epsilon-greedy: mock_constellation_iql.yaml; or
the RNNAgent forward + the SAP selector: mock_constellation_reda.yaml) the GPU runner draws an episode's coin flips when it plans the episode (fused_mode), in the
reference's order (one per select_actions call, t = 0, 1, ...): the epsilon-greedy selector
draws nothing from numpy's global stream, so the stream is consumed exactly as the
reference's per-step draws consume it.  When every flip picks the RL branch the episode is
one asg_rollout kernel; otherwise the RL steps still fuse env.step(t) with
select_actions(t + 1) (SAP: with the agent forward of t + 1, the LSA kernel after it), and the
HAA steps run env.step + the HAA selector.  Any other RL
selector may draw from the same stream itself (EpsilonGreedySAPTestActionSelector,
sap_selectors.py:36): then nothing is pre-drawn and each select_actions draws its flip when
it runs, interleaved with the selector's draws as in the reference."""
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
        self._flips = []  # pre-drawn coin flips of the planned episode (True: the jumpstart selector acts)

    def _eps(self, t_env, test_mode):
        self.jumpstart_epsilon = self.jumpstart_eps_schedule.eval(t_env)
        if test_mode:
            self.jumpstart_epsilon = self.args.jumpstart_evaluation_epsilon
        return self.jumpstart_epsilon

    def _coin(self, t_env, test_mode):
        eps = self._eps(t_env, test_mode)
        if self._flips:
            return self._flips.pop(0)
        return np.random.rand() < eps

    def select_actions(self, ep_batch, t_ep, t_env, bs=slice(None), test_mode=False, out=None):
        if self._coin(t_env, test_mode):
            return self.jumpstart_action_selector.select_action(ep_batch[bs, t_ep])
        return super().select_actions(ep_batch, t_ep, t_env, bs=bs, test_mode=test_mode, out=out)

    def fused_mode(self, env, ep_batch, t_env=0, test_mode=False):
        """When the RL MAC fuses (its selector is epsilon-greedy or the fused SAP selector,
        neither of which draws from numpy's global stream): draw the episode's T coin flips now (the reference's order);
        "episode" when every one picks the RL branch, else "step" (the RL steps' env.step +
        selection fused).  Otherwise None, and no flip is pre-drawn: each select_actions
        draws its own, interleaved with the RL selector's draws as in the reference."""
        base = super().fused_mode(env, ep_batch, t_env, test_mode)
        if base is None:
            self._flips = []
            return None
        eps = self._eps(t_env, test_mode)
        self._flips = list(np.random.rand(env.T) < eps)
        if base == "step_q":
            return base  # per step either way; the SAP selector's noise is Philox, not numpy
        return "episode" if base == "episode" and not any(self._flips) else "step"

    def fused_episode(self, env, ep_batch, t_env, test_mode=False, reset=False):
        self._flips = []  # all RL: consumed by the one kernel
        super().fused_episode(env, ep_batch, t_env, test_mode, reset=reset)

    def fused_step_select(self, env, ep_batch, t_ep, t_env, test_mode=False):
        """env.step(t) and select_actions(t + 1): one kernel when the flip for t + 1 picks the
        RL branch, else env.step then the jumpstart selector on row t + 1."""
        if not self._coin(t_env, test_mode):
            return super().fused_step_select(env, ep_batch, t_ep, t_env, test_mode)
        env.step(ep_batch, ts=t_ep)
        acts = self.jumpstart_action_selector.select_action(ep_batch[:, t_ep + 1])
        ep_batch.update({"actions": acts}, ts=t_ep + 1, mark_filled=False, preprocess=False)

    def fused_reset_select(self, env, ep_batch, t_env, test_mode=False):
        """env.reset() + select_actions(0): the fused reset + forward when the flip for row 0 picks
        the RL branch, else env.reset then the jumpstart selector."""
        if not self._coin(t_env, test_mode):
            return super().fused_reset_select(env, ep_batch, t_env, test_mode)
        env.reset(ep_batch, ts=0)
        acts = self.jumpstart_action_selector.select_action(ep_batch[:, 0])
        ep_batch.update({"actions": acts}, ts=0, mark_filled=False, preprocess=False)

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
