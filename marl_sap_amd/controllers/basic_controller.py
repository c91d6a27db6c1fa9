"""Shared-parameter multi-agent controller (reference: controllers/basic_controller.py:7-101).

The reference keeps a CPU copy (`selector_agent`) for action selection.  Here the agent
lives on the GPU next to the batched env, so by default selection uses the agent itself
(`selector_agent` is the same module); with args.separate_selector_agent=True a distinct
copy is kept and `update_action_selector_agent` syncs it, as in the reference.
"""
import torch

from ..action_selectors import REGISTRY as action_REGISTRY
from ..modules.agents import REGISTRY as agent_REGISTRY


def _accepts_out(selector):
    import inspect
    try:
        return "out" in inspect.signature(selector.select_action).parameters
    except (TypeError, ValueError):
        return False


class BasicMAC:
    def __init__(self, scheme, groups, args):
        self.n = args.n
        self.args = args
        input_shape = self._get_input_shape(scheme)
        self._build_agents(input_shape)
        self.agent_output_type = args.agent_output_type
        self.action_selector = action_REGISTRY[args.action_selector](args)
        self.hidden_states = None

    def select_actions(self, ep_batch, t_ep, t_env, bs=slice(None), test_mode=False, out=None):
        """`out` (optional, int64 [B, n]): selectors that support it write the actions
        there in place (the runner passes the EpisodeBatch actions row)."""
        avail_actions = ep_batch["avail_actions"][:, t_ep]
        if out is not None and out.dtype == torch.float32 and self._fused_bids_ok(bs, out):
            # bids_as_actions: the agent's raw outputs -> asg_bids_select (pi_logits softmax,
            # the selector's softmax over agents + noise, the bids row, their LSA)
            q, self.hidden_states = self.selector_agent(self._build_inputs(ep_batch, t_ep), self.hidden_states)
            return self.action_selector.fused_bids(q.view(ep_batch.batch_size, self.n, -1), out, t_env, test_mode,
                                                   row_softmax=self.agent_output_type == "pi_logits")
        if out is not None and out.dtype != torch.int64:
            out = None  # e.g. the real env's int16 actions: the caller casts through update()
        if out is not None and self._fused_select_ok(bs):
            # agent forward + epsilon-greedy in one HIP kernel: Q never leaves the chip
            eps, seed, counter, status, base = self.action_selector.fused_params(t_env, test_mode, out.device)
            self.hidden_states = self.selector_agent.forward_select(
                self._build_inputs(ep_batch, t_ep), self.hidden_states, avail_actions, self.n, eps, seed, counter,
                out, status, env_index_base=base)
            return out
        agent_outputs = self.forward(ep_batch, t_ep, test_mode=test_mode, action_selection_mode=True)
        if t_ep == 0 and hasattr(self.action_selector, "episode_start"):
            self.action_selector.episode_start()
        kw = {"out": out} if out is not None and _accepts_out(self.action_selector) else {}
        return self.action_selector.select_action(agent_outputs[bs], avail_actions[bs], t_env,
                                                  test_mode=test_mode, beta=ep_batch["beta"][bs, t_ep], **kw)

    def _fused_select_ok(self, bs):
        from ..action_selectors.classic_selectors import EpsilonGreedyActionSelector
        from ..modules.agents.rnn_agent import RNNFusedAgent
        return (not torch.is_grad_enabled() and isinstance(bs, slice) and bs == slice(None)
                and self.agent_output_type == "q" and type(self.action_selector) is EpsilonGreedyActionSelector
                and isinstance(self.selector_agent, RNNFusedAgent)
                and not getattr(self.args, "unfused_selection", False))

    def _fused_q_ok(self):
        """The REDA selector (SequentialAssignmentProblemSelector, n <= m <= 64: its fused
        noise + LSA kernel) acts on the agent's Q outside the rollout kernel: the env step and
        the agent forward fuse (asg_step_forward), the selection stays a separate launch."""
        from ..action_selectors.sap_selectors import SequentialAssignmentProblemSelector
        from ..modules.agents.rnn_agent import RNNFusedAgent
        return (not torch.is_grad_enabled() and self.agent_output_type == "q"
                and type(self.action_selector) is SequentialAssignmentProblemSelector
                and isinstance(self.selector_agent, RNNFusedAgent) and self.n <= self.selector_agent.n_out <= 64
                and not getattr(self.args, "unfused_selection", False))

    def _fused_bids_ok(self, bs=slice(None), out=None):
        """bids_as_actions with the ContinuousActionSelector on the batched env (n <= m <= 64):
        asg_bids_select turns the agent's raw outputs into the bids row and its LSA."""
        from ..action_selectors.bet_selectors import ContinuousActionSelector
        from ..modules.agents.rnn_agent import RNNFusedAgent
        env = getattr(self.action_selector, "envs", None)
        ok = (not torch.is_grad_enabled() and isinstance(bs, slice) and bs == slice(None)
              and type(self.action_selector) is ContinuousActionSelector
              and self.agent_output_type in ("pi_logits", "q") and getattr(env, "bids_as_actions", False)
              and hasattr(env, "bids_select") and isinstance(self.selector_agent, RNNFusedAgent)
              and self.n <= self.selector_agent.n_out <= 64 and self.selector_agent.n_out == getattr(env, "m", -1)
              and not getattr(self.args, "unfused_selection", False))
        if ok and out is not None:
            ok = tuple(out.shape) == (env.num_envs, self.n, env.m) and out.device == env.device
        return ok

    def _fused_kind(self, env, ep_batch):
        """"select" (the selection runs in the rollout kernel: epsilon-greedy), "q" (the kernel
        writes Q for the SAP selector), "bids" (Q for asg_bids_select) or None."""
        from ..modules.agents.rnn_agent import RNNFusedAgent
        mode = getattr(self.args, "fused_rollout", True)
        if not mode:
            return None
        kind = "select" if self._fused_select_ok(slice(None)) else ("q" if self._fused_q_ok() else None)
        if kind is None and self._fused_bids_ok():
            kind = "bids"
        ok = (kind is not None and hasattr(env, "can_step_select")
              and env.can_step_select(prefer=(mode != "always"), use_rnn=bool(self.args.use_rnn),
                                      bids_ok=kind == "bids")
              and getattr(ep_batch, "time_major", False) and not self.args.obs_last_action
              and not self.args.obs_agent_id and isinstance(self.selector_agent, RNNFusedAgent)
              and self.selector_agent.n_out == env.m)
        return kind if ok else None

    def fused_step_ok(self, env, ep_batch):
        """The runner may fuse env.step(t) with select_actions(t + 1) (asg_rollout): the fused
        agent (GRU or Linear RNNAgent) + epsilon-greedy selection -- or, for the SAP selector,
        env.step(t) with the agent forward of t + 1 (asg_step_forward) -- on plain observation
        inputs, a time-major batch and an env that takes it.  args.fused_rollout: True /
        "episode" / "always" (default: a whole episode per launch), "step" (one launch per
        step), False (separate env-step and agent launches)."""
        return self._fused_kind(env, ep_batch) is not None

    def fused_mode(self, env, ep_batch, t_env=0, test_mode=False):
        """How the runner schedules this episode: "episode" (asg_rollout over all T steps),
        "step" (asg_rollout per step), "step_q" (asg_step_forward + the SAP selection per
        step) or None (separate launches)."""
        kind = self._fused_kind(env, ep_batch)
        if kind is None:
            return None
        if kind in ("q", "bids"):
            return "step_q"
        return "step" if getattr(self.args, "fused_rollout", True) == "step" else "episode"

    def fused_step_select(self, env, ep_batch, t_ep, t_env, test_mode=False):
        """env.step at row t_ep and select_actions for row t_ep + 1 in one kernel; the
        hidden state advances as select_actions would advance it.  SAP selector: the kernel
        ends with the agent's Q (kept in one reused buffer), which the selector's kernel turns
        into the actions of row t_ep + 1, written in place."""
        if self._fused_bids_ok() or self._fused_q_ok():
            q, self.hidden_states = env.step_forward(ep_batch, t_ep, self.selector_agent, self.hidden_states,
                                                     q_out=getattr(self, "_q_buf", None))
            self._select_on_q(q, ep_batch, t_ep + 1, t_env, test_mode)
            return
        eps, seed, counter, status, _base = self.action_selector.fused_params(t_env, test_mode, env.device)
        self.hidden_states = env.step_select(ep_batch, t_ep, self.selector_agent, self.hidden_states, eps, seed,
                                             counter, status)

    def _select_on_q(self, q, ep_batch, t, t_env, test_mode):
        """The step_q schedule's selection on the agent outputs q [B n, m] of row t (kept in one
        reused buffer): SAP -- its noise + LSA kernel, actions into the batch row in place; bids --
        asg_bids_select (the bids row and its LSA)."""
        self._q_buf = q
        B = ep_batch.batch_size
        if t == 0 and hasattr(self.action_selector, "episode_start"):
            self.action_selector.episode_start()
        if self._fused_bids_ok():
            self.action_selector.fused_bids(q.view(B, self.n, -1), ep_batch["actions"][:, t], t_env, test_mode,
                                            row_softmax=self.agent_output_type == "pi_logits")
            return
        row = ep_batch["actions"][:, t, :, 0]
        acts = self.action_selector.select_action(q.view(B, self.n, -1), ep_batch["avail_actions"][:, t], t_env,
                                                  test_mode=test_mode, beta=ep_batch["beta"][:, t], out=row)
        if acts is not row:
            ep_batch.update({"actions": acts}, ts=t, mark_filled=False, preprocess=False)

    def fused_reset_ok(self, env):
        """The step_q schedule may fold env.reset() into the forward on the reset row
        (asg_reset_forward): the env's reset runs inside a launch (Philox bump / dense, MT19937)."""
        return (getattr(env, "fused_reset_ok", False) and hasattr(env, "reset_forward")
                and (self._fused_bids_ok() or self._fused_q_ok()))

    def fused_reset_select(self, env, ep_batch, t_env, test_mode=False):
        """env.reset() + select_actions(0) on the step_q schedule: the reset and the agent forward
        on the reset row in one launch (asg_reset_forward), then the selector's kernel on its Q --
        the batch, hidden state and actions of the separate calls."""
        q, self.hidden_states = env.reset_forward(ep_batch, 0, self.selector_agent, self.hidden_states,
                                                  q_out=getattr(self, "_q_buf", None))
        self._select_on_q(q, ep_batch, 0, t_env, test_mode)

    def fused_episode(self, env, ep_batch, t_env, test_mode=False, reset=False):
        """select_actions(0), then env.step(t) + select_actions(t + 1) for the whole episode
        (the last step without a selection after it) in ONE kernel launch; selector counters
        and the hidden state advance as T select_actions calls would advance them.  reset:
        the env's reset() runs in the same launch (the runner then skips it)."""
        T = env.T
        eps, seed, counter, status, _base = self.action_selector.fused_params(t_env, test_mode, env.device, calls=T)
        self.hidden_states = env.rollout(ep_batch, 0, T, self.selector_agent, self.hidden_states, eps, seed, counter,
                                         status, select_first=True, select_last=False, reset=reset)

    def forward(self, ep_batch, t, test_mode=False, action_selection_mode=False):
        agent_inputs = self._build_inputs(ep_batch, t)
        net = self.selector_agent if action_selection_mode else self.agent
        agent_outs, self.hidden_states = net(agent_inputs, self.hidden_states)
        if self.agent_output_type == "pi_logits":
            agent_outs = torch.nn.functional.softmax(agent_outs, dim=-1)
        return agent_outs.view(ep_batch.batch_size, self.n, -1)

    def init_hidden(self, batch_size):
        self.hidden_states = self.agent.init_hidden().unsqueeze(0).expand(batch_size, self.n, -1)

    def parameters(self):
        return self.agent.parameters()

    def load_state(self, other_mac):
        self.agent.load_state_dict(other_mac.agent.state_dict())

    def cuda(self):
        self.agent.cuda()
        if self.selector_agent is not self.agent:
            self.selector_agent.cuda()

    def to(self, device):
        self.agent.to(device)
        if self.selector_agent is not self.agent:
            self.selector_agent.to(device)
        return self

    def save_models(self, path):
        torch.save(self.agent.state_dict(), "{}/agent.th".format(path))

    def load_models(self, path):
        self.agent.load_state_dict(torch.load("{}/agent.th".format(path), map_location=lambda s, loc: s,
                                              weights_only=True))
        self.update_action_selector_agent()

    def _build_agents(self, input_shape):
        self.agent = agent_REGISTRY[self.args.agent](input_shape, self.args)
        if getattr(self.args, "separate_selector_agent", False):
            self.selector_agent = agent_REGISTRY[self.args.agent](input_shape, self.args)
        else:
            self.selector_agent = self.agent

    def update_action_selector_agent(self):
        if self.selector_agent is not self.agent:
            self.selector_agent.load_state_dict(self.agent.state_dict())

    def _build_inputs(self, batch, t):
        bs = batch.batch_size
        inputs = [batch["obs"][:, t].float()]
        if self.args.obs_last_action:
            if t == 0:
                inputs.append(torch.zeros_like(batch["actions_onehot"][:, t]))
            else:
                inputs.append(batch["actions_onehot"][:, t - 1])
        if self.args.obs_agent_id:
            inputs.append(torch.eye(self.n, device=batch.device).unsqueeze(0).expand(bs, -1, -1))
        if len(inputs) == 1:
            return inputs[0].reshape(bs * self.n, -1)
        return torch.cat([x.reshape(bs * self.n, -1).to(torch.float32) for x in inputs], dim=1)

    def _get_input_shape(self, scheme):
        input_shape = scheme["obs"]["vshape"]
        if self.args.obs_last_action:
            input_shape += scheme["actions_onehot"]["vshape"][0]
        if self.args.obs_agent_id:
            input_shape += self.n
        return input_shape
