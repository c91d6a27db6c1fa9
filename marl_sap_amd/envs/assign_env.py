"""The batched sequential-assignment environment on MI355X.

`AssignEnvBatch` owns E MockConstellationEnv episodes resident on one GPU (one C-ABI
handle, include/asg.h) and advances them all with one HIP kernel per call, writing
straight into an EpisodeBatch.  `MockConstellationEnv` is the reference's single-env
plugin surface (envs/mock_constellation_env.py:13-274) on top of a 1-env handle, for
callers that drive one env at a time.

Modes:
  rng="philox"  native: counter-based draws keyed (seed, global env index, episode);
                a 1-GPU and an 8-GPU run of the same global envs are bitwise identical.
  rng="mt19937" compat: each env replays numpy's legacy global stream exactly as
                np.random.seed(seed [+ env index]) followed by the reference's
                __init__ + reset draws (bit-exact benefit parameters, prev_assigns).
  benefits="bump" | "dense" | "injected" (sat_prox_mat=..., constant across episodes)
  quirks: prev_assigns_zero (the reference never writes the batch prev_assigns field),
          parallel_terminated (ParallelRunner's terminated-flag bug),
          replicate_stream (all ParallelRunner workers share one forked stream)
"""
import ctypes

import numpy as np
import torch

from .. import _lib
from ..components.transforms import OneHot
from .multiagentenv import MultiAgentEnv

_QUIRKS = {"prev_assigns_zero": _lib.ASG_QUIRK_PREV_ASSIGNS_ZERO,
           "parallel_terminated": _lib.ASG_QUIRK_PARALLEL_TERMINATED,
           "replicate_stream": _lib.ASG_QUIRK_REPLICATE_STREAM}

_VIEW_KEYS = ["obs", "actions", "avail_actions", "rewards", "terminated", "prev_assigns", "beta",
              "actions_onehot", "filled"]


def make_scheme(n, m, L, bids_as_actions=False):
    """Scheme + preprocess of the env (reference mock_constellation_env.py:67-92)."""
    obs_size = L * m + m
    scheme = {
        "obs": {"vshape": obs_size, "group": "agents", "dtype": torch.float32},
        "actions": {"vshape": (1,), "group": "agents", "dtype": torch.int64},
        "avail_actions": {"vshape": (m,), "group": "agents", "dtype": torch.bool},
        "rewards": {"vshape": (n,), "dtype": torch.float32},
        "terminated": {"vshape": (1,), "dtype": torch.bool},
        "prev_assigns": {"vshape": (n,), "dtype": torch.int64, "part_of_state": True},
        "beta": {"vshape": (n, m), "dtype": torch.float32, "part_of_state": True},
    }
    preprocess = {"actions": ("actions_onehot", [OneHot(out_dim=m)])}
    if bids_as_actions:
        scheme["actions"] = {"vshape": (m,), "group": "agents", "dtype": torch.float32}
        preprocess = {}
    return scheme, preprocess


def batch_view(data):
    """asg_batch_view over an EpisodeBatch (or a dict of its transition tensors)."""
    td = data.data.transition_data if hasattr(data, "data") else data
    v = _lib.AsgBatchView()
    for k in _VIEW_KEYS:
        setattr(v, k, _lib.field(td.get(k)))
    return v


class AssignEnvBatch(MultiAgentEnv):
    """E assignment-env episodes on one GPU, stepped in lockstep by HIP kernels."""

    def __init__(self, n, m, T, L, lambda_, bids_as_actions=False, seed=0, sat_prox_mat=None,
                 T_trans=None, num_envs=1, env_index_base=0, device=None, rng="philox",
                 benefits=None, quirks=()):
        if not torch.cuda.is_available():
            raise RuntimeError("AssignEnvBatch needs a ROCm GPU (HIP path only, no CPU fallback)")
        self.n, self.m, self.T, self.L, self.lambda_ = int(n), int(m), int(T), int(L), float(lambda_)
        self.bids_as_actions = bool(bids_as_actions)
        self.num_envs = int(num_envs)
        self.env_index_base = int(env_index_base)
        self.seed_value = 0 if seed is None else int(seed)
        self.device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
        self.rng = rng
        if benefits is None:
            benefits = "injected" if sat_prox_mat is not None else "bump"
        self.benefits = benefits
        self.quirks = tuple(quirks)
        self.T_trans = None if T_trans is None else np.ascontiguousarray(T_trans, dtype=np.float64)
        self._T_trans_dev = None if self.T_trans is None else torch.as_tensor(self.T_trans, device=self.device)
        self.obs_space_size = self.L * self.m + self.m
        self.scheme, self.preprocess = make_scheme(self.n, self.m, self.L, self.bids_as_actions)
        self.k = 0

        cfg = _lib.AsgConfig()
        cfg.num_envs, cfg.n, cfg.m, cfg.T, cfg.L = self.num_envs, self.n, self.m, self.T, self.L
        cfg.lambda_ = self.lambda_
        cfg.bids_as_actions = int(self.bids_as_actions)
        cfg.rng_mode = {"philox": _lib.ASG_RNG_PHILOX, "mt19937": _lib.ASG_RNG_MT19937}[rng]
        cfg.benefit_mode = {"bump": _lib.ASG_BENEFIT_BUMP, "dense": _lib.ASG_BENEFIT_DENSE,
                            "injected": _lib.ASG_BENEFIT_INJECTED}[benefits]
        cfg.quirks = sum(_QUIRKS[q] for q in self.quirks)
        cfg.seed = self.seed_value & 0xFFFFFFFFFFFFFFFF
        cfg.env_index_base = self.env_index_base
        self._tt_host = self.T_trans  # keep alive during create
        cfg.T_trans = (self._tt_host.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
                       if self._tt_host is not None else None)
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            _lib.check(_lib.lib().asg_create(ctypes.byref(cfg), self.device.index, _lib.stream_ptr(self.device),
                                             ctypes.byref(h)))
        self._h = h
        if sat_prox_mat is not None:
            self.set_benefits(sat_prox_mat)

    # ------------------------------------------------------------------ plumbing
    def _call(self, fn, *args):
        L = _lib.lib()
        with torch.cuda.device(self.device):
            L.asg_set_stream(self._h, _lib.stream_ptr(self.device))
            _lib.check(getattr(L, fn)(self._h, *args), self._h)

    def close(self):
        if getattr(self, "_h", None):
            _lib.lib().asg_destroy(self._h)
            self._h = None
        return True

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __len__(self):
        return self.num_envs

    def __getitem__(self, b):
        return _EnvView(self, b)

    # ------------------------------------------------------------------ hot path
    def reset(self, batch, ts=0):
        """New episode for every env; writes the pre-transition row `ts` of `batch`."""
        self._call("asg_reset", ctypes.byref(batch_view(batch)), int(ts))
        self.k = 0
        self._bids_token = None

    def step(self, batch, ts):
        """Reads actions at row ts; writes rewards/terminated/actions_onehot at ts and the
        next pre-transition row ts+1.  Returns the `done` flag (identical for all envs)."""
        self._call("asg_step_ex", ctypes.byref(batch_view(batch)), int(ts), self._bids_flags(batch, ts))
        self.k += 1
        return self.k >= self.T

    def _bids_flags(self, batch, ts):
        """ASG_STEP_USE_SELECTED_BIDS when batch row ts holds exactly the bids bids_select wrote:
        the same row (pointer, strides) and the actions tensor's version counter unchanged since
        (torch bumps it on every in-place write -- EpisodeBatch.update, slice assignment, copy_ --
        to any view of the tensor; the kernel's own write does not touch it).  Otherwise 0: the
        step solves the row as it is.  The token is spent by the step."""
        tok, self._bids_token = getattr(self, "_bids_token", None), None
        if not self.bids_as_actions or tok is None:
            return 0
        td = batch.data.transition_data if hasattr(batch, "data") else batch
        row = td["actions"][:, int(ts)]
        return _lib.ASG_STEP_USE_SELECTED_BIDS if tok == (row.data_ptr(), tuple(row.stride()), row._version) else 0

    def can_step_select(self, prefer=True, use_rnn=True, bids_ok=False):
        """Whether asg_rollout (env steps fused with the agent forward + epsilon-greedy
        selections, up to a whole episode per launch) takes this env: integer actions,
        16 <= m <= 256, n <= 256, L >= 1 -- with the GRU or the Linear RNNAgent -- and any
        benefit source: Philox bumps regenerated in the kernel, or the float32 table of the
        MT19937-compat / injected modes read for the lookahead rows.  `prefer` (kept for
        callers that ask whether it is also the faster schedule): measured on MI355X it is
        wherever it applies.  bids_ok: the caller's schedule is the bids one
        (asg_step_forward + asg_bids_select), which takes bids_as_actions envs with m <= 64."""
        if self.bids_as_actions and not (bids_ok and self.m <= 64):
            return False
        return _lib.lib().asg_rollout_l2_slices(self.n, self.m, self.L, int(bool(use_rnn))) >= 0

    @property
    def fused_reset_ok(self):
        """asg_reset_rollout (the reset inside the episode's launch) takes the Philox bump / dense
        modes and the MT19937 mode (its draw kernels, then the launch writes the reset row); an
        injected table under Philox resets with asg_reset."""
        return (self.rng == "philox" and self.benefits in ("bump", "dense")) or self.rng == "mt19937"

    def step_select(self, batch, ts, agent, hidden_state, epsilon, seed, counter, status):
        """asg_step at row ts and the fused agent forward + epsilon-greedy for row ts + 1 in
        one kernel: the observations of ts + 1 are written to the batch and consumed on the
        chip.  `agent` is the RNNFusedAgent; returns the new hidden state [E n, hidden].  Same
        batch, returns, actions and hidden state as env.step(batch, ts) followed by
        mac.select_actions(batch, ts + 1)."""
        return self.rollout(batch, ts, 1, agent, hidden_state, epsilon, seed, counter, status, select_first=False,
                            select_last=True)

    def reset_forward(self, batch, ts, agent, hidden_state, q_out=None):
        """asg_reset_forward: reset() and the agent forward on the reset row ts in one kernel
        (the row is written to the batch and consumed on chip) -- env.reset + mac.forward(0) for a
        selector acting on Q outside the kernel.  Needs fused_reset_ok.  Returns (Q [E n, m]
        float32, the new hidden state [E n, hidden])."""
        q_out, h_out, args = self._forward_args(batch, agent, hidden_state, q_out)
        self._call("asg_reset_forward", ctypes.byref(batch_view(batch)), int(ts), *args[:-1],
                   ctypes.c_void_p(h_out.data_ptr()), ctypes.c_void_p(q_out.data_ptr()), _lib.stream_ptr(self.device))
        self.k = 0
        self._bids_token = None
        return q_out, h_out

    def _forward_args(self, batch, agent, hidden_state, q_out):
        args = agent.step_select_args(hidden_state, batch["obs"].shape[-1], self.device, self.num_envs * self.n)
        R = self.num_envs * self.n
        if q_out is None or q_out.dtype != torch.float32 or q_out.numel() != R * self.m or not q_out.is_contiguous():
            q_out = torch.empty((R, self.m), dtype=torch.float32, device=self.device)
        return q_out, args[-1], args

    def step_forward(self, batch, ts, agent, hidden_state, q_out=None):
        """asg_step_forward: asg_step at row ts and the agent forward on row ts + 1 in one
        kernel (the observation row is written to the batch and consumed on chip) -- env.step
        + mac.forward for a selector that acts on Q outside the kernel (SAP).  Returns
        (Q [E n, m] float32, the new hidden state [E n, hidden])."""
        q_out, h_out, args = self._forward_args(batch, agent, hidden_state, q_out)
        self._call("asg_step_forward_ex", ctypes.byref(batch_view(batch)), int(ts), *args[:-1],
                   ctypes.c_void_p(h_out.data_ptr()), ctypes.c_void_p(q_out.data_ptr()), self._bids_flags(batch, ts),
                   _lib.stream_ptr(self.device))
        self.k += 1
        return q_out, h_out

    def bids_select(self, q, out, row_softmax, col_softmax, std, seed, counter, count_steps=None):
        """asg_bids_select: the bids of every env from the agent outputs q ([E n, m] or [E, n, m]
        float32) -- softmax over the tasks (row_softmax), over the agents (col_softmax), + N(0,
        std) -- written to `out` [E, n, m] float32 (the batch's actions row), and their
        LSA(maximize) assignments kept in the handle for the step on that row."""
        E, n, m = self.num_envs, self.n, self.m
        q = q.view(E, n, m)
        if q.dtype != torch.float32 or out.dtype != torch.float32 or tuple(out.shape) != (E, n, m):
            raise ValueError("bids_select: float32 q and out of shape [E, n, m]")
        if count_steps is not None:  # instrumentation (bench.py): int32 [E] augmenting-path steps
            self._call("asg_bids_select_count", ctypes.c_void_p(q.data_ptr()), _lib.i64arr(q.stride()),
                       ctypes.c_void_p(out.data_ptr()), _lib.i64arr(out.stride()), int(bool(row_softmax)),
                       int(bool(col_softmax)), float(std), int(seed) & 0xFFFFFFFFFFFFFFFF, int(counter),
                       ctypes.c_void_p(count_steps.data_ptr()), _lib.stream_ptr(self.device))
        else:
            self._call("asg_bids_select", ctypes.c_void_p(q.data_ptr()), _lib.i64arr(q.stride()),
                       ctypes.c_void_p(out.data_ptr()), _lib.i64arr(out.stride()), int(bool(row_softmax)),
                       int(bool(col_softmax)), float(std), int(seed) & 0xFFFFFFFFFFFFFFFF, int(counter),
                       _lib.stream_ptr(self.device))
        self._bids_token = (out.data_ptr(), tuple(out.stride()), out._version)
        return out

    def rollout(self, batch, ts, steps, agent, hidden_state, epsilon, seed, counter, status, select_first=True,
                select_last=False, reset=False):
        """asg_rollout: `steps` env transitions from the current step (batch rows ts ..) with
        the agent forward + epsilon-greedy selections in between, in one kernel --
        select_first: also the selection on the reset row ts (k == 0); select_last: also the
        selection after the last transition.  The selections use Philox counters counter,
        counter + 1, ... in row order.  Returns the hidden state after the last selection
        [E n, hidden] (the MAC's hidden_states).  A whole episode after reset():
        rollout(batch, 0, T, ...); reset=True folds that reset() into the same launch
        (asg_reset_rollout; implies select_first)."""
        args = agent.step_select_args(hidden_state, batch["obs"].shape[-1], self.device, self.num_envs * self.n)
        h_out = args[-1]
        tail = (*args[:-1], ctypes.c_void_p(h_out.data_ptr()), float(epsilon), seed & 0xFFFFFFFFFFFFFFFF, int(counter),
                ctypes.c_void_p(status.data_ptr()), _lib.stream_ptr(self.device))
        self._bids_token = None
        if reset and not self.fused_reset_ok:
            self.reset(batch, ts)  # table modes: asg_reset, then the episode from the reset row
            reset, select_first = False, True
        if reset:
            self._call("asg_reset_rollout", ctypes.byref(batch_view(batch)), int(ts), int(steps),
                       int(bool(select_last)), *tail)
            self.k = int(steps)
        else:
            self._call("asg_rollout", ctypes.byref(batch_view(batch)), int(ts), int(steps), int(bool(select_first)),
                       int(bool(select_last)), *tail)
            self.k += int(steps)
        return h_out

    def random_actions(self, batch, ts):
        self._call("asg_random_actions", ctypes.byref(batch_view(batch)), int(ts))

    def random_rollout(self, batch, ts, steps, reset=False):
        """The uniform random policy's next `steps` steps in one launch (asg_random_rollout):
        random_actions(ts + s) + step(ts + s) for s < steps, after reset(ts) when `reset` --
        bit-identical to those separate calls.  The MT19937 mode's reset is asg_reset (its stream's
        draw kernels) followed by the launch."""
        self._bids_token = None
        if reset and self.rng == "mt19937":
            self.reset(batch, ts)
            reset = False
        self._call("asg_random_rollout", ctypes.byref(batch_view(batch)), int(ts), int(steps), int(bool(reset)))
        self.k = (0 if reset else self.k) + int(steps)
        return self.k >= self.T

    def sync(self):
        """Block on the env's stream and raise the first sticky device error, if any."""
        self._call("asg_sync_status")

    def get_returns(self):
        out = torch.empty(self.num_envs, dtype=torch.float64, device=self.device)
        self._call("asg_get_returns", ctypes.c_void_p(out.data_ptr()))
        return out

    def set_benefits(self, table):
        t = torch.as_tensor(np.asarray(table, dtype=np.float64) if not torch.is_tensor(table) else table,
                            dtype=torch.float64)
        if t.dim() == 3:
            t = t.unsqueeze(0)
        t = t.to(self.device).contiguous()
        self._benefit_keepalive = t
        self._call("asg_set_benefits", ctypes.c_void_p(t.data_ptr()), t.numel(), 1)

    def export_benefits(self):
        """Current episode's benefit table [E, n, m, T] float64 (reference layout)."""
        out = torch.empty((self.num_envs, self.n, self.m, self.T), dtype=torch.float64, device=self.device)
        self._call("asg_export_benefits", ctypes.c_void_p(out.data_ptr()))
        return out

    def export_bump_params(self):
        """Philox modes: float32 [E, n, m, 3] (scale, center, a) of the current episode."""
        out = torch.empty((self.num_envs, self.n, self.m, 3), dtype=torch.float32, device=self.device)
        self._call("asg_export_bump_params", ctypes.c_void_p(out.data_ptr()))
        return out

    def export_prev_assigns(self):
        out = torch.empty((self.num_envs, self.n), dtype=torch.int64, device=self.device)
        self._call("asg_export_prev_assigns", ctypes.c_void_p(out.data_ptr()))
        return out

    def advance_stream(self, words):
        self._call("asg_advance_stream", int(words))

    # ------------------------------------------------------------------ env surface
    def beta_hat(self, beta, prev_assigns):
        """MockConstellationEnv.beta_hat (mock :228-274) for any leading batch dims, on
        the GPU; returns float64 like the reference."""
        beta_t = torch.as_tensor(beta, device=self.device)
        prev_t = torch.as_tensor(prev_assigns, device=self.device, dtype=torch.int64)
        if beta_t.dtype not in (torch.float32, torch.float64):
            beta_t = beta_t.to(torch.float64)
        lead = beta_t.shape[:-2]
        b3 = beta_t.reshape(-1, self.n, self.m)
        p2 = prev_t.reshape(-1, self.n)
        if p2.shape[0] != b3.shape[0]:
            raise ValueError("beta and prev_assigns batch dims differ")
        out = torch.empty(b3.shape, dtype=torch.float64, device=self.device)
        with torch.cuda.device(self.device):
            _lib.check(_lib.lib().asg_beta_hat(
                ctypes.c_void_p(b3.data_ptr()), _lib.dtype_code(b3.dtype), _lib.i64arr(b3.stride()),
                ctypes.c_void_p(p2.data_ptr()), _lib.i64arr(p2.stride()), b3.shape[0], self.n, self.m,
                ctypes.c_void_p(self._T_trans_dev.data_ptr()) if self._T_trans_dev is not None else None,
                self.lambda_, ctypes.c_void_p(out.data_ptr()), _lib.stream_ptr(self.device)))
        return out.reshape(*lead, self.n, self.m)

    def get_obs_size(self):
        return self.obs_space_size

    def get_state_size(self):
        return self.n * self.obs_space_size

    def get_total_actions(self):
        return self.m

    def get_stats(self):
        return {}

    def get_env_info(self):
        return {"state_shape": self.get_state_size(), "obs_shape": self.get_obs_size(),
                "m": self.get_total_actions(), "n": self.n, "T": self.T}

    def save_replay(self):
        pass

    def render(self):
        pass


class _EnvView:
    """One env of a batch, as the selectors see `self.envs[b]` (non_rl_selectors.py:39)."""

    def __init__(self, batch_env, b):
        self._env, self.b = batch_env, b
        self.n, self.m, self.T, self.L = batch_env.n, batch_env.m, batch_env.T, batch_env.L
        self.lambda_, self.T_trans = batch_env.lambda_, batch_env.T_trans

    @property
    def k(self):
        return self._env.k

    def beta_hat(self, beta, prev_assigns):
        return self._env.beta_hat(beta, prev_assigns)


class MockConstellationEnv(MultiAgentEnv):
    """The reference's single-env plugin (envs/mock_constellation_env.py:13-274) on a
    1-env GPU handle.  `stream_seed` plays numpy's global seed in rng="mt19937" mode
    (np.random.seed(s) before constructing the reference env)."""

    def __init__(self, n, m, T, L, lambda_, bids_as_actions=False, seed=None, sat_prox_mat=None,
                 T_trans=None, stream_seed=None, rng="mt19937", device=None):
        self.n, self.m, self.T, self.L, self.lambda_ = n, m, T, L, lambda_
        self._seed = seed
        self.bids_as_actions = bool(bids_as_actions)
        self.constant_benefits = sat_prox_mat is not None
        s = stream_seed if stream_seed is not None else (seed if seed is not None else 0)
        self._batch = AssignEnvBatch(n, m, T, L, lambda_, bids_as_actions=bids_as_actions, seed=s,
                                     sat_prox_mat=sat_prox_mat, T_trans=T_trans, num_envs=1, device=device,
                                     rng=rng, quirks=("prev_assigns_zero",))
        self.scheme, self.preprocess = self._batch.scheme, self._batch.preprocess
        self.obs_space_size = self._batch.obs_space_size
        self.T_trans = self._batch.T_trans if T_trans is not None else np.ones((m, m)) - np.eye(m)
        dev = self._batch.device
        W = self.obs_space_size
        amshape = (1, T + 1, n, m) if self.bids_as_actions else (1, T + 1, n, 1)
        adt = torch.float32 if self.bids_as_actions else torch.int64
        self._td = {
            "obs": torch.zeros((1, T + 1, n, W), dtype=torch.float32, device=dev),
            "actions": torch.zeros(amshape, dtype=adt, device=dev),
            "avail_actions": torch.zeros((1, T + 1, n, m), dtype=torch.bool, device=dev),
            "rewards": torch.zeros((1, T + 1, n), dtype=torch.float32, device=dev),
            "terminated": torch.zeros((1, T + 1, 1), dtype=torch.bool, device=dev),
            "prev_assigns": torch.zeros((1, T + 1, n), dtype=torch.int64, device=dev),
            "beta": torch.zeros((1, T + 1, n, m), dtype=torch.float32, device=dev),
            "filled": torch.zeros((1, T + 1, 1), dtype=torch.int64, device=dev),
        }
        self.k = 0

    @property
    def sat_prox_mat(self):
        return self._batch.export_benefits()[0].cpu().numpy()

    @property
    def prev_assigns(self):
        return self._batch.export_prev_assigns()[0].cpu().numpy()

    @property
    def beta(self):
        return self._td["beta"][0, self.k].double().cpu().numpy()

    @property
    def _obs(self):
        return list(self._td["obs"][0, self.k].double().cpu().numpy())

    def reset(self):
        self._batch.reset(self._td, 0)
        self.k = 0
        return self.get_obs(), self.get_state()

    def step(self, actions):
        if self.k >= self.T:
            raise ValueError("step after the episode ended (k >= T)")
        if self.bids_as_actions:
            a = torch.as_tensor(np.asarray(actions, dtype=np.float32)).reshape(self.n, self.m)
        else:
            a = torch.as_tensor(np.asarray(actions, dtype=np.int64)).reshape(self.n, 1)
        self._td["actions"][0, self.k].copy_(a)
        ts = self.k
        done = self._batch.step(self._td, ts)
        self._batch.sync()
        self.k += 1
        rewards = self._td["rewards"][0, ts].double().cpu().tolist()
        return rewards, done, {}

    def get_pretransition_data(self):
        return {"obs": [self._obs], "avail_actions": [self.get_avail_actions()], "beta": [self.beta]}

    def beta_hat(self, beta, prev_assigns):
        out = self._batch.beta_hat(beta, prev_assigns)
        return out.cpu().numpy()

    def get_obs(self):
        return self._obs

    def get_obs_agent(self, agent_id):
        return self._obs[agent_id]

    def get_obs_size(self):
        return self.obs_space_size

    def get_state(self):
        return np.concatenate(self._obs, axis=0).astype(np.float32)

    def get_state_size(self):
        return self.n * self.obs_space_size

    def get_avail_actions(self):
        return [self.get_avail_agent_actions(i) for i in range(self.n)]

    def get_avail_agent_actions(self, agent_id):
        return [1] * self.m

    def get_total_actions(self):
        return self.m

    def get_stats(self):
        return {}

    def seed(self, seed=None):
        self._seed = seed

    def close(self):
        self._batch.close()
        return True

    def save_replay(self):
        pass

    def render(self):
        pass
