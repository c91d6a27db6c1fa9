"""GPU vectorised rollout runner: drop-in for EpisodeRunner / ParallelRunner
(reference: runners/episode_runner.py:8-137, runners/parallel_runner.py:12-243).

Constructed as GpuVecRunner(args, logger) and used exactly like the reference runners
(get_env / setup / run / t_env / close_env / save_replay).  Instead of one OS process and
one pickled Pipe round-trip per env per step, all `batch_size_run` envs of this rank live
in HBM behind one C-ABI handle and every step is:

    mac.select_actions (PyTorch-ROCm)  ->  actions row write  ->  asg_step (one HIP kernel)

or, with the fused RNN agent and epsilon-greedy, the whole episode in one asg_rollout
kernel -- with the EpisodeBatch kept resident on the GPU in time-major storage.  Under
torch.distributed (one process per GPU, RCCL) each rank owns the contiguous global envs
[sum(E_<r), sum(E_<r) + E_r) -- [rank*E, (rank+1)*E) for equal shards; the rank env counts
are all-gathered once at construction, so the env-step counter of an episode is
T * sum_r E_r on every rank without a per-episode collective.  The only per-episode
collective is an all-gather of the float64 episode returns.

Protocols (args.runner_protocol):
  "episode"  EpisodeRunner semantics per env: T selection passes, true terminated flag,
             row T actions left 0.
  "parallel" ParallelRunner semantics: one extra selection pass at t = T writing row T
             actions (+ one-hot), and its terminated-flag quirk when args.env_quirks
             contains "parallel_terminated".
"""

import numpy as np
import torch

from .. import dist as asg_dist
from ..components.episode_buffer import EpisodeBatch
from ..envs import BATCHED_REGISTRY


class GpuVecRunner:
    def __init__(self, args, logger):
        self.args = args
        self.logger = logger
        self.batch_size = args.batch_size_run
        self.rank, self.world = asg_dist.rank_world()
        self.device = torch.device("cuda", torch.cuda.current_device())
        self.rank_envs = asg_dist.envs_per_rank(self.batch_size)
        self.global_envs = sum(self.rank_envs)
        env_args = dict(args.env_args)
        env_args.pop("seed", None)
        self.env = BATCHED_REGISTRY[args.env](
            **env_args, seed=args.env_args.get("seed", 0) or 0, num_envs=self.batch_size,
            env_index_base=asg_dist.env_index_base(self.rank_envs, self.rank), device=self.device,
            rng=getattr(args, "env_rng", "philox"), quirks=tuple(getattr(args, "env_quirks", ())))
        self.T = self.env.T
        self.protocol = getattr(args, "runner_protocol", "episode")
        # reuse_batch: one EpisodeBatch allocated once and overwritten by every run() (the
        # throughput loops opt in); off by default, so run() returns a fresh batch per
        # episode as the reference runners' new_batch() does
        self.reuse_batch = getattr(args, "reuse_batch", False)
        self.t = 0
        self.t_env = 0
        self.train_returns, self.test_returns = [], []
        self.train_stats, self.test_stats = {}, {}
        self.log_train_stats_t = -1000000
        self.last_returns = None  # device tensor of the last episode's (gathered) returns
        self.batch = None
        self._pending, self._pending_steps = [], []  # finished episodes awaiting flush_pending()

    # ------------------------------------------------------------------ plugin surface
    def setup(self, scheme, groups, preprocess, mac):
        self.scheme, self.groups, self.preprocess = scheme, groups, preprocess
        self.mac = mac
        self.mac.action_selector.envs = self.env
        if hasattr(self.mac, "jumpstart_action_selector"):
            self.mac.jumpstart_action_selector.envs = self.env

    def new_batch(self):
        return EpisodeBatch(self.scheme, self.groups, self.batch_size, self.T + 1, preprocess=self.preprocess,
                            device=self.device, time_major=True)

    def get_env_info(self):
        return self.env.get_env_info()

    def get_env(self):
        return self.env

    def save_replay(self):
        self.env.save_replay()

    def close_env(self):
        self.env.close()

    def reset(self, env_reset=True):
        if self.batch is None or not self.reuse_batch:
            self.batch = self.new_batch()
        if env_reset:
            self.env.reset(self.batch, ts=0)
        self.t = 0

    # ------------------------------------------------------------------ rollout
    @torch.no_grad()
    def rollout(self, test_mode=False):
        """One episode of every env, fully asynchronous (no host sync).  When the MAC and env
        allow it the whole loop -- select(0); for t: env.step(t), select(t + 1) -- is ONE
        kernel (asg_rollout, mode "episode"), or one kernel per step ("step"; "step_q": the
        env step + agent forward kernel, then the SAP selection kernel): the observations are
        generated on chip and never re-read, and the batch is the separate launches' bit for
        bit."""
        self.reset(env_reset=False)
        self.mac.init_hidden(batch_size=self.batch_size)
        mode = self.mac.fused_mode(self.env, self.batch, self.t_env, test_mode) \
            if hasattr(self.mac, "fused_mode") else None
        if mode == "episode":
            # the env reset runs in the episode's launch (asg_reset_rollout)
            self.mac.fused_episode(self.env, self.batch, self.t_env, test_mode, reset=True)
        else:
            if mode == "step_q" and self.mac.fused_reset_ok(self.env):
                # the reset and the forward on its row in one launch, then the selector's kernel
                self.mac.fused_reset_select(self.env, self.batch, self.t_env, test_mode)
            else:
                self.env.reset(self.batch, ts=0)
                self.select_into_batch(0, test_mode)
            for t in range(self.T):
                if mode in ("step", "step_q") and t + 1 < self.T:
                    self.mac.fused_step_select(self.env, self.batch, t, self.t_env, test_mode)
                    continue
                self.env.step(self.batch, ts=t)
                if t + 1 < self.T:
                    self.select_into_batch(t + 1, test_mode)
        self.t = self.T
        if self.protocol == "parallel":
            actions = self.mac.select_actions(self.batch, t_ep=self.T, t_env=self.t_env, test_mode=test_mode)
            self.batch.update({"actions": actions}, ts=self.T, mark_filled=False)
        return self.batch

    def select_into_batch(self, t, test_mode=False):
        """mac.select_actions at t_ep = t, actions written into the batch row t (in place
        when the selector supports `out`, else through EpisodeBatch.update)."""
        # the actions row: int64 [B, n]; bids_as_actions: the float32 bids [B, n, m]
        row = self.batch["actions"][:, t] if self.env.bids_as_actions else self.batch["actions"][:, t, :, 0]
        actions = self.mac.select_actions(self.batch, t_ep=t, t_env=self.t_env, test_mode=test_mode, out=row)
        if row is None or actions is not row:
            self.batch.update({"actions": actions}, ts=t, mark_filled=False, preprocess=False)

    def finish_episode(self, test_mode=False, sync=True):
        """Per-episode bookkeeping: returns gathered over ranks, counters, logging.

        sync=True (the reference runners' behaviour): block on the env's stream, raise the
        first device error, log.  sync=False (throughput loops): only enqueue the returns
        snapshot and its all-gather and advance the counters; the host sync, error checks
        and host-side statistics wait for flush_pending() (the GPU never idles at episode
        boundaries)."""
        returns = asg_dist.all_gather_returns(self.env.get_returns(), self.rank_envs)
        self._pending.append((returns, test_mode))
        # every env of every rank ran T steps (the reference's per-env accounting,
        # parallel_runner.py:178-179, summed over ranks: the env counts were all-gathered
        # at construction, so no per-episode collective or sync is needed)
        steps = self.global_envs * self.T
        if not test_mode:
            self.t_env += steps
        self._pending_steps.append(steps)
        if sync:
            self.flush_pending()

    def flush_pending(self):
        """Host side of the finished episodes: selector status, device errors, logging.
        The selectors' status goes first: an env whose noisy Q was invalid gets -1 in its actions
        row (asg_sap_select_into) and the next transition then sets the env's sticky action-range
        error -- the LSA's "invalid numeric entries" is the cause and is the error raised.  Whatever
        raises, the env's sticky device error word is read and cleared (its action-range error
        chained under the selector's) and the pending episodes are dropped, so a caller that
        catches the exception and continues sees no stale error on the next flush."""
        try:
            try:
                for sel in (getattr(self.mac, "action_selector", None),
                            getattr(self.mac, "jumpstart_action_selector", None)):
                    if hasattr(sel, "flush"):
                        sel.flush()
                    st = getattr(sel, "status", None)
                    if hasattr(st, "flush"):
                        st.flush()
            except BaseException as sel_err:
                try:
                    self.env.sync()
                except Exception as env_err:  # the consequence (-1 actions), not the cause
                    raise sel_err from env_err
                raise
            self.env.sync()
        except BaseException:
            self._pending.clear()
            self._pending_steps.clear()
            raise
        for (returns, test_mode), steps in zip(self._pending, self._pending_steps):
            self.last_returns = returns
            cur_stats = self.test_stats if test_mode else self.train_stats
            cur_returns = self.test_returns if test_mode else self.train_returns
            log_prefix = "test_" if test_mode else ""
            n_eps = self.global_envs
            cur_stats["n_episodes"] = n_eps + cur_stats.get("n_episodes", 0)
            cur_stats["ep_length"] = steps + cur_stats.get("ep_length", 0)
            cur_returns.extend(returns.cpu().tolist())
            n_test_runs = max(1, self.args.test_nepisode // n_eps) * n_eps
            if test_mode and len(self.test_returns) == n_test_runs:
                self._log(cur_returns, cur_stats, log_prefix)
            elif self.t_env - self.log_train_stats_t >= self.args.runner_log_interval:
                self._log(cur_returns, cur_stats, log_prefix)
                if hasattr(self.mac.action_selector, "epsilon"):
                    self.logger.log_stat("epsilon", self.mac.action_selector.epsilon, self.t_env)
                self.log_train_stats_t = self.t_env
                self.logger.log_stat("steps", self.t_env, self.t_env)
        self._pending.clear()
        self._pending_steps.clear()

    def run(self, test_mode=False):
        batch = self.rollout(test_mode=test_mode)
        self.finish_episode(test_mode=test_mode)
        return batch

    def _log(self, returns, stats, prefix):
        if self.rank == 0 and self.logger is not None:
            self.logger.log_stat(prefix + "return_mean", np.mean(returns), self.t_env)
            self.logger.log_stat(prefix + "return_std", np.std(returns), self.t_env)
            for k, v in stats.items():
                if k != "n_episodes":
                    self.logger.log_stat(prefix + k + "_mean", v / stats["n_episodes"], self.t_env)
        returns.clear()
        stats.clear()
