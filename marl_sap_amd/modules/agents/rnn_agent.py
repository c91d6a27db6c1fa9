"""Shared-parameter agent network (reference: modules/agents/rnn_agent.py:7-31):
fc1 -> ReLU -> GRUCell (use_rnn) or Linear+ReLU -> fc2, fp32, run in PyTorch-ROCm."""
import ctypes

import torch
import torch.nn as nn
import torch.nn.functional as F

from ... import _lib


class RNNAgent(nn.Module):
    def __init__(self, input_shape, args, n_out=None):
        super().__init__()
        self.args = args
        self.n_out = args.m if n_out is None else int(n_out)
        self.fc1 = nn.Linear(input_shape, args.hidden_dim)
        if self.args.use_rnn:
            self.rnn = nn.GRUCell(args.hidden_dim, args.hidden_dim)
        else:
            self.rnn = nn.Linear(args.hidden_dim, args.hidden_dim)
        self.fc2 = nn.Linear(args.hidden_dim, self.n_out)

    def init_hidden(self):
        return self.fc1.weight.new(1, self.args.hidden_dim).zero_()

    def forward(self, inputs, hidden_state):
        x = F.relu(self.fc1(inputs))
        h_in = hidden_state.reshape(-1, self.args.hidden_dim)
        if self.args.use_rnn:
            h = self.rnn(x, h_in)
        else:
            h = F.relu(self.rnn(x))
        q = self.fc2(h)
        return q, h


class RNNFusedAgent(RNNAgent):
    """RNNAgent with the same parameters / state_dict, whose inference forward (no autograd:
    the rollout's action selection) is one fused HIP kernel (asg_rnn_agent_forward: f32
    MFMA, fc1 + GRUCell + fc2 with every intermediate in registers; hidden 64, any input
    size, n_out = m up to 512 -- the real envs' m = 450 included).  With autograd enabled
    (learner training) it is the plain PyTorch module, so gradients are unchanged."""

    def __init__(self, input_shape, args, n_out=None):
        super().__init__(input_shape, args, n_out)
        if not self.supports(input_shape, args, self.n_out):
            raise ValueError("rnn_fused needs hidden_dim == 64 and 1 <= n_out <= 512; use agent 'rnn_torch'")

    @staticmethod
    def supports(input_shape, args, n_out):
        """Shapes the fused inference kernels take (hidden 64, 1 <= n_out <= 512, any input)."""
        return args.hidden_dim == 64 and 1 <= int(n_out) <= 512 and int(input_shape) >= 1

    def _prep(self, inputs, hidden_state):
        x = inputs
        if x.dtype != torch.float32 or x.stride(-1) != 1 or x.stride(0) < x.shape[1]:
            x = x.float().contiguous()
        H = self.args.hidden_dim
        h = hidden_state
        if h.dim() == 3 and h.stride(0) == 0 and h.stride(1) == 0 and h.stride(2) == 1:
            hs = 0  # init_hidden's expanded zero row: one row broadcast to all agents
        else:
            h = h.reshape(-1, H)
            if h.stride(-1) != 1 or h.stride(0) % 4 != 0 or h.data_ptr() % 16 != 0:
                h = h.contiguous()
            hs = h.stride(0)
        return x, h, hs

    def _common(self, x, h, hs):
        R, K = x.shape
        rnn = bool(self.args.use_rnn)
        p = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
        h_out = torch.empty((R, self.args.hidden_dim), dtype=torch.float32, device=x.device)
        args = [p(x), x.stride(0), R, K, p(h), hs, p(self._packed(K, x.device)), p(self.fc1.bias),
                p(self.rnn.bias_ih if rnn else self.rnn.bias), p(self.rnn.bias_hh) if rnn else None,
                p(self.fc2.bias), self.args.hidden_dim, self.n_out, int(rnn), p(h_out)]
        return h_out, args, p

    def forward(self, inputs, hidden_state):
        if torch.is_grad_enabled() or not inputs.is_cuda:
            return super().forward(inputs, hidden_state)
        x, h, hs = self._prep(inputs, hidden_state)
        with torch.cuda.device(x.device):
            h_out, args, p = self._common(x, h, hs)
            q = torch.empty((x.shape[0], self.n_out), dtype=torch.float32, device=x.device)
            _lib.check(_lib.lib().asg_rnn_agent_forward(*args, p(q), _lib.stream_ptr(x.device)))
        return q, h_out

    def forward_select(self, inputs, hidden_state, avail, n, epsilon, seed, counter, out, status, q_out=None,
                       env_index_base=0):
        """forward + epsilon-greedy in one kernel (asg_rnn_agent_select): actions into `out`
        ([B, n] int64 view, e.g. the EpisodeBatch actions row); avail [B, n, m] bool;
        env_index_base: global index of env 0 (exploration draws are keyed by global row).
        Returns the new hidden state [B*n, hidden]."""
        x, h, hs = self._prep(inputs, hidden_state)
        if avail.dtype != torch.bool or avail.stride(-1) != 1:
            avail = (avail != 0).contiguous()
        with torch.cuda.device(x.device):
            h_out, args, p = self._common(x, h, hs)
            _lib.check(_lib.lib().asg_rnn_agent_select(
                *args, p(q_out), p(avail), _lib.i64arr(avail.stride()[:2]), n, float(epsilon),
                seed & 0xFFFFFFFFFFFFFFFF, counter, int(env_index_base), p(out), _lib.i64arr(out.stride()), p(status),
                _lib.stream_ptr(x.device)))
        return h_out

    def step_select_args(self, hidden_state, K, device, R):
        """The agent half of asg_rollout's arguments: packed weights, biases (GRU: b_ih, b_hh;
        Linear: its bias, NULL), K, hidden, use_rnn, h_in (+ row stride), and a fresh h_out
        tensor (last)."""
        H = self.args.hidden_dim
        h = hidden_state
        if h.dim() == 3 and h.stride(0) == 0 and h.stride(1) == 0 and h.stride(2) == 1:
            hs = 0  # init_hidden's expanded zero row
        else:
            h = h.reshape(-1, H)
            if h.stride(-1) != 1 or h.stride(0) % 4 != 0 or h.data_ptr() % 16 != 0:
                h = h.contiguous()
            hs = h.stride(0)
        if hs and h.shape[0] != R:
            raise ValueError(f"hidden state has {h.shape[0]} rows, the batch {R}")
        p = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
        self._h_keep = h  # alive until the kernel has read it (stream order)
        h_out = torch.empty((R, H), dtype=torch.float32, device=device)
        rnn = bool(self.args.use_rnn)
        return [p(self._packed(K, device)), p(self.fc1.bias), p(self.rnn.bias_ih if rnn else self.rnn.bias),
                p(self.rnn.bias_hh) if rnn else None, p(self.fc2.bias), int(K), int(H), int(rnn), p(h), int(hs),
                h_out]

    def _packed(self, K, device):
        """Weights in the kernel's fragment order, re-packed only when a weight changed
        (optimizer steps bump the tensors' version counters; load_state_dict too)."""
        rnn = self.args.use_rnn
        ws = [self.fc1.weight, self.rnn.weight_ih if rnn else self.rnn.weight,
              self.rnn.weight_hh if rnn else None, self.fc2.weight]
        key = (K, str(device), tuple((w.data_ptr(), w._version) for w in ws if w is not None))
        if getattr(self, "_pack_key", None) != key:
            L = _lib.lib()
            nbytes = L.asg_rnn_agent_packed_size(K, self.args.hidden_dim, self.n_out, int(bool(rnn)))
            _lib.check(int(nbytes) if nbytes < 0 else 0)
            buf = torch.empty(int(nbytes) // 4, dtype=torch.float32, device=device)
            p = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
            _lib.check(L.asg_rnn_agent_pack(p(ws[0]), p(ws[1]), p(ws[2]), p(ws[3]), K, self.args.hidden_dim,
                                            self.n_out, int(bool(rnn)), p(buf), _lib.stream_ptr(device)))
            self._pack_buf, self._pack_key = buf, key
        return self._pack_buf


class FlatConstAgent(RNNAgent):
    """FlatConstellationAgent (reference: modules/agents/flat_const_agent.py:9-34): the
    RNNAgent network with M + 1 outputs (one per top-M task and the baseline), the agent of
    the filtered real-env algorithms (filtered_reda.yaml, iql_sap.yaml)."""

    def __init__(self, input_shape, args):
        super().__init__(input_shape, args, n_out=int(args.env_args["M"]) + 1)


class FlatConstFusedAgent(RNNFusedAgent):
    """FlatConstAgent whose no-grad rollout forward is the fused HIP kernel."""

    def __init__(self, input_shape, args):
        super().__init__(input_shape, args, n_out=int(args.env_args["M"]) + 1)
