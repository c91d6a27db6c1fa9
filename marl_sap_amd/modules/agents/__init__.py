"""Agent registry (reference: modules/agents/__init__.py).

The reference's names resolve to the module with the fused HIP inference forward whenever it
takes the shape: "rnn" -> RNNFusedAgent (RNNAgent's parameters, state_dict and -- under
autograd -- its PyTorch forward; only the no-grad rollout selection runs the kernel), so the
reference's unchanged YAML (agent: "rnn", config/default.yaml:43) lands on the fast path.
"rnn_torch" / "flat_const_agent_torch" keep the plain PyTorch module (explicit opt-out, e.g.
bench.py's pytorch_agent leg); args.fused_agent = False does the same for the default names."""
from .rnn_agent import FlatConstAgent, FlatConstFusedAgent, RNNAgent, RNNFusedAgent


def _fused_when_supported(fused_cls, torch_cls, n_out):
    def make(input_shape, args):
        if getattr(args, "fused_agent", True) and fused_cls.supports(input_shape, args, n_out(args)):
            return fused_cls(input_shape, args)
        return torch_cls(input_shape, args)
    make.__name__ = torch_cls.__name__
    return make


REGISTRY = {"rnn": _fused_when_supported(RNNFusedAgent, RNNAgent, lambda a: a.m),
            "rnn_fused": RNNFusedAgent, "rnn_torch": RNNAgent,
            "flat_const_agent": _fused_when_supported(FlatConstFusedAgent, FlatConstAgent,
                                                      lambda a: int(a.env_args["M"]) + 1),
            "flat_const_agent_fused": FlatConstFusedAgent, "flat_const_agent_torch": FlatConstAgent}
