from .rnn_agent import FlatConstAgent, FlatConstFusedAgent, RNNAgent, RNNFusedAgent

REGISTRY = {"rnn": RNNAgent, "rnn_fused": RNNFusedAgent, "flat_const_agent": FlatConstAgent,
            "flat_const_agent_fused": FlatConstFusedAgent}
