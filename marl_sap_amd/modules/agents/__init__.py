from .rnn_agent import RNNAgent, RNNFusedAgent

REGISTRY = {"rnn": RNNAgent, "rnn_fused": RNNFusedAgent}
