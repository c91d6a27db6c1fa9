"""Learner-side pieces on the rollout path's kernels.  The learners
themselves (optimisers, mixers, critics) stay the reference's PyTorch code."""
from .sap_targets import sap_target_max_qvals

__all__ = ["sap_target_max_qvals"]
