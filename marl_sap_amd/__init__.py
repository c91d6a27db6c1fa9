"""marl_sap_amd: MI355X-native batched rollout + sequential-assignment environment for
EPyMARL-style MARL (drop-in for josh-holder/marl_sap's runner/env hot path).

The compute path is HIP (libmarl_sap_amd.so, C-ABI in include/asg.h); agent networks
and action selectors run in PyTorch-ROCm; multi-GPU is one process per GPU over RCCL.
"""
from . import _lib  # noqa: F401

__all__ = ["envs", "runners", "components", "controllers", "action_selectors", "dist"]
