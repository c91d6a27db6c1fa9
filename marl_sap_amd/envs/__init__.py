"""Env registry (reference: envs/__init__.py:19-30).

REGISTRY holds the single-env plugin classes (constructed as Cls(**env_args));
BATCHED_REGISTRY holds the batched GPU envs the "gpu" runner constructs with
num_envs / env_index_base added.
"""
from functools import partial

from .multiagentenv import MultiAgentEnv
from .assign_env import AssignEnvBatch, MockConstellationEnv, make_scheme, batch_view
from .real_env import InterferenceAssignEnvBatch, RealAssignEnvBatch, RealPowerAssignEnvBatch, make_real_scheme


def env_fn(env, **kwargs) -> MultiAgentEnv:
    return env(**kwargs)


REGISTRY = {"mock_constellation_env": partial(env_fn, env=MockConstellationEnv)}
BATCHED_REGISTRY = {"mock_constellation_env": partial(env_fn, env=AssignEnvBatch),
                    "real_constellation_env": partial(env_fn, env=RealAssignEnvBatch),
                    "real_power_constellation_env": partial(env_fn, env=RealPowerAssignEnvBatch),
                    "interference_constellation_env": partial(env_fn, env=InterferenceAssignEnvBatch)}
