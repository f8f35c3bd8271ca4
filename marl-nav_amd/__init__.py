"""marlnav_amd - the MARL-nav environment step on AMD MI355X (gfx950).

A drop-in for ``marlnav.environment.Env`` (JussiM01/MARL-nav) whose step runs
as one hand-written HIP kernel (libmarlnav.so, C ABI in include/marlnav.h).
The package directory is ``marl-nav_amd/``; import it as ``marlnav_amd``
(the alias module at the repository root) or with
``importlib.import_module('marl-nav_amd')``.
"""
from . import abi, rollout, shard
from .environment import Env
from .utils import (ActionScaler, ConstantSampler, MockInitializer, MockSampler,
                    ObsNormalizer, Observations, TriangleIntitializer, action_sampler, default_args,
                    init_sampler, set_all_seeds, set_env_params, set_init_params,
                    set_normalizer_params, set_sampler_params, set_scaler_params)

__all__ = ["Env", "Observations", "ObsNormalizer", "ActionScaler", "MockInitializer",
           "TriangleIntitializer", "ConstantSampler", "MockSampler", "init_sampler",
           "action_sampler", "set_all_seeds", "set_env_params", "set_init_params",
           "set_sampler_params", "set_normalizer_params", "set_scaler_params", "default_args",
           "abi", "rollout", "shard"]
