"""madigan_amd -- MI355X-native batched market-simulation step of madigan.

The hot path (Portfolio/Broker accounting, Sine/OU/TrendOU/Composite
generators, DSR/DDR/PPC rewards, sliding-window observation) runs as
hand-written HIP kernels for gfx950 behind a C ABI (include/madigan_amd.h,
libmadigan_hip.so); this package is the host side mirroring the reference's
Python surface (madigan/environments, madigan/utils/preprocessor.py).
"""
from . import _lib
from . import reward_normalization
from .config import ConfigError, SourceSpec, replay_spec, spec_from_config
from .env import (Asset, BatchedEnv, BrokerResponse, DataSourceTick, Env, EnvInfo, RiskInfo, State,
                  get_env_info, make_batched_env, make_env)
from .hdf import HDFSourceSingle, write_hdf
from .preprocessor import (MultiStackerDiscrete, PreProcessor, StackerDiscrete, StackerDiscretePairs,
                           StackerDiscreteReturns, make_preprocessor)

__all__ = ["Asset", "BatchedEnv", "BrokerResponse", "ConfigError", "DataSourceTick", "Env",
           "EnvInfo", "HDFSourceSingle", "PreProcessor", "RiskInfo", "SourceSpec",
           "StackerDiscrete", "State", "get_env_info", "make_batched_env", "make_env",
           "make_preprocessor", "MultiStackerDiscrete", "StackerDiscretePairs",
           "StackerDiscreteReturns", "replay_spec", "spec_from_config", "write_hdf"]


def load_extension():
    """Load libmadigan_hip.so and libmadigan_hdf.so (raises if not built)."""
    from .hdf import load_hdf
    load_hdf()
    return _lib.load()
