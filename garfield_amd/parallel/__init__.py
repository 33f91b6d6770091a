"""Distributed execution: RCCL/gloo process groups and the robust data-parallel engines."""
from garfield_amd.parallel.comm import DistContext, init_distributed, make_role_groups, shutdown
from garfield_amd.parallel.engine import EngineConfig, RobustDataParallel, synthetic_batches

__all__ = ["DistContext", "init_distributed", "make_role_groups", "shutdown", "EngineConfig", "RobustDataParallel",
           "synthetic_batches"]
