"""gRPC transport: the reference's TensorFlow deployment model (pull-based
``MessageExchange`` service, TF_CONFIG cluster files, PS/worker/Byzantine nodes),
re-hosted on the PyTorch-ROCm stack.

Reference: ``tensorflow_impl/libs`` and ``tensorflow_impl/rsrcs/{network.py,
aggregator_tf}``. TensorFlow itself is not part of this framework: models, gradients
and GARs run on the framework's own (HIP) path; only the deployment and wire
protocol are kept.
"""
from garfield_amd.grpcnet.aggregator import Aggregator, Aggregator_tf
from garfield_amd.grpcnet.attacker import Attacker
from garfield_amd.grpcnet.network import Network, make_config, write_configs

__all__ = ["Aggregator", "Aggregator_tf", "Attacker", "Network", "make_config", "write_configs"]
