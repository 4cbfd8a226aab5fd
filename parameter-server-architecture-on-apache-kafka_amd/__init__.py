"""psx -- an MI355X-native parameter-server training engine.

Same capabilities as the Kafka-Streams parameter server of
kiminh/Parameter-Server-Architecture-On-Apache-Kafka (online multinomial
logistic regression over a rate-controlled stream, adaptive sliding-window
buffers, sequential / bounded-delay / eventual consistency, the
ServerAppRunner / WorkerAppRunner CLIs and the reference CSV log schema), built
on PyTorch-ROCm + hand-written HIP/CDNA4 kernels + RCCL over xGMI.

The importable name is ``psx``; the on-disk package directory is
``parameter-server-architecture-on-apache-kafka_amd`` (``psx`` is a symlink).
"""
__version__ = "0.1.0"

from . import _native  # noqa: F401  (loads the native host runtime)
