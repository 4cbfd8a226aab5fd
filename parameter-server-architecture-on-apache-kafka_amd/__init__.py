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

import os as _os

# Kernel arguments in device memory: a local solve is a chain of ~8 dependent
# latency-bound launches, and host-memory kernargs cost ~20 us per solve
# (tools/bench_solver.py: 84.3 us with 0, 63.8 us with 1; profiles/r01_v8).
# Read by the HIP runtime at its first call, so set before any GPU work.
_os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")

from . import _native  # noqa: F401  (loads the native host runtime)
