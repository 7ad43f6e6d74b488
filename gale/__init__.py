"""gale — an MI355X-native streaming image-inference engine.

Same capabilities and external contract as the Storm topology of
HyoJong-Moon/Distributed-Inference-System-based-Storm (Kafka in -> CNN inference replicas ->
Kafka out; ``<TOPOLOGY_NAME> <INPUT_TOPIC> <OUTPUT_TOPIC>`` CLI, ``{"instances": [N][H][W][C]}``
records in, ``{"predictions": [N][classes]}`` records out), re-designed for AMD CDNA4:
hand-written gfx950 HIP kernels, a C++ host runtime (Kafka wire protocol, JSON codec,
micro-batching scheduler, hipGraph executor) and RCCL over xGMI for multi-GPU replicas.
"""

__version__ = "0.1.0"

from gale._native import native, native_available  # noqa: F401
