"""erasurehead_amd — MI355X-native straggler-tolerant distributed gradient descent with gradient codes.

Capabilities of Distributed-Deep-Learning/ErasureHead (uncoded, cyclic-MDS, fractional
repetition, approximate gradient coding, ignore-stragglers, partial hybrids; logistic and
least-squares models; GD/AGD) rebuilt on PyTorch-ROCm + gfx950 HIP kernels + RCCL.
"""
__version__ = "0.1.0"

from .config import RunConfig  # noqa: E402
