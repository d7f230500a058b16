"""flr — MI355X-native federated-round engine (gfx950).

Drop-in for the per-round hot path of Shashank8834/multimodal-fl-security:
K clients' local SGD on a multimodal model, then Byzantine-robust
aggregation (FedAvg, Krum / Multi-Krum, trimmed mean, median) over the K
flattened client vectors.  See DESIGN.md.
"""
from . import ops  # noqa: F401
from .matrix import ClientMatrix  # noqa: F401

__version__ = "0.1.0"
