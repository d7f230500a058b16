"""Defense registry (mirror of src/defenses/__init__.py:28-59).

Every name of the reference factory is registered and runs on the HIP kernels
(FLTrust's server update runs on the client-batched trainer).
"""
from .base_defense import BaseDefense, NoDefense
from .krum import KrumDefense, KrumTrimmedMeanDefense, MultiKrumDefense
from .fltrust import FLTrustDefense
from .geometric_median import GeometricMedianDefense
from .norm_based import DPSGDDefense, GradientClippingDefense, NormBoundingDefense
from .trimmed_mean import MedianDefense, TrimmedMeanDefense

__all__ = [
    "BaseDefense", "NoDefense", "KrumDefense", "MultiKrumDefense", "KrumTrimmedMeanDefense",
    "TrimmedMeanDefense", "MedianDefense", "GeometricMedianDefense",
    "GradientClippingDefense", "NormBoundingDefense", "DPSGDDefense", "FLTrustDefense", "get_defense",
]

_DEFENSES = {
    "none": NoDefense,
    "fedavg": NoDefense,
    "krum": KrumDefense,
    "multi_krum": MultiKrumDefense,
    "trimmed_mean": TrimmedMeanDefense,
    "median": MedianDefense,
    "geometric_median": GeometricMedianDefense,
    "dp_sgd": DPSGDDefense,
    "gradient_clipping": GradientClippingDefense,
    "norm_bounding": NormBoundingDefense,
    "fltrust": FLTrustDefense,
    # build extension: Multi-Krum selection then trimmed mean (BASELINE.json configs[4])
    "krum_trimmed_mean": KrumTrimmedMeanDefense,
}


def get_defense(defense_type: str, defense_config: dict):
    """Factory by name; unknown names raise ValueError like the reference."""
    if defense_type not in _DEFENSES:
        raise ValueError(f"Unknown defense type: {defense_type}. Available: {list(_DEFENSES.keys())}")
    return _DEFENSES[defense_type](defense_config)
