"""Defense registry (mirror of src/defenses/__init__.py:28-59).

The names of the reference factory are all registered and run on the HIP
kernels, except FLTrust (needs server-side root-set
training), which raises NotImplementedError instead of silently doing
something else.
"""
from .base_defense import BaseDefense, NoDefense
from .krum import KrumDefense, MultiKrumDefense
from .geometric_median import GeometricMedianDefense
from .norm_based import DPSGDDefense, GradientClippingDefense, NormBoundingDefense
from .trimmed_mean import MedianDefense, TrimmedMeanDefense

__all__ = [
    "BaseDefense", "NoDefense", "KrumDefense", "MultiKrumDefense",
    "TrimmedMeanDefense", "MedianDefense", "GeometricMedianDefense",
    "GradientClippingDefense", "NormBoundingDefense", "DPSGDDefense", "get_defense",
]

_NOT_IN_SCOPE = ("fltrust",)


def _out_of_scope(name):
    def make(_cfg):
        raise NotImplementedError(
            f"defense {name!r} is not on this engine's hot path (see DESIGN.md, out-of-scope rows)")
    return make


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
}
_DEFENSES.update({n: _out_of_scope(n) for n in _NOT_IN_SCOPE})


def get_defense(defense_type: str, defense_config: dict):
    """Factory by name; unknown names raise ValueError like the reference."""
    if defense_type not in _DEFENSES:
        raise ValueError(f"Unknown defense type: {defense_type}. Available: {list(_DEFENSES.keys())}")
    return _DEFENSES[defense_type](defense_config)
