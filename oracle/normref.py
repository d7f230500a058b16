"""ORACLE (test infrastructure only) — ctypes access to oracle/norm_ref.c, the
C restatement of the reference's per-pair fp32 ``torch.norm(fi - fj).item()``
(src/defenses/krum.py:89-97, accumulation model SURVEY.md App. C).

``norm_diff`` is pinned against torch.norm itself by tests/test_oracle.py;
``distance_matrix`` is then krum.py:89-97's matrix for a [K, P] float32
array, computed with OpenMP over the pairs (the fast way to get the
reference's exact D for the GPU parity tests)."""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "_build", "libnormref.so")
_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            subprocess.run(["make", "-C", _HERE], check=True, capture_output=True)
        h = ctypes.CDLL(_LIB)
        h.flr_oracle_norm_diff.restype = ctypes.c_float
        h.flr_oracle_norm_diff.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]
        h.flr_oracle_norm_pairs.restype = None
        h.flr_oracle_norm_pairs.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                            ctypes.c_void_p]
        _lib = h
    return _lib


def norm_diff(a: np.ndarray, b: np.ndarray) -> float:
    """torch.norm(a - b).item() for 1-D float32 arrays (returned as the fp32 value widened)."""
    a = np.ascontiguousarray(a, dtype=np.float32)
    b = np.ascontiguousarray(b, dtype=np.float32)
    assert a.shape == b.shape and a.ndim == 1
    return float(lib().flr_oracle_norm_diff(a.ctypes.data, b.ctypes.data, a.size))


def distance_matrix(X: np.ndarray) -> np.ndarray:
    """[K, K] float64: D[i][j] = torch.norm(X[i] - X[j]).item() (krum.py:89-97)."""
    X = np.ascontiguousarray(X, dtype=np.float32)
    K, P = X.shape
    D = np.zeros((K, K), dtype=np.float64)
    lib().flr_oracle_norm_pairs(X.ctypes.data, K, P, P, D.ctypes.data)
    return D
