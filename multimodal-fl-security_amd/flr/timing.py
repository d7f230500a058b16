"""Raw HIP events for timing one kernel inside a multi-kernel op.

torch.cuda.Event only brackets torch's own stream position; the flr C ABI can
record caller-owned hipEvent_t handles immediately around a specific kernel
launch (flr_pairwise_l2_ex).  The events come from the HIP runtime torch
already loaded (same libamdhip64.so.7 SONAME), so they live on the same
device/streams.
"""
from __future__ import annotations

import ctypes

_hip = None


def _rt():
    global _hip
    if _hip is None:
        import torch  # noqa: F401  (loads torch's libamdhip64 first)
        _hip = ctypes.CDLL("libamdhip64.so.7", mode=ctypes.RTLD_GLOBAL)
        _hip.hipEventCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
        _hip.hipEventDestroy.argtypes = [ctypes.c_void_p]
        _hip.hipEventSynchronize.argtypes = [ctypes.c_void_p]
        _hip.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_void_p, ctypes.c_void_p]
    return _hip


class HipEventPair:
    def __init__(self):
        rt = _rt()
        self.begin = ctypes.c_void_p()
        self.end = ctypes.c_void_p()
        assert rt.hipEventCreate(ctypes.byref(self.begin)) == 0
        assert rt.hipEventCreate(ctypes.byref(self.end)) == 0

    @property
    def handles(self):
        return (self.begin.value, self.end.value)

    def elapsed_ms(self) -> float:
        rt = _rt()
        assert rt.hipEventSynchronize(self.end) == 0
        ms = ctypes.c_float()
        assert rt.hipEventElapsedTime(ctypes.byref(ms), self.begin, self.end) == 0
        return float(ms.value)

    def __del__(self):
        try:
            rt = _rt()
            rt.hipEventDestroy(self.begin)
            rt.hipEventDestroy(self.end)
        except Exception:
            pass
