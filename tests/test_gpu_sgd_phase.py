"""a6 + a7: the clip + SGD-momentum step split into its norm phase and
parameter-group update phases (flr_clip_sgd_step_phase, the native trainers'
side-stream overlap) is bit-identical to the one-call step
(flr_clip_sgd_step_blocked_src), for first, middle and last steps, with the
clip active (run_experiments.py:206-211, 234-235)."""
import ctypes

import pytest
import torch

from flr import _capi

pytestmark = pytest.mark.gpu


def _arr(vals, ct):
    return (ct * len(vals))(*vals)


def _run(cuda, K, sizes, groups, flags, phased, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    xs = [torch.randn(K, n, generator=g).to(cuda) for n in sizes]
    gs = [torch.randn(K, n, generator=g).mul_(3.0).to(cuda) for n in sizes]
    ms = [torch.randn(K, n, generator=g).to(cuda) for n in sizes]
    nb = len(sizes)
    ws = torch.zeros(int(_capi.lib().flr_clip_sgd_workspace(K)), dtype=torch.uint8, device=cuda)
    norms = torch.zeros(K, device=cuda)
    st = torch.cuda.current_stream(cuda).cuda_stream

    def ptrs(ts):
        return _arr([t.data_ptr() for t in ts], ctypes.c_void_p)

    n_arr = _arr(list(sizes), ctypes.c_int64)
    common = (0.05, 0.9, 0.0, 1.0, flags)
    if not phased:
        _capi.call("flr_clip_sgd_step_blocked_src", ptrs(xs), ptrs(gs), ptrs(ms), n_arr, None, nb, K, *common,
                   None, None, 0, 0, None, None, 0, None, None, norms.data_ptr(), ws.data_ptr(), ws.numel(), st)
    else:
        _capi.call("flr_clip_sgd_step_phase", ptrs(xs), ptrs(gs), ptrs(ms), n_arr, None, nb, K, *common,
                   None, None, 0, 0, None, None, 0, None, None, norms.data_ptr(), 1, ws.data_ptr(), ws.numel(), st)
        for j0, j1 in reversed(groups):  # any order, any subset
            _capi.call("flr_clip_sgd_step_phase", ptrs(xs[j0:j1]), ptrs(gs[j0:j1]), ptrs(ms[j0:j1]),
                       _arr(list(sizes[j0:j1]), ctypes.c_int64), None, j1 - j0, K, *common, None, None, 0, 0, None,
                       None, 0, None, None, None, 2, ws.data_ptr(), ws.numel(), st)
    torch.cuda.synchronize(cuda)
    return [t.cpu() for t in xs + ms] + [norms.cpu()]


@pytest.mark.parametrize("flags", [0, 1, 2], ids=["middle", "first", "last"])
def test_phased_step_bit_identical(cuda, flags):
    K = 5
    sizes = [9408, 64, 64, 36864, 3, 147456, 1000, 4096 * 9 + 5]
    groups = [(0, 3), (3, 4), (4, 6), (6, 8)]
    one = _run(cuda, K, sizes, groups, flags, phased=False)
    two = _run(cuda, K, sizes, groups, flags, phased=True)
    for a, b in zip(one, two):
        assert torch.equal(a, b)
    assert (one[-1] > 1.0).all()  # the clip was active


def test_phase_rejects_bad_phase(cuda):
    x = torch.zeros(1, 4, device=cuda)
    p = _arr([x.data_ptr()], ctypes.c_void_p)
    rc = _capi.lib().flr_clip_sgd_step_phase(p, p, p, _arr([4], ctypes.c_int64), None, 1, 1, 0.1, 0.9, 0.0, 0.0, 0,
                                              None, None, 0, 0, None, None, 0, None, None, None, 4, None, 0, None)
    assert rc != 0
