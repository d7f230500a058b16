import glob
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "multimodal-fl-security_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


def golden_files(prefix):
    return sorted(glob.glob(os.path.join(GOLDEN, f"{prefix}_*.npz")))


def load_golden(path):
    z = np.load(path, allow_pickle=False)
    return {k: z[k] for k in z.files}


def shapes_of(fx):
    return [tuple(int(v) for v in row[:nd]) for row, nd in zip(fx["shapes"], fx["ndims"])]


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU visible")
    return torch.device("cuda:0")


@pytest.fixture
def knob():
    """Set one of the library's A/B switches for this test (flr_set_knob: the
    library reads the FLR_* environment once, at load); restored afterwards."""
    from flr import _capi
    names = []

    def set_(name, value):
        names.append(name)
        _capi.set_knob(name, value)
    yield set_
    for n in names:
        _capi.set_knob(n, os.environ.get(n))


@pytest.fixture
def ablation_build():
    """Tests of the measured-slower / timing-only kernel forms: they exist only
    in the tools build (make ABLATION=1; run with FLR_LIB pointing at it)."""
    from flr import _capi
    if "ablation" not in _capi.build_info():
        pytest.skip("tools-build kernel form (make ABLATION=1)")
