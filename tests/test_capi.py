"""CPU: the C-ABI library loads and exports every symbol include/flr.h declares."""
import ctypes
import os
import re

import pytest

from flr import _capi


def header_functions():
    text = open(_capi.HEADER_PATH).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(flr_[a-z0-9_]+)\s*\(", text)))


def test_library_built():
    assert os.path.exists(_capi.LIB_PATH), "run __graft_entry__.build() first"


def test_header_symbols_exported():
    handle = ctypes.CDLL(_capi.LIB_PATH)
    names = header_functions()
    assert len(names) >= 10
    for n in names:
        assert hasattr(handle, n), f"{n} declared in include/flr.h but not exported"


def test_signatures_cover_header():
    assert sorted(_capi.SIGNATURES) == header_functions()


def test_status_strings_and_version():
    lib = _capi.lib()
    assert lib.flr_version().decode().startswith("flr ")
    assert lib.flr_status_string(_capi.FLR_ERR_KRUM_N).decode() == "Krum requires n >= 2f + 3"
    assert lib.flr_status_string(0).decode() == "ok"


def test_workspace_queries_are_host_only():
    lib = _capi.lib()
    assert lib.flr_pairwise_l2_workspace(128, 10_000_000) > 0
    assert lib.flr_pairwise_l2_direct_workspace(5, 110) > 0
    assert lib.flr_pairwise_l2_workspace(0, 10) == 0


def test_argument_validation_without_gpu():
    lib = _capi.lib()
    # null pointers / bad shapes are rejected before any device work
    assert lib.flr_krum_select(None, 5, 2, None, None, None) == _capi.FLR_ERR_ARG
    assert lib.flr_rows_mean(None, 4, 10, 10, None, 2, 2, None, None) == _capi.FLR_ERR_ARG
    assert lib.flr_trimmed_mean(None, 4, 10, 10, 2, None, None) == _capi.FLR_ERR_ARG


def test_tap_major_rule_matches_library():
    from flr import _capi
    from flr.models.multimodal import ModelSpec, param_layout, tap_major_names
    lib = _capi.lib()
    names = tap_major_names(ModelSpec())
    for n, s in param_layout(ModelSpec()):
        if len(s) == 4:
            assert (n in names) == bool(lib.flr_conv2d_tap_major_ok(s[1], s[0])), n
    assert len(names) == 19
