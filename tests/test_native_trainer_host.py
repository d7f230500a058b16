"""flr_train_clients' host-side layout (no GPU needed): the parameter count
of the C entry's model equals the reference-structured module's, for the C3
model and the test-size spec; unsupported shapes are refused."""
import dataclasses

import pytest

from flr.models.multimodal import TINY, ModelSpec, num_params
from flr import native_trainer as nt


@pytest.mark.parametrize("spec", [ModelSpec(), TINY, dataclasses.replace(ModelSpec(), num_classes=200, vocab=312)],
                         ids=["c3", "tiny", "classes200"])
def test_param_count_matches_module(spec):
    assert nt.num_params(spec) == num_params(spec)
    assert nt.workspace_bytes(spec, 4, 8, 2) > 0


def test_unsupported_shapes_refused():
    # a 64x64 image leaves a 2x2 map after the trunk (global pooling is the 1x1 view)
    assert nt.workspace_bytes(dataclasses.replace(ModelSpec(), image_size=64), 4, 8, 2) == 0
    assert nt.workspace_bytes(ModelSpec(), 0, 8, 2) == 0
    with pytest.raises(ValueError):
        nt.ResNetGruSpec.of(dataclasses.replace(ModelSpec(), family="cub"))
