import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_ROOT = os.path.join(REPO, "multimodal-ssl-avmnist_amd")
for p in (REPO, PKG_ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def pytest_collection_modifyitems(config, items):
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:  # pragma: no cover
        has_gpu = False
    if has_gpu:
        return
    skip = pytest.mark.skip(reason="no HIP device in this container")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture
def avd_opts():
    """Set libavdino's launch options (avd_set_options: grid_cap, generic_conv, generic_m2)
    inside a test: avd_opts(grid_cap=3); every setting is undone when the test ends."""
    import contextlib

    from avdino import ops
    stack = contextlib.ExitStack()

    def set_(**kw):
        stack.enter_context(ops.options(**kw))

    yield set_
    stack.close()
