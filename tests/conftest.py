import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu)")


@pytest.fixture
def tune():
    """Per-test tuning of the shared cuda:0 context: tune(name, value) calls
    pnetgpu_ctx_set_tuning (libpnet_amd.engine.TUNING_KEYS); every key is
    restored when the test ends. GPU tests only (it creates the context)."""
    from libpnet_amd import engine
    ctx = engine.context(0)
    saved = {k: ctx.get_tuning(k) for k in engine.TUNING_KEYS}
    yield ctx.set_tuning
    for k, v in saved.items():
        ctx.set_tuning(k, v)
