import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and the built librtamd.so")


@pytest.fixture(scope="session")
def golden():
    import json
    with open(os.path.join(GOLDEN, "golden_meta.json")) as fh:
        meta = json.load(fh)
    return {
        "meta": meta,
        "small": dict(np.load(os.path.join(GOLDEN, "renders_small.npz"))),
        "full": dict(np.load(os.path.join(GOLDEN, "renders_full_subsample.npz"))),
        "kats": dict(np.load(os.path.join(GOLDEN, "kats.npz"))),
    }


@pytest.fixture(scope="session")
def oracle():
    from oracle import pyoracle
    pyoracle.lib()
    return pyoracle


@pytest.fixture(scope="session")
def ctx():
    """The HIP context for GPU tests.  No skip: on a GPU box a missing device or library is a
    failure (the renderer has no CPU fallback)."""
    from raytracingengine_amd import capi
    c = capi.Context(0)
    yield c
    c.close()
