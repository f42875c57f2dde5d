import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP engine)")
    config.addinivalue_line("markers", "experimental: A/B alternates compiled only into an AMX_EXPERIMENTAL=1 "
                                       "build (include/amx_hip_experimental.h)")


def _experimental_built() -> bool:
    try:
        import ctypes
        from amp_extensions_amd import _build, _native
        return _native.has_experimental(ctypes.CDLL(_build.LIB_PATH))
    except OSError:
        return False


def pytest_collection_modifyitems(config, items):
    """Tests of the measured-slower alternates run only against an AMX_EXPERIMENTAL=1 build."""
    if any("experimental" in it.keywords for it in items) and not _experimental_built():
        skip = pytest.mark.skip(reason="experimental A/B path: the library is built without AMX_EXPERIMENTAL=1")
        for it in items:
            if "experimental" in it.keywords:
                it.add_marker(skip)


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    def load(name):
        return np.load(os.path.join(GOLDEN, name), allow_pickle=False)

    return load
