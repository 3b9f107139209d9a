import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")
PC12 = os.path.join(GOLDEN, "point_cloud_12.ply")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session")
def built():
    """Build libgsplat.so and the oracle once per session (fast no-op when up to date)."""
    import __graft_entry__

    __graft_entry__.build()
    return True


@pytest.fixture(scope="session")
def pc12_scene(built):
    from gaussian_splat_ipu_amd import scene

    ply = scene.load_ply(PC12)
    g, bb = scene.prepare_scene(ply)
    return g, bb


# gs_test_set keys (include/gsplat.h) and their automatic values
TEST_HOOK_DEFAULTS = {"bin_chunk_size": 0, "bin_agg": -1, "debug_poison": 0, "cov_cache": -1, "bin_direct": -1}


@pytest.fixture
def test_hook(built):
    """gs_test_set: a process-wide test hook read by gs_create (no environment
    variable selects a path); every hook is back at its automatic value after
    the test."""
    from gaussian_splat_ipu_amd._lib import check, lib

    def set_hook(key, value):
        check(lib().gs_test_set(key.encode(), int(value)), "gs_test_set")

    yield set_hook
    for k, v in TEST_HOOK_DEFAULTS.items():
        lib().gs_test_set(k.encode(), v)
