import os
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
GOLDEN = ROOT / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C ABI)")


@pytest.fixture(scope="session")
def native_lib():
    from directcomputeraytracing_amd.build import build_native
    build_native()
    from directcomputeraytracing_amd import _abi
    return _abi.load_library()


@pytest.fixture(scope="session")
def oracle_mod():
    from directcomputeraytracing_amd.build import build_oracle
    build_oracle()
    import oracle
    oracle.load()
    return oracle


@pytest.fixture(scope="session")
def golden_luts(oracle_mod):
    return oracle_mod.luts_from_arrays(dict(np.load(GOLDEN / "bxdf_luts.npz")))


def cornell(width, height, max_bounce):
    from directcomputeraytracing_amd import Scene, scenes
    s = Scene((width, height))
    scenes.setup_cornell(s, width, height, max_bounce)
    return s


@pytest.fixture(scope="session")
def gpu_tracer(native_lib, golden_luts):
    from directcomputeraytracing_amd import WavefrontPathTracer
    t = WavefrontPathTracer(path_pool_size=1 << 16, iterations_per_render=8, debug_rng=True)
    yield t
    t.destroy()
