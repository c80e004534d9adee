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


# every material type (Material.h EMaterialType) with the reference field meanings
MATERIAL_CASES = {
    # name: list of (material index, type, albedo, roughness, ior, k, multiscattering, two_sided)
    "diffuse": [(i, 0, None, 1.0, None, None, False, False) for i in range(6)],
    "plastic_ms": [(3, 1, (0.8, 0.2, 0.2), 0.4, (1.5, 1.5, 1.5), None, True, False),
                   (4, 1, (0.2, 0.2, 0.8), 0.05, (1.8, 1.8, 1.8), None, False, True)],
    "conductor": [(3, 2, (0.9, 0.6, 0.3), 0.3, (0.2, 0.9, 1.1), (3.9, 2.4, 2.2), True, False),
                  (4, 2, (1.0, 1.0, 1.0), 0.0, (0.15, 0.4, 1.4), (3.6, 2.6, 2.3), False, False),
                  (0, 2, (0.9, 0.9, 0.9), 0.6, (1.0, 0.9, 0.8), (5.0, 4.0, 3.0), False, False)],
    "dielectric": [(3, 3, (1.0, 1.0, 1.0), 0.2, (1.5, 1.5, 1.5), None, True, False),
                   (4, 3, (1.0, 1.0, 1.0), 0.0, (1.33, 1.33, 1.33), None, False, False)],
    "thin_dielectric": [(3, 4, (0.9, 0.95, 1.0), 0.0, (1.5, 1.5, 1.5), None, False, False),
                        (5, 4, (1.0, 1.0, 1.0), 0.0, (1.45, 1.45, 1.45), None, False, True)],
}




def configure_lights(s, kind):
    from directcomputeraytracing_amd import scenes
    if kind == "constant":
        s.set_environment_light((0.4, 0.5, 0.6))
    elif kind == "cube":
        s.set_environment_light((1.0, 1.0, 1.0), scenes.env_cube(8))
    elif kind == "directional":
        s.add_directional_light((0.6, 0.3, 0.0), (1.5, 1.4, 1.2))
