"""MI355X-native wavefront path tracer (drop-in for DirectComputeRayTracing's
``WavefrontPathTracing.hlsl`` hot path).

The product is ``libdcrt.so`` (gfx950 HIP kernels + host scene/BVH/loader C++)
behind the C ABI in ``include/dcrt.h``. Python here is a host mirror of the
reference's ``CScene`` / ``CWavefrontPathTracer`` interface over that ABI.
"""
from ._abi import (DCRTError, FEATURE_ALLOW_ANYHIT, FEATURE_DEFAULT, FEATURE_GGX_SAMPLE_VNDF, FEATURE_LIGHT_VISIBLE,  # noqa: F401
                   FEATURE_NO_FRONT_TO_BACK, FEATURE_WATERTIGHT, FILTER_BOX, FILTER_GAUSSIAN, FILTER_LANCZOS,
                   FILTER_MITCHELL, FILTER_TRIANGLE, FilterParams, FrameParams, LIB_PATH, load_library)
from .scene import Scene  # noqa: F401
from ._abi import PostFxParams  # noqa: F401
from .tracer import (HIT_DTYPE, RAY_DTYPE, WavefrontPathTracer, device_count, make_pipelines, make_rays, prepare_pipelines, probe_row_cost,  # noqa: F401
                     render_images_concurrently, save_bmp, srgb_thresholds)

__version__ = "0.1.0"


def version() -> str:
    return load_library().dcrt_version().decode()
