#!/bin/bash
# A/B (round 6): the cache-only IDENT cast over the entry-free node order (no BLAS-entry step per
# visit) against the same kernel over PackBVH's order; Cornell --steps 20, interleaved passes
set -e
python - <<'PY'
from directcomputeraytracing_amd import Scene, WavefrontPathTracer, scenes
s = Scene((1920, 1080)); scenes.setup_cornell(s, 1920, 1080, 8)
t = WavefrontPathTracer(path_pool_size=1 << 24); t.on_scene_loaded(s)
print("info:", {k: v for k, v in t.info().items() if k in ("cast_identity", "stack_lds_rows", "cached_nodes", "cast_waves_per_cu", "cast_grid")})
t.destroy()
PY
export AB_CONFIGS="cornell" AB_STEPS=20 PASSES=3
export AB_VARIANTS="flat
noflat DCRT_FLAT_CAST=0"
tools/ab_env2.sh
