"""Render a few Cornell images with optional material overrides (for PMC probes)."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from directcomputeraytracing_amd import Scene, WavefrontPathTracer, scenes  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "default"
s = Scene((1920, 1080))
scenes.setup_cornell(s, 1920, 1080, 8)
if mode == "diffuse":
    for i in range(s.material_count):
        s.set_material(i, 0, (0.7, 0.7, 0.7), 1.0)
t = WavefrontPathTracer(path_pool_size=1 << 21, iterations_per_render=16)
t.on_scene_loaded(s)
t.render_images(0, 3)
t.synchronize()
print(mode, t.counters())
