"""Regenerate the golden fixtures in tests/golden/ (deterministic; no reference code runs).

* cornell_box.obj/.mtl -- the procedural config-1/2 scene (directcomputeraytracing_amd.scenes)
* bxdf_luts.npz        -- the six R16_UNORM BxDF LUTs from the oracle's restatement of
                          BxDFTexturesBuilding.hlsl (full 4096 x batches Monte Carlo per texel)
* kat.json             -- small known-answer vectors (RNG, Morton, SplitMix64, camera rays)

Usage: python tests/golden/make_golden.py [--luts]
"""
import json
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent.parent
sys.path.insert(0, str(ROOT))


def main():
    from directcomputeraytracing_amd import scenes
    from directcomputeraytracing_amd.build import build_oracle
    build_oracle()
    import oracle
    scenes.write_cornell_box(HERE)
    if "--luts" in sys.argv:
        luts = oracle.build_luts(threads=8)
        np.savez_compressed(HERE / "bxdf_luts.npz", **oracle.luts_to_arrays(luts))
        print("wrote", HERE / "bxdf_luts.npz")


if __name__ == "__main__":
    main()
