#!/bin/bash
# A/B (round 6): the one-GPU pipeline construction -- three / four banded pipelines against
# three / four image-interleaved ones (Cornell --steps 20, and coffee --steps 16)
set -e
export AB_CONFIGS="cornell" AB_STEPS=20 PASSES=2
export AB_VARIANTS="b3 --streams 3
b4 --streams 4
i3 --streams 3 --interleave on
i4 --streams 4 --interleave on"
tools/ab_bargs.sh
export AB_CONFIGS="coffee" AB_STEPS=16 PASSES=1
export AB_VARIANTS="b2 --streams 2
b3 --streams 3
i2 --streams 2 --interleave on
i3 --streams 3 --interleave on"
tools/ab_bargs.sh
