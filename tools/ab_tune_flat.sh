#!/bin/bash
# A/B (round 6): refill / park thresholds re-swept for the entry-free cache-only cast (Cornell --steps 20)
set -e
export AB_CONFIGS="cornell" AB_STEPS=20 PASSES=2
export AB_VARIANTS="t36_24
t32_24 DCRT_TRAVERSAL_TUNE=32,24
t40_24 DCRT_TRAVERSAL_TUNE=40,24
t36_20 DCRT_TRAVERSAL_TUNE=36,20
t36_28 DCRT_TRAVERSAL_TUNE=36,28
t44_28 DCRT_TRAVERSAL_TUNE=44,28"
tools/ab_env2.sh
