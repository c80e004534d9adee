#!/bin/bash
# A/B (round 6): the film kernel's grid (every sequenced iteration launches it; it returns at once
# unless a batch completed, but its workgroups wait for slots behind the other pipelines' persistent casts)
set -e
export AB_CONFIGS="cornell" AB_STEPS=20 PASSES=2
export AB_VARIANTS="base
g1024 DCRT_FILM_GRID=1024
g256 DCRT_FILM_GRID=256"
tools/ab_env2.sh
