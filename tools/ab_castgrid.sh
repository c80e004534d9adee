#!/bin/bash
# A/B (round 6): fewer resident cast workgroups per CU, so the other pipelines' MATERIAL waves
# can co-reside with a persistent cast launch (three pipelines, Cornell --steps 20)
set -e
export AB_CONFIGS="cornell" AB_STEPS=20 PASSES=2
export AB_VARIANTS="base
b7 DCRT_CAST_BLOCKS_PER_CU=7
b6 DCRT_CAST_BLOCKS_PER_CU=6
b5 DCRT_CAST_BLOCKS_PER_CU=5"
tools/ab_env2.sh
