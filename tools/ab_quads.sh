#!/bin/bash
# A/B (round 6): the quad node layout (DCRT_NODE_QUADS=1) on the pair-traversal configs
set -e
export AB_CONFIGS="spaceship_close spaceship" AB_STEPS=8 PASSES=2
export AB_VARIANTS="base
quads DCRT_NODE_QUADS=1"
tools/ab_env2.sh
