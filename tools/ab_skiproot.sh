#!/bin/bash
# A/B (round 6): rays starting strictly inside the root's box take the root's descend -- and the
# near children's while their boxes hold the origin -- without the box tests (trav_skip_root)
set -e
export AB_CONFIGS="cornell coffee" AB_STEPS=16 PASSES=2
export AB_VARIANTS="l0 DCRT_SKIP_ROOT=0
l1 DCRT_SKIP_ROOT=1
l4 DCRT_SKIP_ROOT=4
l16 DCRT_SKIP_ROOT=16"
tools/ab_env2.sh
