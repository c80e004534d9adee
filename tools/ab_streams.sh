#!/bin/bash
# A/B (round 6, final tree): pipelines per GPU for the Cornell headline
set -e
export AB_CONFIGS="cornell" AB_STEPS=20 PASSES=2
export AB_VARIANTS="s3 --streams 3
s2 --streams 2
s4 --streams 4"
tools/ab_bargs.sh
