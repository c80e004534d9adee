#!/bin/bash
# A/B (round 6, final tree): visits per phase-A check on the entry-free Cornell cast
set -e
PASSES=2 AB_STEPS=20 tools/ab_libs.sh
