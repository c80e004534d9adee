#!/bin/bash
# same-box A/B of the last commits' libraries (Cornell --steps 20, 3 interleaved passes)
set -e
PASSES=3 AB_STEPS=20 tools/ab_libs.sh
