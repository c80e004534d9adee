#!/bin/bash
# Build libdcrt.so of git revision $1 into gpu_ab/$2.so (A/B against the working tree).
set -eu
rev=$1; name=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d /tmp/dcrt_rev.XXXX)
git -C "$ROOT" archive "$rev" | tar -x -C "$tmp"
mkdir -p "$ROOT/gpu_ab"
(cd "$tmp" && python3 -c "from directcomputeraytracing_amd.build import build_native; build_native()" >/dev/null)
cp "$tmp/directcomputeraytracing_amd/libdcrt.so" "$ROOT/gpu_ab/$name.so"
rm -rf "$tmp"
echo "gpu_ab/$name.so <- $rev"
