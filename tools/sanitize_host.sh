#!/bin/bash
# Host code under AddressSanitizer + UBSan (no GPU needed): builds the sanitized libdcrt
# (directcomputeraytracing_amd.build.build_sanitized) and runs the CPU suite against it --
# the OBJ / XML loaders, the BVH builder, the scene flattening and the C ABI, including the
# pins against the reference's own tinyobjloader / RapidXml. Any ASan or UBSan report fails it.
#   tools/sanitize_host.sh [pytest args]   -> exit status of pytest
set -u
cd "$(dirname "$0")/.."
LIB=$(python3 -c "from directcomputeraytracing_amd.build import build_sanitized; print(build_sanitized())") || exit 1
RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
export DCRT_LIB="$LIB"
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
LD_PRELOAD="$RT" python3 -m pytest tests -q -m "not gpu" -p no:cacheprovider "$@"
