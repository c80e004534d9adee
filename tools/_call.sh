set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
DCRT_LIB=gpu_ab/b_xcd.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "virtual or config or spaceship or render" > gpurun_out/pytest_xcd.log 2>&1; rc=$?; echo "pytest(xcd) rc=$rc"; tail -3 gpurun_out/pytest_xcd.log
[ $rc -eq 0 ] || exit $rc
AB_CONFIGS="spaceship_close spaceship cornell" PASSES=2 bash tools/ab_configs2.sh
