set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_CONFIGS="spaceship_close spaceship" AB_STEPS=8 PASSES=2 BENCH_ARGS="--repeats 3" bash tools/ab_configs2.sh
