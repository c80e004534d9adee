set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_CONFIGS="spaceship spaceship_close lamp" AB_STEPS=8 PASSES=2 BENCH_ARGS="--repeats 3" AB_VARIANTS="off
d4k DCRT_DRAIN_PATHS=4096
d32k DCRT_DRAIN_PATHS=32768" bash tools/ab_env2.sh
