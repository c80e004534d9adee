set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
AB_CONFIGS="spaceship spaceship_close" AB_STEPS=8 PASSES=2 BENCH_ARGS="--repeats 3" AB_VARIANTS="guard
guard_nocache DCRT_NO_LDS_CACHE=1
guard_blk5 DCRT_CAST_BLOCKS_PER_CU=5" bash tools/ab_env2.sh
for cfg in spaceship coffee lamp cornell; do timeout -k 10 300 python bench.py --config $cfg --steps 1 --warmup 0 --no-cpu-baseline --repeats 1 --roofline-images 1 --spaceship-spp 0 2>/dev/null | tail -1 | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('$cfg', d['roofline']['launch'])" || exit 1; done
