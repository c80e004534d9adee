set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
DCRT_COMPACT_STACK=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "spaceship or config or pair or traversal or trace_rays" > gpurun_out/pytest_compact.log 2>&1 || { tail -30 gpurun_out/pytest_compact.log; exit 1; }
tail -1 gpurun_out/pytest_compact.log
for c in 0 1; do DCRT_COMPACT_STACK=$c timeout -k 10 300 python bench.py --config spaceship --steps 1 --warmup 0 --no-cpu-baseline --repeats 1 --roofline-images 1 --spaceship-spp 0 2>/dev/null | tail -1 | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('compact $c', d['roofline']['launch'])" || exit 1; done
AB_CONFIGS="spaceship spaceship_close" AB_STEPS=8 PASSES=2 BENCH_ARGS="--repeats 3" AB_VARIANTS="base
compact DCRT_COMPACT_STACK=1" bash tools/ab_env2.sh
