set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_CONFIGS="spaceship spaceship_close" AB_STEPS=8 PASSES=2 BENCH_ARGS="--repeats 3" AB_VARIANTS="b256
b128 DCRT_CAST_BLOCK=128
b64 DCRT_CAST_BLOCK=64" bash tools/ab_env2.sh
for b in 256 128 64; do DCRT_CAST_BLOCK=$b timeout -k 10 300 python bench.py --config spaceship --steps 1 --warmup 0 --no-cpu-baseline --repeats 1 --roofline-images 1 --spaceship-spp 0 2>/dev/null | tail -1 | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('block $b', d['roofline']['launch'])" || exit 1; done
