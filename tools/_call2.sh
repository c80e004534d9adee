set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_CONFIGS="coffee lamp" PASSES=2 BENCH_ARGS="--repeats 3" AB_VARIANTS="r12k
r0 DCRT_CAST_LDS_RESERVE=0" bash tools/ab_env2.sh
for r in 0 12288; do for cfg in coffee lamp; do DCRT_CAST_LDS_RESERVE=$r timeout -k 10 300 python bench.py --config $cfg --steps 1 --warmup 0 --no-cpu-baseline --repeats 1 --roofline-images 1 --spaceship-spp 0 2>/dev/null | tail -1 | python -c "import sys,json; d=json.loads(sys.stdin.read()); l=d['roofline']['launch']; print('$cfg reserve $r', l['cast_grid'], l['cached_nodes'])" || exit 1; done; done
