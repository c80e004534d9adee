set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_CONFIGS="coffee lamp" PASSES=2 BENCH_ARGS="--repeats 3" bash tools/ab_configs2.sh
for cfg in coffee lamp; do for lib in a_base b_glob7; do DCRT_LIB=gpu_ab/$lib.so timeout -k 10 300 python bench.py --config $cfg --steps 1 --warmup 0 --no-cpu-baseline --repeats 1 --roofline-images 1 --spaceship-spp 0 2>/dev/null | tail -1 | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('$cfg $lib', d['roofline']['launch'])" || exit 1; done; done
