set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_CONFIGS="cornell" PASSES=2 bash tools/ab_configs2.sh || exit $?
for pass in 1 2; do
for mg in 4 2 8; do
  DCRT_MATERIAL_GRID=$mg timeout -k 10 300 python bench.py --config cornell --steps 16 --warmup 2 --no-cpu-baseline --repeats 3 --roofline-images 4 --spaceship-spp 0 > gpurun_out/ab.json 2>gpurun_out/ab.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/ab.json'));print('cornell materialGrid=$mg', d['ms_per_spp'], d['repeat_ms_per_spp'], 'material us', d['material']['avg_launch_us'], 'cast us', d['roofline']['avg_launch_us'])"
done
done
