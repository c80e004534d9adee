set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for pass in 1 2; do
for b in 0 6 5; do
  if [ $b = 0 ]; then unset DCRT_CAST_BLOCKS_PER_CU; else export DCRT_CAST_BLOCKS_PER_CU=$b; fi
  timeout -k 10 300 python bench.py --config cornell --steps 16 --warmup 2 --no-cpu-baseline --repeats 3 --roofline-images 2 --spaceship-spp 0 > gpurun_out/ab.json 2>gpurun_out/ab.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/ab.json'));print('cornell castBlocksPerCU=$b', d['ms_per_spp'], d['repeat_ms_per_spp'], 'cast us', d['roofline']['avg_launch_us'], d['roofline']['launch']['cast_grid'])"
done
unset DCRT_CAST_BLOCKS_PER_CU
for gm in 2 4; do
  DCRT_CAST_GRID_MUL=$gm timeout -k 10 300 python bench.py --config cornell --steps 16 --warmup 2 --no-cpu-baseline --repeats 3 --roofline-images 2 --spaceship-spp 0 > gpurun_out/ab.json 2>gpurun_out/ab.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/ab.json'));print('cornell castGridMul=$gm', d['ms_per_spp'], d['repeat_ms_per_spp'], 'cast us', d['roofline']['avg_launch_us'], d['roofline']['launch']['cast_grid'])"
done
for st in 2 3; do
  timeout -k 10 300 python bench.py --config cornell --steps 16 --warmup 2 --no-cpu-baseline --repeats 3 --roofline-images 2 --spaceship-spp 0 --streams $st > gpurun_out/ab.json 2>gpurun_out/ab.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/ab.json'));print('cornell streams=$st', d['ms_per_spp'], d['repeat_ms_per_spp'])"
done
done
