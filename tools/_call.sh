set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit $?
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
AB_CONFIGS="spaceship cornell" PASSES=2 BENCH_ARGS="--repeats 3" bash tools/ab_configs2.sh
for lib in a_base b_filmdirect; do
  OUT=gpurun_out/seq_$lib; mkdir -p $OUT
  (cd /tmp && DCRT_LIB=$GRAFT_REPO_ROOT/gpu_ab/$lib.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$GRAFT_REPO_ROOT/$OUT" -o trace -- python3 "$GRAFT_REPO_ROOT/bench.py" --config spaceship --steps 8 --warmup 0 --no-cpu-baseline --streams 1 --repeats 1 --roofline-images 1 --spaceship-spp 0 > "$GRAFT_REPO_ROOT/$OUT/bench.log" 2>&1) || exit $?
  grep film_kernel $OUT/trace_kernel_stats.csv | head -2
done
