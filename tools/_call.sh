set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for cfg in spaceship spaceship_close cornell; do
  OUT=gpurun_out/seq_$cfg; mkdir -p $OUT
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$GRAFT_REPO_ROOT/$OUT" -o trace -- python3 "$GRAFT_REPO_ROOT/bench.py" --config $cfg --steps 8 --warmup 0 --no-cpu-baseline --streams 1 --repeats 1 --roofline-images 1 --spaceship-spp 0 > "$GRAFT_REPO_ROOT/$OUT/bench.log" 2>&1) || exit $?
  f=$(ls $OUT/*kernel_trace.csv | head -1)
  python tools/kseq.py $f 0 30 > $OUT/seq.txt; head -34 $OUT/seq.txt
done
for pass in 1 2; do
for cfg in cornell spaceship_close; do
  timeout -k 10 300 python bench.py --config $cfg --steps 16 --warmup 2 --no-cpu-baseline --repeats 3 --roofline-images 16 --spaceship-spp 0 > gpurun_out/b_$cfg.json 2>gpurun_out/b_$cfg.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/b_$cfg.json'));r=d['roofline'];print('$cfg', d['ms_per_spp'], d['repeat_ms_per_spp'], d['value'], r['per_ext_ray'], r['per_shadow_ray'], r['avg_launch_us'], r['extension_rays']/16/(d['config']['resolution'][0]*d['config']['resolution'][1]), r['shadow_rays']/16/(d['config']['resolution'][0]*d['config']['resolution'][1]))"
done
done
