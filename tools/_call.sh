set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_CONFIGS="spaceship cornell" PASSES=2 bash tools/ab_configs2.sh || exit $?
for cfg in spaceship; do
  OUT=gpurun_out/seq_$cfg; mkdir -p $OUT
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$GRAFT_REPO_ROOT/$OUT" -o trace -- python3 "$GRAFT_REPO_ROOT/bench.py" --config $cfg --steps 8 --warmup 0 --no-cpu-baseline --streams 1 --repeats 1 --roofline-images 1 --spaceship-spp 0 > "$GRAFT_REPO_ROOT/$OUT/bench.log" 2>&1) || exit $?
  f=$(ls $OUT/*kernel_trace.csv | head -1)
  python tools/kseq.py $f 0 48 > $OUT/seq.txt; cat $OUT/seq.txt
done
