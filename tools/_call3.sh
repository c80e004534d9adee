set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/profiles
export TMPDIR=/tmp
: > gpurun_out/profiles/r04_configs.jsonl
for item in "cornell" "coffee" "coffee --no-multiscattering" "spaceship" "spaceship_close" "lamp"; do
  set -- $item
  timeout -k 10 400 python bench.py --config $item --steps 16 --warmup 2 --no-cpu-baseline --repeats 3 --roofline-images 16 --spaceship-spp 0 > gpurun_out/cfg.json 2>gpurun_out/cfg.err || exit $?
  tail -1 gpurun_out/cfg.json >> gpurun_out/profiles/r04_configs.jsonl
  python -c "import json;d=json.load(open('gpurun_out/cfg.json'));print('$item', d['ms_per_spp'], d['repeat_ms_per_spp'], d['roofline'].get('frac'), d.get('pipeline_roofline',{}).get('frac'))"
done
timeout -k 10 600 python bench.py > gpurun_out/profiles/r04_bench_default.json 2>gpurun_out/bd.err || exit $?
timeout -k 10 600 python bench.py --steps 20 > gpurun_out/profiles/r04_bench_s20.json 2>gpurun_out/b20.err || exit $?
cat gpurun_out/profiles/r04_bench_default.json gpurun_out/profiles/r04_bench_s20.json
