set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/profiles
export TMPDIR=/tmp
WORKLOADS="spaceship 16 s16;spaceship_close 16 sclose" bash tools/refresh_profiles.sh || exit $?
cp gpurun_out/profiles/r04_*_pmc_traffic.json profiles/
timeout -k 10 600 python bench.py > gpurun_out/profiles/r04_bench_default.json 2>gpurun_out/bd.err || exit $?
timeout -k 10 600 python bench.py --steps 20 > gpurun_out/profiles/r04_bench_s20.json 2>gpurun_out/b20.err || exit $?
python -c "
import json
for f in ('r04_bench_default','r04_bench_s20'):
    d=json.load(open('gpurun_out/profiles/'+f+'.json')); print(f, d['value'], d['ms_per_spp'], d['repeat_ms_per_spp'], 'cast', d['roofline']['avg_launch_us'], d['roofline']['frac'], 'pipe', d['pipeline_roofline']['frac'], 'spaceship', d['spaceship']['ms_per_spp'], d['spaceship'].get('roofline',{}).get('frac'))
"
: > gpurun_out/profiles/r04_configs_sp.jsonl
for item in "spaceship" "spaceship_close"; do
  timeout -k 10 400 python bench.py --config $item --steps 16 --warmup 2 --no-cpu-baseline --repeats 3 --roofline-images 16 --spaceship-spp 0 > gpurun_out/cfg.json 2>gpurun_out/cfg.err || exit $?
  tail -1 gpurun_out/cfg.json >> gpurun_out/profiles/r04_configs_sp.jsonl
  python -c "import json;d=json.load(open('gpurun_out/cfg.json'));print('$item', d['ms_per_spp'], d['repeat_ms_per_spp'], d['value'], d['roofline'].get('frac'), d.get('pipeline_roofline',{}).get('frac'), d['roofline'].get('frac_algorithmic'))"
done
