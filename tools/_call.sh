set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/profiles
export TMPDIR=/tmp
WORKLOADS="cornell 20 c20;cornell 64 c64;cornell 16 c16" bash tools/refresh_profiles.sh || exit $?
cp gpurun_out/profiles/r04_*_pmc_traffic.json profiles/
timeout -k 10 600 python bench.py > gpurun_out/profiles/r04_bench_default.json 2>gpurun_out/bd.err || exit $?
timeout -k 10 600 python bench.py --steps 20 > gpurun_out/profiles/r04_bench_s20.json 2>gpurun_out/b20.err || exit $?
python -c "
import json
for f in ('r04_bench_default','r04_bench_s20'):
    d=json.load(open('gpurun_out/profiles/'+f+'.json')); print(f, d['value'], d['ms_per_spp'], d['repeat_ms_per_spp'], 'cast', d['roofline']['avg_launch_us'], d['roofline']['frac'], d['roofline']['compute']['valu_issue_frac'], 'mat', d['material']['avg_launch_us'], d['material']['frac'], 'pipe', d['pipeline_roofline']['frac'], 'spaceship', d['spaceship']['ms_per_spp'])
"
timeout -k 10 400 python bench.py --config cornell --steps 16 --warmup 2 --no-cpu-baseline --repeats 3 --roofline-images 16 --spaceship-spp 0 > gpurun_out/cfg.json 2>gpurun_out/cfg.err || exit $?
tail -1 gpurun_out/cfg.json > gpurun_out/profiles/r04_config_cornell.json
python -c "import json;d=json.load(open('gpurun_out/cfg.json'));print('cornell16', d['ms_per_spp'], d['repeat_ms_per_spp'], d['roofline'].get('frac'), d.get('pipeline_roofline',{}).get('frac'))"
