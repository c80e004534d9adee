set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/profiles
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
timeout -k 10 600 python bench.py > gpurun_out/profiles/r04_bench_default.json 2>gpurun_out/bd.err || exit $?
timeout -k 10 600 python bench.py --steps 20 > gpurun_out/profiles/r04_bench_s20.json 2>gpurun_out/b20.err || exit $?
python -c "
import json
for f in ('r04_bench_default','r04_bench_s20'):
    d=json.load(open('gpurun_out/profiles/'+f+'.json')); print(f, d['value'], d['ms_per_spp'], d['repeat_ms_per_spp'], 'cast', d['roofline']['avg_launch_us'], d['roofline']['frac'], 'pipe', d['pipeline_roofline']['frac'], 'spaceship', d['spaceship']['ms_per_spp'], d['spaceship']['roofline']['frac'], d['spaceship']['roofline']['avg_launch_us'])
"
