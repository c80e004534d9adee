set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/profiles
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
WORKLOADS="cornell 20 c20;cornell 64 c64" bash tools/refresh_profiles.sh || exit $?
cp gpurun_out/profiles/r04_*_pmc_traffic.json profiles/
timeout -k 10 600 python bench.py > gpurun_out/profiles/r04_bench_default.json 2>gpurun_out/bd.err || exit $?
timeout -k 10 600 python bench.py --steps 20 > gpurun_out/profiles/r04_bench_s20.json 2>gpurun_out/b20.err || exit $?
python -c "
import json
for f in ('r04_bench_default','r04_bench_s20'):
    d=json.load(open('gpurun_out/profiles/'+f+'.json')); print(f, d['value'], d['ms_per_spp'], d['repeat_ms_per_spp'], 'cast', d['roofline']['avg_launch_us'], d['roofline']['frac'], 'mat', d['material']['avg_launch_us'], d['material']['frac'], 'pipe', d['pipeline_roofline']['frac'], 'spaceship', d['spaceship']['ms_per_spp'])
"
