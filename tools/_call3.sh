set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench_final.json 2>gpurun_out/bench_final.err || exit $?
python -c "import json;d=json.loads(open('gpurun_out/bench_final.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_spp'], d['repeat_ms_per_spp'], 'spaceship', d['spaceship']['ms_per_spp'])"
