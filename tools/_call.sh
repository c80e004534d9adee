set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bd.json 2>gpurun_out/bd.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/bd.json'));print('default', d['value'], d['ms_per_spp'], d['repeat_ms_per_spp'], d['roofline']['launch'])"
