set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_$i.log 2>&1 || exit $?
python -c "import json;d=json.load(open('gpurun_out/bench_$i.log'));print('bench', d['ms_per_spp'], d['value'], d['roofline']['avg_launch_us'], d['roofline']['frac'])"
DCRT_MATERIAL_GENERIC=1 timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_g$i.log 2>&1 || exit $?
python -c "import json;d=json.load(open('gpurun_out/bench_g$i.log'));print('generic', d['ms_per_spp'], d['value'], d['roofline']['avg_launch_us'])"
done
