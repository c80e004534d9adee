set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for pass in 1 2; do
for cfg in cornell; do
for ml in 16384 0; do
  DCRT_MATERIAL_LDS=$ml timeout -k 10 300 python bench.py --config $cfg --steps 16 --warmup 2 --no-cpu-baseline --repeats 3 --roofline-images 4 --spaceship-spp 0 > gpurun_out/ab.json 2>gpurun_out/ab.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/ab.json'));print('$cfg materialLds=$ml', d['ms_per_spp'], d['repeat_ms_per_spp'], 'material us', d['material']['avg_launch_us'], 'cast us', d['roofline']['avg_launch_us'])"
done
done
done
