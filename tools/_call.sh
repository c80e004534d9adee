set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for pass in 1 2; do
for cfg in coffee lamp spaceship; do
for pm in 1 0; do
  DCRT_MATERIAL_LDS_PARTIAL=$pm timeout -k 10 300 python bench.py --config $cfg --steps 16 --warmup 2 --no-cpu-baseline --repeats 3 --roofline-images 2 --spaceship-spp 0 > gpurun_out/ab.json 2>gpurun_out/ab.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/ab.json'));print('$cfg partial=$pm', d['ms_per_spp'], d['repeat_ms_per_spp'], 'mat us', d['material']['avg_launch_us'], 'lds', d['roofline']['launch']['material_lds'])"
done
done
done
