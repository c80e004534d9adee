set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for dp in 0 4096 32768; do
  DCRT_DRAIN_PATHS=$dp timeout -k 10 300 python bench.py --config spaceship --steps 16 --warmup 2 --no-cpu-baseline --repeats 3 --roofline-images 1 --spaceship-spp 0 > gpurun_out/ab.json 2>gpurun_out/ab.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/ab.json'));print('spaceship drain=$dp', d['ms_per_spp'], d['repeat_ms_per_spp'])"
done
AB_CONFIGS="cornell spaceship" PASSES=2 bash tools/ab_configs2.sh
