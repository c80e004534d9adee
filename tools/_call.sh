set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "virtual or megakernel" > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for pass in 1 2; do
for cfg in spaceship lamp; do
for dp in 0 4096 32768; do
  DCRT_DRAIN_PATHS=$dp timeout -k 10 300 python bench.py --config $cfg --steps 16 --warmup 2 --no-cpu-baseline --repeats 3 --roofline-images 1 --spaceship-spp 0 > gpurun_out/ab.json 2>gpurun_out/ab.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/ab.json'));print('$cfg drain=$dp', d['ms_per_spp'], d['repeat_ms_per_spp'])"
done
done
done
timeout -k 10 300 python bench.py --steps 16 --warmup 2 --no-cpu-baseline --repeats 3 --roofline-images 1 --spaceship-spp 0 --mode megakernel > gpurun_out/ab.json 2>gpurun_out/ab.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/ab.json'));print('cornell megakernel', d['ms_per_spp'], d['repeat_ms_per_spp'])"
