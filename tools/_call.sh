set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for pass in 1 2; do
for cfg in spaceship coffee cornell; do
for vd in "0 0" "1 0" "1 32768" "1 131072"; do
  set -- $vd
  DCRT_VIRTUAL_START=$1 DCRT_DRAIN_PATHS=$2 timeout -k 10 300 python bench.py --config $cfg --steps 16 --warmup 2 --no-cpu-baseline --repeats 3 --roofline-images 1 --spaceship-spp 0 > gpurun_out/ab.json 2>gpurun_out/ab.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/ab.json'));print('$cfg virtual=$1 drain=$2', d['ms_per_spp'], d['repeat_ms_per_spp'])"
done
done
done
