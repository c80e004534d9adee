set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
CONFIG=cornell STEPS=20 OUT=gpurun_out/prof_c20 bash tools/prof_config.sh || exit $?
python tools/pmc_traffic.py gpurun_out/prof_c20 gpurun_out/r04pre_c20 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --traffic-json gpurun_out/r04pre_c20_pmc_traffic.json --spaceship-spp 0 > gpurun_out/bench_s20.json 2> gpurun_out/bench_s20.err; echo "bench rc=$?"
