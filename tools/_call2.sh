set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
bash tools/lane_util.sh > gpurun_out/lane_util.txt 2>&1; rc=$?; cat gpurun_out/lane_util.txt; exit $rc
