set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
WORKLOADS="${WL:-coffee 16 coffee;coffee 16 coffee_noms --no-multiscattering;spaceship_close 16 sclose}" bash tools/refresh_profiles.sh
