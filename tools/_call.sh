set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 8 --warmup 1 --dist-backend gloo --no-cpu-baseline --spaceship-spp 0 > gpurun_out/two_rank.json 2>gpurun_out/two_rank.err; rc=$?; echo "rc=$rc"; tail -c 1500 gpurun_out/two_rank.json; tail -5 gpurun_out/two_rank.err
