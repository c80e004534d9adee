#!/bin/bash
# The N = 4 launch path rehearsed on one MI355X (four gloo ranks sharing the box's GPU), full size,
# with bench.py's N > 1 defaults (one calibrated cost-balanced band per rank, three image-interleaved
# pipelines), film compared bit for bit with one rank rendering the same 32 images.
set -e
mkdir -p gpurun_out
C="--warmup 1 --repeats 1 --no-cpu-baseline --spaceship-spp 0"
timeout -k 10 300 python bench.py $C --steps 32 --save-film gpurun_out/f1.npy > gpurun_out/r06_reh_n1.json
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 4 --dist-backend gloo $C --steps 8 --save-film gpurun_out/f4.npy > gpurun_out/r06_reh_n4.json
python - <<'PY'
import json, numpy as np
a, b = np.load("gpurun_out/f1.npy"), np.load("gpurun_out/f4.npy")
print("film shapes", a.shape, b.shape, "bit-identical:", bool(np.array_equal(a.view(np.uint32), b.view(np.uint32))))
d = json.loads([l for l in open("gpurun_out/r06_reh_n4.json") if l.startswith("{")][-1])
m = d["multi_gpu"]
print("n4 config:", d["config"]["parallelism"], "| partition", d["config"]["partition"], "interleave", d["config"]["interleave"])
print("per-rank render ms", m["per_rank_render_ms"], "reduce ms", m["per_rank_reduce_ms"])
print("rank 0 rows owned", m["rank0_rows_owned"], "rendered", m["rank0_rows_rendered"], "halo overhead", m["rank0_halo_overhead"])
print("calibration", m["calibration"])
PY
