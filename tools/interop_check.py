#!/usr/bin/env python3
"""GPU check of the multi-GPU film path's buffer interop, in one fresh process.

bench.py --gpus N hands torch (PyTorch-ROCm's HIP runtime, RCCL) device buffers to
libdcrt.so (the system ROCm's HIP runtime) and back: copy_film_device into a torch
tensor, dist.reduce (RCCL, world size 1 here) of that tensor, add_film_device between
two tracers. torch must initialise the device before the tracers are created (the
order bench.py uses); then every value must come back bit-identical.
"""
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    import numpy as np
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", sys.argv[1] if len(sys.argv) > 1 else "29611")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    from directcomputeraytracing_amd import Scene, WavefrontPathTracer, scenes
    s = Scene((160, 96))
    scenes.setup_cornell(s, 160, 96, 4)
    tracers = []
    try:
        for _ in range(2):
            t = WavefrontPathTracer(path_pool_size=1 << 16, device=0)
            tracers.append(t)
            t.on_scene_loaded(s)
            t.clear_film()
            t.render_images(0, 2)
        a, b = tracers
        ref = a.read_film().reshape(-1)
        buf = torch.zeros(ref.size, dtype=torch.float32, device="cuda")
        a.copy_film_device(buf.data_ptr())
        torch.cuda.synchronize()
        ok_copy = np.array_equal(buf.cpu().numpy().view(np.uint32), ref.view(np.uint32))
        dist.reduce(buf, dst=0, op=dist.ReduceOp.SUM)
        torch.cuda.synchronize()
        ok_reduce = np.array_equal(buf.cpu().numpy().view(np.uint32), ref.view(np.uint32))
        a.add_film_device(b.film_device_ptr())
        ok_add = np.array_equal(a.read_film().reshape(-1).view(np.uint32), (ref + b.read_film().reshape(-1)).view(np.uint32))
    finally:
        for t in tracers:
            t.destroy()
        dist.destroy_process_group()
    print(f"copy {ok_copy} reduce {ok_reduce} add {ok_add}")
    sys.exit(0 if ok_copy and ok_reduce and ok_add else 1)


if __name__ == "__main__":
    main()
