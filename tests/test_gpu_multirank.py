"""Multi-rank bench path on one GPU box: two ranks (gloo, both on cuda:0) render their
film stripes and reduce; the reduced film must equal the single-rank film bit for bit."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_bench_film_equals_single_rank(tmp_path):
    common = ["--steps", "1", "--warmup", "0", "--width", "256", "--height", "144", "--bounces", "4",
              "--pool", str(1 << 16), "--no-cpu-baseline", "--roofline-images", "1", "--stripe", "16",
              "--spaceship-spp", "0"]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    single = tmp_path / "single.npy"
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), *common, "--save-film", str(single)],
                       capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    multi = tmp_path / "multi.npy"
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                        "--master-addr", "127.0.0.1", "--master-port", str(_port()), str(ROOT / "bench.py"),
                        "--gpus", "2", *common, "--dist-backend", "gloo", "--save-film", str(multi)],
                       capture_output=True, text=True, timeout=900, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(line) == 1 and '"n_gpus": 2' in line[0]
    import json
    d = json.loads(line[0])
    # the diagnosable multi-GPU fields: every rank's render time, the reduce, the halo overhead
    m = d["multi_gpu"]
    assert m["world_size"] == 2 and len(m["per_rank_render_ms"]) == 2 and len(m["per_rank_reduce_ms"]) == 2
    assert all(x > 0 for x in m["per_rank_render_ms"]) and all(x >= 0 for x in m["per_rank_reduce_ms"])
    assert m["rank0_rows_rendered"] >= m["rank0_rows_owned"] > 0 and m["rank0_halo_overhead"] >= 0
    assert d["repeats"] == 5 and len(d["repeat_ms_per_spp"]) == 5
    # N > 1 default: image-interleaved pipelines over one calibrated cost-balanced band per rank
    assert d["config"]["interleave"] is True and d["config"]["partition"] == "balanced"
    assert len(m["calibration"]["rank_ms_per_step"]) == 1 and len(m["calibration"]["rank_ms_per_step"][0]) == 2
    a, b = np.load(single), np.load(multi)
    # 2 images on 2 ranks vs 1 image on 1 rank: compare the 1-rank film of the same 2 images
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), *common, "--steps", "2", "--save-film", str(single)],
                       capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    a = np.load(single)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


def test_bench_gpus_without_launcher_starts_its_ranks(tmp_path):
    """`python bench.py --gpus 2` with no launcher: bench.py starts torch.distributed.run as a
    child process (before touching the GPU) and relays rank 0's line, which must say n_gpus 2
    -- never a silent one-process n_gpus 1 line. Both ranks share the box's one GPU (gloo)."""
    import json
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--dist-backend", "gloo", "--steps", "1",
                        "--warmup", "0", "--width", "256", "--height", "144", "--bounces", "4", "--pool", str(1 << 16),
                        "--no-cpu-baseline", "--roofline-images", "1", "--stripe", "16", "--spaceship-spp", "0",
                        "--repeats", "1"], capture_output=True, text=True, timeout=900, env=env)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert all(json.loads(l)["n_gpus"] != 1 for l in lines), lines
    assert r.returncode == 0, r.stderr[-3000:]
    assert len(lines) == 1 and json.loads(lines[0])["n_gpus"] == 2 and json.loads(lines[0])["multi_gpu"]["world_size"] == 2
    # a launcher that started a different number of ranks than --gpus: refused before any GPU work
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--steps", "1"], capture_output=True,
                       text=True, timeout=120, env=dict(env, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"))
    assert r.returncode == 2 and not [l for l in r.stdout.splitlines() if l.startswith("{")]


def test_bench_runs_other_baseline_configs(tmp_path):
    """bench.py --config: BASELINE configs[2] (coffee-like XML scene) through the same
    path; one JSON line with its own metric name and the ray totals."""
    import json
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--config", "coffee", "--steps", "1", "--warmup", "0",
                        "--no-cpu-baseline", "--scene-dir", str(tmp_path)], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(line) == 1
    d = json.loads(line[0])
    assert d["config"]["name"] == "coffee" and "coffee" in d["metric"] and d["config"]["rays"] > 0


def test_progressive_snapshots_give_the_same_film(tmp_path):
    """bench.py --snapshot-spp K (configs[4]'s progressive reduce every K images, two
    pipelines summed per snapshot): the last snapshot is the film of one pass, bit for bit."""
    common = ["--steps", "3", "--warmup", "0", "--width", "160", "--height", "96", "--bounces", "4",
              "--pool", str(1 << 16), "--no-cpu-baseline", "--roofline-images", "1", "--spaceship-spp", "0"]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    films = []
    for extra in ([], ["--snapshot-spp", "1"]):
        out = tmp_path / f"film{len(films)}.npy"
        r = subprocess.run([sys.executable, str(ROOT / "bench.py"), *common, *extra, "--save-film", str(out)],
                           capture_output=True, text=True, timeout=600, env=env)
        assert r.returncode == 0, r.stderr[-2000:]
        films.append(np.load(out))
    assert np.array_equal(films[0].view(np.uint32), films[1].view(np.uint32))


def test_bench_default_line_fields(tmp_path):
    """The default Cornell line's protocol fields: median of the repeats with each repeat
    listed, the cast roofline as a measured-HBM statement with the algorithmic fraction
    beside it, the pipeline figure labelled algorithmic, the CPU baseline's host, and the
    configs[3] spaceship leg (ms/spp, traversal counts, its own roofline)."""
    import json
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--steps", "2", "--warmup", "1", "--width", "320",
                        "--height", "180", "--pool", str(1 << 18), "--cpu-seconds", "1", "--spaceship-spp", "1",
                        "--scene-dir", str(tmp_path)], capture_output=True, text=True, timeout=900, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert d["repeats"] == 5 and len(d["repeat_ms_per_spp"]) == 5
    # N = 1: three pipelines over cost-balanced bands, not interleaved
    assert d["config"]["interleave"] is False and d["config"]["partition"] == "balanced"
    assert abs(d["ms_per_spp"] - sorted(d["repeat_ms_per_spp"])[2]) < 1e-3
    roof = d["roofline"]
    assert roof["frac_algorithmic"] > 0 and roof["bound"].startswith("lds/valu") and roof["scene_in_lds"]
    pipe = d["pipeline_roofline"]   # no PMC profile of a 320x180 workload: measured fields null
    assert pipe["frac"] is None and pipe["bound"].startswith("unmeasured") and pipe["frac_algorithmic"] > 0
    mat = d["material"]             # MATERIAL's HIP-event launch time from the roofline leg
    assert mat["launches"] > 0 and mat["avg_launch_us"] > 0
    cb = d["cpu_baseline"]
    assert cb["cores"] >= 1 and cb["nproc"] >= cb["cores"] and cb["cpu_model"]
    assert cb["config0"]["rays"] > 128 * 128 and cb["config0"]["ms_per_spp"] > 0   # BASELINE configs[0] in full
    assert "compute" in roof   # the VALU statement (null without a PMC profile of this workload)
    sp = d["spaceship"]
    assert sp["ms_per_spp"] > 0 and sp["roofline"]["per_shadow_ray"]["nodes"] > 0
    assert sp["roofline"]["bound"].startswith("memory latency") and not sp["roofline"]["scene_in_lds"]


def test_torch_rccl_buffer_interop():
    """The N-GPU film path's buffer handoff (libdcrt <-> torch tensor <-> RCCL reduce,
    device-side film add), in a fresh process: tools/interop_check.py."""
    r = subprocess.run([sys.executable, str(ROOT / "tools" / "interop_check.py"), str(_port())], capture_output=True,
                       text=True, timeout=600, env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0"))
    assert r.returncode == 0, (r.stdout[-1000:], r.stderr[-2000:])
    assert "copy True reduce True add True" in r.stdout

