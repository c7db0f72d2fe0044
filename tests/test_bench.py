"""bench.py's contract pieces that run without a GPU: refusing more ranks than
visible devices, the BASELINE config labels, and that the committed PMC
traffic summary belongs to the kernel source being shipped (bench.py replays
it only then, and labels it)."""
import importlib.util
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _load(path, name):
    spec = importlib.util.spec_from_file_location(name, os.path.join(ROOT, path))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_bench_refuses_more_ranks_than_gpus():
    import torch
    if torch.cuda.device_count() > 0:
        return  # only meaningful on a machine without GPUs
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "1", "--warmup", "0"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 2, r.stdout + r.stderr
    assert "one rank per GPU" in r.stderr


def test_shape_labels_name_baseline_configs():
    bench = _load("bench.py", "bench_mod")
    assert bench.shape_label(8, 12, 256).startswith("C3+C4")
    assert bench.shape_label(4, 6, 64).startswith("C2")
    assert bench.shape_label(10, 14, 1024).startswith("C5")
    assert bench.shape_label(8, 12, 512).startswith("north-star")
    assert bench.shape_label(3, 5, 7) == ""


def test_committed_traffic_matches_shipped_kernel_source():
    bench = _load("bench.py", "bench_mod2")
    tool = _load("tools/pmc_traffic.py", "pmc_traffic")
    assert bench.kernel_source_id() == tool.kernel_source_id()
    tj = json.load(open(os.path.join(ROOT, "profiles", "r02", "pmc_traffic.json")))
    assert tj["kernel_source"] == bench.kernel_source_id(), \
        "apply kernel changed since its PMC passes: re-run tools/gpu_r02.sh pmc_fetch pmc_write"
    assert tj["config"] == "8/12 L=8388608 nobj=128" and tj["kernel"] == "rs_apply_queue_kernel"
    alg = 128 * 4 * 8388608 * 12
    assert abs(tj["hbm_bytes_per_launch"] / alg - 1) < 0.01  # no wasted re-reads
