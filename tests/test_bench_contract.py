"""The bench JSON contract, checked on the committed MI355X bench lines (CPU only).

bench.py prints one JSON line per run; the driver and the judge read `metric`, `value`,
`unit`, the timing fields, `roofline` (dominant kernel against its peak, with the PMC
traffic) and `cpu_baseline` (the oracle on the host cores).  These tests pin that shape on
the lines profiles/ holds for the headline run (config 4, N = 1), so a bench change that
drops or renames a field fails here before it reaches a GPU box.
"""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROFILES = os.path.join(REPO, "profiles")
HEADLINE = ["r02h_bench_bf16.json", "r02l_bench_default.json"]


def _line(name):
    with open(os.path.join(PROFILES, name)) as f:
        text = f.read().strip()
    try:
        return json.loads(text)  # a pretty-printed line (profiles/r05final_*)
    except json.JSONDecodeError:
        return json.loads(text.splitlines()[-1])


def test_current_default_line():
    """The round's last default line (config 4, f16x3): the accurate path is `value`, priced at
    the f16 peak / 3, with its legs -- bf16 / fp32, config 3, config 5 in fp32 and fp16, the
    sequence mode -- and the north-star gate met by every accurate leg."""
    d = _line("r06final_bench_default.json")
    with open(os.path.join(REPO, "BASELINE.json")) as f:
        base = json.load(f)
    assert d["metric"] == base["metric"] and d["dtype"] == "f16x3" and d["n_gpus"] == 1
    assert d["value"] == pytest.approx(65536 / (d["ms_per_step"] * 1e-3), rel=1e-3)
    r = d["roofline"]
    assert r["peak"] == pytest.approx(2500.0 / 3) and r["frac"] == pytest.approx(r["achieved"] / r["peak"], rel=1e-3)
    assert r["achieved"] == pytest.approx(r["flop_per_launch"] / (r["avg_launch_ms"] * 1e-3) / 1e12, rel=1e-3)
    p = d["parity"]
    assert p["f16x3_meets_north_star_1e-4mm"] and p["f16x3_mpjpe_delta_mm"] <= 1e-4
    assert p["fp32_mpjpe_delta_mm"] <= 1e-4 and p["reference_fp32_vs_fp64_mpjpe_delta_mm"] >= 0
    assert d["config5"]["fp32"]["parity"]["meets_north_star_1e-4mm"]
    for k in ("median", "p90", "p99"):
        assert d["config5"]["fp32"]["serve_latency_us"][k] > 0
    for k in ("f16x3", "fp32"):
        assert d["sequence"][k]["meets_north_star_1e-4mm"] and d["sequence"][k]["roofline"]["frac"] > 0
    assert d["config3"]["f16x3"]["mpjpe_delta_mm"] <= 1e-4
    c = d["cpu_baseline"]
    assert c["kind"] in ("port", "reference") and c["cores"] >= 1 and c["affinity_cpus"] >= 1
    # round 6: the CPU baseline's threads pinned one per physical core, the line's traffic taken
    # on the same build, faults checked after every leg, and the headline keys last
    assert c["threads_pinned"] >= c["cores"] and len(c["runs"]) == 5
    assert r["traffic"] is not None and r["traffic_source"]["same_build"]
    assert d["faults"] == 0
    assert list(d.keys())[-1] == "parity" and "roofline" in list(d.keys())[-7:]


@pytest.mark.parametrize("name", HEADLINE)
def test_headline_line_fields(name):
    d = _line(name)
    with open(os.path.join(REPO, "BASELINE.json")) as f:
        base = json.load(f)
    assert d["metric"] == base["metric"]
    for k in ("value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["higher_is_better"] is True and d["vs_baseline"] is None
    assert d["scaling"] == "strong" and d["config"]["global_batch"] == 65536
    assert "workload" in d["config"] and "model" not in d["config"]
    # value = global batch x steps / wall time; ms_per_step is the same clock
    assert d["value"] == pytest.approx(65536 / (d["ms_per_step"] * 1e-3), rel=1e-3)


@pytest.mark.parametrize("name", HEADLINE)
def test_roofline_and_cpu_baseline(name):
    d = _line(name)
    r = d["roofline"]
    assert r["bound"] in ("hbm", "mfma") and r["unit"] in ("GB/s", "TFLOP/s")
    assert r["frac"] == pytest.approx(r["achieved"] / r["peak"], rel=1e-3)
    assert r["peak"] == 2500.0  # bf16 dense MFMA peak (MI355X_MICROARCH.md)
    # achieved = algorithmic FLOP of the launch / its mean duration
    assert r["achieved"] == pytest.approx(r["flop_per_launch"] / (r["avg_launch_ms"] * 1e-3) / 1e12, rel=1e-3)
    assert r["traffic"] is None or r["traffic"] > 0
    c = d["cpu_baseline"]
    assert c["kind"] in ("port", "reference") and c["cores"] >= 1 and c["value"] > 0
    assert c["unit"] == d["unit"] and c["sample"]
    # the parity path rides in the same line and meets the north-star gate
    assert d["fp32"]["mpjpe_delta_mm"] <= 1e-4


def test_bench_cli_parses():
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--help"], capture_output=True,
                         text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    for flag in ("--gpus", "--steps", "--warmup", "--global-batch", "--traj", "--stream"):
        assert flag in out.stdout, flag


def _bench(args, env_extra, timeout=300):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.update(env_extra)
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], capture_output=True, text=True,
                          timeout=timeout, env=env, cwd=REPO)


def test_bench_gpus_n_launches_n_ranks_dry():
    """`bench.py --gpus 2` without a launcher starts 2 ranks itself (torch.distributed.run child,
    gloo in the dry mode): ONE line from rank 0 labelled n_gpus 2, the two shards covering the
    global batch."""
    r = _bench(["--gpus", "2", "--steps", "3", "--warmup", "1"], {"VP3D_BENCH_DRY": "1"})
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["dry_run"] is True and d["steps"] == 3
    assert d["config"]["windows_per_gpu"] == 32768 and d["config"]["windows_all_ranks"] == 65536


def test_bench_world_size_mismatch_refused():
    """A launcher's WORLD_SIZE that differs from --gpus is refused (rc 2), never mislabelled."""
    r = _bench(["--gpus", "2"], {"WORLD_SIZE": "4", "VP3D_BENCH_DRY": "1"}, timeout=120)
    assert r.returncode == 2 and "WORLD_SIZE=4" in r.stderr


def test_bench_gpus_n_refused_without_n_devices():
    """--gpus N > visible GPUs (none in this container) outside a rehearsal: rc 2, no ranks."""
    r = _bench(["--gpus", "8"], {}, timeout=120)
    assert r.returncode == 2 and "needs 8 visible GPUs" in r.stderr


def test_emit_line_puts_headline_keys_last(capsys):
    """The driver keeps only the tail of stdout: roofline, cpu_baseline, faults and parity of the
    headline come after the long legs."""
    sys.path.insert(0, REPO)
    import bench
    bench.emit_line({"metric": "m", "parity": {"a": 1}, "value": 1, "roofline": {}, "config5": {"x": 1},
                     "cpu_baseline": {}, "faults": 0})
    keys = list(json.loads(capsys.readouterr().out).keys())
    assert keys == ["metric", "value", "config5", "roofline", "cpu_baseline", "faults", "parity"]


def test_cpu_baseline_child_pins_threads():
    """The CPU baseline runs the oracle in a child process with one torch thread pinned per
    distinct physical core (oracle/cpu_timer.py), here on a tiny lifter."""
    sys.path.insert(0, REPO)
    import numpy as np
    import bench
    from vp3d_amd import synth
    from common.models.TemporalModel import TemporalModelOptimized1f
    m = TemporalModelOptimized1f(17, 2, 17, [3, 3], channels=32)
    sd = synth.lifter_state_dict([(k, tuple(v.shape)) for k, v in m.state_dict().items()], seed=0)
    x = np.random.default_rng(0).standard_normal((4, 9, 17, 2)).astype(np.float32)
    c = bench.cpu_baseline(bench.cpu_job("lifter", sd, {"x": x}, fw=[3, 3], strided=True), 4, "poses/s",
                           "test", repeats=2, target_s=0.05)
    assert c["value"] > 0 and c["cores"] == len(c["pinned_cpus"]) >= 1 and len(c["runs"]) == 2
    assert c["threads_pinned"] >= 1 and set(c["pinned_threads_ran_on"]) <= set(c["pinned_cpus"])
