"""ORACLE (test infrastructure only): the timing child of bench.py's `cpu_baseline` leg.

bench.py writes one job file (inputs, the model's state dict, what to run) and starts

    python -m oracle.cpu_timer JOB.npz

as a CHILD process (the bench process keeps the GPU; this one never touches it) whose
environment pins the torch-CPU threads one per physical core: the parent picks the CPUs
(`pick_cores`: one logical CPU of each of the least-busy physical cores inside the parent's
sched_getaffinity set, from a /proc/stat sample), sets OMP_NUM_THREADS / OMP_PLACES={c0},{c1},... / OMP_PROC_BIND=close,
and this module narrows its own affinity to those CPUs before torch loads.  It then times the
oracle (the reference's torch-CPU op sequence, oracle/temporal_ref.py etc.) exactly like the
in-process baseline did -- one warm-up, a calibration run, `repeats` timed runs of ~target_s --
and prints ONE JSON line: rates, the observed thread -> CPU map (/proc/self/task/*/stat field
39, the CPU each thread last ran on, and its allowed list) and the run spread.

Job kinds (meta["kind"]):
  lifter       oracle.temporal_ref.lifter_forward(sd, x, fw, causal, strided)   (TemporalModel.py:62-198)
  train        oracle.train_ref.TrainLoop(sd, fw).step(x, tgt)                   (run.py:451-487)
  transformer  oracle.seq_lifter_ref.transformer_forward(sd, x, xc, 4, 2, 3)     (CamTransformer.py:95-205)
  lstm         oracle.seq_lifter_ref.lstm_forward(sd, x, xc, 128, 2, 3)          (CamLSTM.py:47-129)
"""
from __future__ import annotations

import json
import os
import sys
import time


def physical_cores(cpus):
    """{(package, core): [logical cpus]} for the given logical CPUs (sysfs topology)."""
    groups = {}
    for c in sorted(cpus):
        base = f"/sys/devices/system/cpu/cpu{c}/topology"
        try:
            with open(f"{base}/physical_package_id") as f:
                pkg = int(f.read())
            with open(f"{base}/core_id") as f:
                core = int(f.read())
        except (OSError, ValueError):
            pkg, core = 0, c
        groups.setdefault((pkg, core), []).append(c)
    return groups


def cpu_busy(cpus, window_s=0.3):
    """{logical cpu: busy fraction over `window_s`} from two /proc/stat samples (empty when
    /proc/stat is unreadable)."""
    def sample():
        out = {}
        try:
            with open("/proc/stat") as f:
                for ln in f:
                    if ln.startswith("cpu") and ln[3:4].isdigit():
                        parts = ln.split()
                        v = [int(x) for x in parts[1:]]
                        idle = v[3] + (v[4] if len(v) > 4 else 0)  # idle + iowait
                        out[int(parts[0][3:])] = (sum(v[:8]), idle)
        except (OSError, ValueError):
            pass
        return out
    a = sample()
    time.sleep(window_s)
    b = sample()
    busy = {}
    for c in cpus:
        if c in a and c in b:
            dt = b[c][0] - a[c][0]
            busy[c] = 1.0 - (b[c][1] - a[c][1]) / dt if dt > 0 else 0.0
    return busy


def pick_cores(n=None):
    """One logical CPU of each of the `n` least-busy physical cores in this process's affinity
    set (all cores when n is None), plus the count of physical cores available.  The boxes are
    shared by the other GPUs' jobs: a fixed choice (the first n cores) landed on cores other
    processes kept busy (round 6: 2,908 -> 271 poses/s over five runs), so the choice follows a
    0.3 s /proc/stat sample -- a core's busy fraction is that of its busier sibling, and the
    idler sibling is the one pinned."""
    try:
        allowed = os.sched_getaffinity(0)
    except (AttributeError, OSError):
        allowed = set(range(os.cpu_count() or 1))
    groups = physical_cores(allowed)
    busy = cpu_busy(allowed) if n is not None else {}
    ranked = sorted(groups.values(), key=lambda v: (max(busy.get(c, 0.0) for c in v), v[0]))
    picks = [min(v, key=lambda c: (busy.get(c, 0.0), c)) for v in ranked]
    return (picks if n is None else sorted(picks[:n])), len(picks)


def cgroup_cpu_quota():
    """cgroup v2 cpu.max as CPUs (quota / period), or None when unlimited / unreadable."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
        return None if q == "max" else round(int(q) / int(p), 2)
    except (OSError, ValueError):
        return None


def child_env(cpus):
    """Environment for a timing child pinned one thread per CPU in `cpus`."""
    env = dict(os.environ)
    env["OMP_NUM_THREADS"] = str(len(cpus))
    env["OMP_PLACES"] = ",".join("{%d}" % c for c in cpus)
    env["OMP_PROC_BIND"] = "close"
    env["VP3D_CPU_TIMER_CPUS"] = ",".join(str(c) for c in cpus)
    return env


def _thread_map():
    """[(tid, last cpu, allowed list)] of this process's threads."""
    out = []
    for tid in sorted(os.listdir("/proc/self/task"), key=int):
        try:
            with open(f"/proc/self/task/{tid}/stat") as f:
                fields = f.read().rsplit(")", 1)[1].split()
            last = int(fields[36])  # field 39 of stat (processor), after pid and (comm)
            with open(f"/proc/self/task/{tid}/status") as f:
                allowed = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("Cpus_allowed_list")), "")
            out.append((int(tid), last, allowed))
        except (OSError, ValueError, IndexError):
            pass
    return out


def _run_fn(meta, arrays):
    import numpy as np
    import torch
    sd = {k[3:]: arrays[k] for k in arrays if k.startswith("sd:")}
    kind = meta["kind"]
    kw = meta.get("kwargs", {})
    if kind == "lifter":
        from oracle.temporal_ref import lifter_forward
        x = torch.from_numpy(arrays["x"])
        return lambda: lifter_forward(sd, x, kw["fw"], causal=kw.get("causal", False),
                                      strided=kw.get("strided", False))
    if kind == "train":
        from oracle.train_ref import TrainLoop
        loop = TrainLoop(sd, kw["fw"], lr=1e-3, amsgrad=True)
        x, t = arrays["x"], arrays["tgt"]
        return lambda: loop.step(x, t)
    if kind in ("transformer", "lstm"):
        from oracle.seq_lifter_ref import lstm_forward, transformer_forward
        sdt = {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in sd.items()}
        x, xc = torch.from_numpy(arrays["x"]), torch.from_numpy(arrays["xc"])
        if kind == "transformer":
            return lambda: transformer_forward(sdt, x, xc, 4, 2, 3)
        return lambda: lstm_forward(sdt, x, xc, 128, 2, 3)
    raise ValueError(f"unknown job kind {kind!r}")


def main(path):
    cpus = [int(c) for c in os.environ.get("VP3D_CPU_TIMER_CPUS", "").split(",") if c]
    if cpus:
        os.sched_setaffinity(0, cpus)  # before torch creates its thread pool
    import numpy as np
    import torch
    with np.load(path, allow_pickle=False) as z:
        arrays = {k: z[k] for k in z.files}
    meta = json.loads(str(arrays.pop("meta")))
    threads = len(cpus) if cpus else int(meta.get("threads", 1))
    torch.set_num_threads(threads)
    run_once = _run_fn(meta, arrays)
    units = int(meta["units"])
    target_s, repeats = float(meta["target_s"]), int(meta["repeats"])
    with torch.no_grad() if meta["kind"] != "train" else torch.enable_grad():
        run_once()  # warm-up: thread pool spin-up, allocator
        t = time.perf_counter()
        run_once()  # calibration on a warm run
        t1 = max(time.perf_counter() - t, 1e-3)
        reps = max(1, int(round(target_s / t1)))
        rates = []
        for _ in range(repeats):
            t = time.perf_counter()
            for _ in range(reps):
                run_once()
            rates.append(reps * units / (time.perf_counter() - t))
    tmap = _thread_map()
    med = float(np.median(rates))
    print(json.dumps({
        "value": round(med, 3), "runs": [round(r, 3) for r in rates], "reps": reps,
        "timed_s": round(sum(reps * units / r for r in rates), 2),
        "spread": round((max(rates) - min(rates)) / med, 4),
        "torch_threads": torch.get_num_threads(), "pinned_cpus": cpus,
        "thread_cpu_map": [{"tid": t_, "last_cpu": c, "allowed": a} for t_, c, a in tmap],
    }), flush=True)


if __name__ == "__main__":
    main(sys.argv[1])
