"""Device-side faults surface where results are consumed.

A forward refuses to start while a fault of an EARLIER forward on its handle is pending, so
the only forward nothing would check is the last one of a run.  `vp3d_amd.evaluate.evaluate`
(run.py:697-740's loop) calls the model's `sync_status()` after its loop, so a fault in the
final forward of an evaluation raises instead of returning an MPJPE; `run.main` (run.py
--evaluate) then ends with the exception (a non-zero exit from the command line).
"""
import numpy as np
import pytest
import torch

from helpers import make_model
from vp3d_amd import synth

pytestmark = pytest.mark.gpu


class _OneBatch:
    """An UnchunkedGenerator stand-in yielding one batch: its forward is the last one."""

    def __init__(self, x, y3d):
        self.x, self.y3d = x, y3d

    def next_epoch(self):
        yield None, self.y3d, self.x, {}


def test_evaluate_raises_split_k_fault_of_final_forward(monkeypatch):
    """Split-K fault injection (VP3D_A4_SPLIT=2 + VP3D_A4_SPLIT_DROP=1: every owner tile of the
    partial last rounds times out) on the ONLY -- hence final -- forward of an evaluation of
    8,192 Optimized1f windows in f16x3: evaluate() raises RuntimeError naming split-K."""
    from vp3d_amd.evaluate import DeviceMetrics, evaluate
    monkeypatch.setenv("VP3D_A4_SPLIT", "2")
    model, _ = make_model(True, (3, 3, 3, 3, 3), False, 1024)
    B = 8192
    x = torch.from_numpy(synth.normalized_windows(5, "x8192_243", B, 243)).cuda()
    y3d = torch.from_numpy(synth.gt_poses(3, "gt", B, 17).reshape(B, 1, 17, 3).astype(np.float32)).cuda()
    model.cuda().eval().set_compute_dtype("f16x3")
    gen = _OneBatch(x, y3d)
    res, _, _, _ = evaluate(gen, model, DeviceMetrics(), verbose=False)  # clean run: no fault
    assert np.isfinite(res).all()
    monkeypatch.setenv("VP3D_A4_SPLIT_DROP", "1")
    monkeypatch.setenv("VP3D_A4_SPLIT_SPIN_TICKS", "100000")
    with pytest.raises(RuntimeError, match="split-K"):
        evaluate(gen, model, DeviceMetrics(), verbose=False)
    monkeypatch.delenv("VP3D_A4_SPLIT_DROP")
    monkeypatch.delenv("VP3D_A4_SPLIT_SPIN_TICKS")
    model.sync_status()  # reported once, then cleared
    res2, _, _, _ = evaluate(gen, model, DeviceMetrics(), verbose=False)
    assert res2 == res


def test_run_evaluate_raises_f16x3_fault_of_final_sequence(monkeypatch):
    """run.py --evaluate --compute-dtype f16x3 on a split whose only (so final) sequence has
    keypoints past the f16 range: the expand's range guard flags it, evaluate's closing
    sync_status raises, and run.main ends with that RuntimeError instead of printing an MPJPE."""
    import run
    orig = run.synthetic_dataset

    def poisoned(args, normalize=None):
        data = orig(args, normalize)
        for s in data:
            for a in data[s]:
                kp = data[s][a]["keypoints"][-1]
                data[s][a]["keypoints"][-1] = kp * 1e7
        return data
    argv = ["--evaluate", "synthetic", "--fcn-architecture", "3,3,3", "--channels", "1024",
            "--synthetic-subjects", "1", "--synthetic-actions", "1", "--synthetic-frames", "200",
            "--seed", "0", "--subjects-test", "*", "--compute-dtype", "f16x3"]
    res = run.main(argv)  # the clean split evaluates
    assert np.isfinite(res["summary"]["p1"])
    monkeypatch.setattr(run, "synthetic_dataset", poisoned)
    with pytest.raises(RuntimeError, match="f16x3"):
        run.main(argv)


def test_pending_f16x3_fault_lets_fp32_run(monkeypatch):
    """a pending f16x3 range fault refuses f16x3 forwards only; the fp32 re-run its
    message recommends goes through, and the fault is still reported by sync_status."""
    model, _ = make_model(True, (3, 3, 3, 3, 3), False, 1024)
    x = torch.from_numpy(synth.normalized_windows(5, "x64_243", 64, 243)).cuda()
    model.cuda().eval()
    with torch.no_grad():
        ref32 = model(x).cpu().numpy()
        model.set_compute_dtype("f16x3")
        model(x * 1e6)
        torch.cuda.synchronize()
        with pytest.raises(RuntimeError, match="f16x3"):
            model(x)
        model.set_compute_dtype("fp32")
        y32 = model(x).cpu().numpy()
        with pytest.raises(RuntimeError, match="non-finite"):
            model.sync_status()
        model.sync_status()
    assert np.array_equal(y32, ref32)
