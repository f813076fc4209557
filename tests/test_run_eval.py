"""run.py --evaluate plumbing (BASELINE config 1: H36M-shaped 17 joints, 27-frame RF).

The golden run_eval_27.npz is the reference's own evaluation loop (run.py:697-771,
906-971) on the seeded synthetic split.  CPU: the harness driven by the oracle
(generator, model, metrics) must reproduce it.  GPU: `run.main` end to end (device
generators, native lifter fp32, native mpjpe) within 1e-4 mm on Protocol #1.
"""
import json
import os

import numpy as np
import pytest
import torch

GOLD = os.path.join(os.path.dirname(__file__), "golden", "run_eval_27.npz")


def _golden():
    g = np.load(GOLD, allow_pickle=False)
    return dict(zip([str(a) for a in g["actions"]], g["errors"])), g["pmcc"], json.loads(str(g["meta"]))


def _argv(meta):
    return ["--evaluate", "synthetic", "--fcn-architecture", ",".join(map(str, meta["fw"])),
            "--channels", str(meta["channels"]), "--synthetic-subjects", str(meta["subjects"]),
            "--synthetic-actions", str(meta["actions"]), "--synthetic-frames", str(meta["frames"]),
            "--seed", str(meta["seed"]), "--subjects-test", "*"]


class OracleMetrics:
    def mpjpe(self, p, t):
        from oracle.loss_ref import mpjpe
        return float(mpjpe(p, t))

    def n_mpjpe(self, p, t):
        from oracle.loss_ref import n_mpjpe
        return float(n_mpjpe(p, t))

    def p_mpjpe(self, p, t):
        from oracle.loss_ref import p_mpjpe
        return p_mpjpe(p.numpy().copy(), t.numpy().copy())  # numpy float32, as run.py accumulates it

    def mpjve(self, p, t):
        from oracle.loss_ref import mean_velocity_error
        return mean_velocity_error(p.numpy(), t.numpy())


def test_run_eval_plumbing_cpu_oracle():
    import run
    from common.arguments import parse_args
    from oracle import camera_ref, generators_ref
    from oracle.temporal_ref import lifter_forward
    from vp3d_amd import synth

    want, want_pmcc, meta = _golden()
    args = parse_args(_argv(meta))
    data = run.synthetic_dataset(args, normalize=camera_ref.normalize_screen_coordinates)
    from common.models.TemporalModel import TemporalModel
    m = TemporalModel(17, 2, 17, meta["fw"], channels=meta["channels"])
    sd = synth.lifter_state_dict([(k, tuple(v.shape)) for k, v in m.state_dict().items()], seed=meta["seed"])
    pad = (m.receptive_field() - 1) // 2

    def make_gen(cams, p3d, p2d):
        for cam, (bc, b3, b2) in zip(cams, generators_ref.unchunked_sequences(cams, p3d, p2d, pad, 0)):
            info = {k: cam[k] for k in cam if k.startswith("cam_")}
            yield (torch.from_numpy(bc.astype(np.float32)), torch.from_numpy(b3.astype(np.float32)),
                   torch.from_numpy(b2.astype(np.float32)), info)

    res = run.run_evaluation(data, run.group_actions(data, list(data)), make_gen,
                             lambda x: lifter_forward(sd, x, meta["fw"]), OracleMetrics())
    for k, v in want.items():
        np.testing.assert_allclose(res["per_action"][k], v, rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose([res["pmcc"][k] for k in res["pmcc"]], want_pmcc, rtol=1e-5)


@pytest.mark.gpu
def test_run_main_gpu_matches_reference():
    import run
    want, want_pmcc, meta = _golden()
    res = run.main(_argv(meta))
    for k, v in want.items():
        got = np.asarray(res["per_action"][k])
        print(k, got, v)
        assert abs(got[0] - v[0]) <= 1e-4, (k, got[0], v[0])          # Protocol #1, mm
        np.testing.assert_allclose(got[1:], v[1:], rtol=0, atol=1e-3)  # post-path protocols
    np.testing.assert_allclose([res["pmcc"][k] for k in res["pmcc"]], want_pmcc, atol=1e-4)
