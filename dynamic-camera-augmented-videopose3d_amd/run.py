#!/usr/bin/env python3
"""Evaluation driver of the temporal-lifter path (drop-in for the FCN branch of the
reference's run.py --evaluate, run.py:290-309 model build, :400-417 device and
checkpoint, :862-995 per-action evaluation).

    python run.py --evaluate synthetic --fcn-architecture 3,3,3 --subjects-test '*'
    python run.py --evaluate epoch_60.bin -c checkpoint --causal --compute-dtype bf16

The reference reads hard-coded .npz paths (run.py:48,84) that ship nowhere, so the
dataset here is a seeded synthetic CMU-style split (subjects x actions, procedural
camera trajectories); .npz ingestion is §8(f) "next".  Sequences
live in HBM (common.generators), the lifter is the native MI355X model
(common.models.TemporalModel), Protocol #1 is the native mpjpe kernel.
"""
from __future__ import annotations

import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def synthetic_dataset(args, normalize=None):
    """Seeded synthetic split (vp3d_amd.synth.synthetic_split); keypoints normalised
    on device by common.camera.normalize_screen_coordinates unless `normalize` is given."""
    from vp3d_amd import synth
    if normalize is None:
        from common.camera import normalize_screen_coordinates as normalize
    return synth.synthetic_split(args.synthetic_subjects, args.synthetic_actions,
                                 args.synthetic_frames, args.joints, args.seed, normalize)


def group_actions(data, subjects):
    """action name (prefix before ' ') -> [(subject, action)] (run.py:866-878)."""
    out = {}
    for s in subjects:
        for a in data[s]:
            out.setdefault(a.split(" ")[0], []).append((s, a))
    return out


def run_evaluation(data, actions, make_generator, model_fn, metrics, action_filter=None):
    """Per-action evaluation + action-wise averages (run.py:906-987)."""
    from vp3d_amd.evaluate import camera_motion_pmcc, evaluate
    errs = {"p1": [], "p2": [], "p3": [], "vel": []}
    per_seq, infos, motion = [], [], []
    per_action = {}
    for key in actions:
        if action_filter is not None and not any(key.startswith(a) for a in action_filter):
            continue
        seqs = actions[key]
        gen = make_generator([data[s][a]["cameras"] for s, a in seqs],
                             [data[s][a]["positions_3d"] for s, a in seqs],
                             [data[s][a]["keypoints"] for s, a in seqs])
        res, e_seq, inf, mot = evaluate(gen, model_fn, metrics, key)
        per_action[key] = res
        for k, v in zip(("p1", "p2", "p3", "vel"), res):
            errs[k].append(v)
        per_seq += e_seq
        infos += inf
        motion += mot
    summary = {k: float(np.mean(v)) for k, v in errs.items()}
    print('Protocol #1   (MPJPE) action-wise average:', round(summary["p1"], 1), 'mm')
    print('Protocol #2 (P-MPJPE) action-wise average:', round(summary["p2"], 1), 'mm')
    print('Protocol #3 (N-MPJPE) action-wise average:', round(summary["p3"], 1), 'mm')
    print('Velocity      (MPJVE) action-wise average:', round(summary["vel"], 2), 'mm')
    pmcc = camera_motion_pmcc(per_seq, infos, motion)
    for k, v in pmcc.items():
        print(f'PMCC (MPJPE and {k.replace("_", " ")}):', v)
    return {"per_action": per_action, "summary": summary, "pmcc": pmcc}


def build_model(args, J):
    from common.models.TemporalModel import TemporalModel
    from vp3d_amd import synth
    fw = [int(x) for x in args.fcn_architecture.split(",")]
    jin = J + 6 if args.trajectory else J
    model = TemporalModel(jin, 2, J, filter_widths=fw, causal=args.causal, dropout=args.fcn_dropout,
                          channels=args.channels, dense=args.dense)
    print('INFO: Receptive field: {} frames'.format(model.receptive_field()))
    print('INFO: Trainable parameter count:', sum(p.numel() for p in model.parameters()))
    if args.evaluate == "synthetic" or not args.evaluate:
        sd = synth.lifter_state_dict([(k, tuple(v.shape)) for k, v in model.state_dict().items()],
                                     seed=args.seed)
        model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    else:
        path = os.path.join(args.checkpoint, args.evaluate)
        print('Loading checkpoint', path)
        ckpt = torch.load(path, map_location="cpu", weights_only=not args.trust_checkpoint)
        model.load_state_dict(ckpt["model_pos"])
    return model


def main(argv=None):
    from common.arguments import parse_args
    from common.generators import UnchunkedGenerator
    from vp3d_amd.evaluate import DeviceMetrics

    args = parse_args(argv)
    if args.model_name != "FCN":
        raise SystemExit(f"--use-model {args.model_name}: only the FCN lifter runs on this path")
    if not torch.cuda.is_available():
        raise SystemExit("run.py evaluates on the MI355X (no CPU fallback)")
    data = synthetic_dataset(args)
    subjects = list(data.keys()) if args.subjects_test in (None, "*") else args.subjects_test.split(",")
    model = build_model(args, args.joints).cuda().eval()
    model.set_compute_dtype(args.compute_dtype)
    pad = (model.receptive_field() - 1) // 2
    causal_shift = pad if args.causal else 0

    def make_generator(cams, p3d, p2d):
        return UnchunkedGenerator(cams, p3d, p2d, pad=pad, causal_shift=causal_shift,
                                  trajectory=args.trajectory).next_epoch()

    action_filter = None if args.actions == "*" else args.actions.split(",")
    print('Evaluating...')
    if not args.by_subject:
        return run_evaluation(data, group_actions(data, subjects), make_generator, model,
                              DeviceMetrics(), action_filter)
    out = {}
    for s in subjects:
        print('Evaluating on subject', s)
        out[s] = run_evaluation(data, group_actions(data, [s]), make_generator, model,
                                DeviceMetrics(), action_filter)
    return out


if __name__ == "__main__":
    main()
