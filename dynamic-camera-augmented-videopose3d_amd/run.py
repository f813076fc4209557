#!/usr/bin/env python3
"""Training and evaluation driver of the temporal-lifter path (drop-in for the FCN
branch of the reference's run.py: :290-309 model build, :400-417 device and
checkpoint, :424-590 the training loop, :653-673 its entry, :862-995 per-action
evaluation), and the --evaluate path of the fork's trajectory lifters
(--use-model Transformer | LSTM-Coupled: :311-363 model build, :712-713 the
sliding_window dispatch).

    python run.py -e 60 -c checkpoint --subjects-train S1,S2 --subjects-test S3   # train
    python run.py --evaluate synthetic --fcn-architecture 3,3,3 --subjects-test '*'
    python run.py --evaluate epoch_60.bin -c checkpoint --causal --compute-dtype bf16
    python run.py --use-model Transformer --evaluate epoch_80.bin -c checkpoint -d CMU

Data: `-d h36m | CMU | CMU_3DPW` reads the reference's .npz layout from --data-dir
(data_3d_<d>.npz, data_2d_<d>_<keypoints>.npz; the reference hard-codes its paths,
run.py:48,84) and prepares it as run.py:65-124 does (vp3d_amd.datasets); `-d synthetic`
(default) is a seeded CMU-style split (subjects x actions, procedural camera
trajectories).  Every action carries one entry per camera view
(H36M: 4).  Sequences live in HBM (common.generators), the lifter is the native
MI355X model (common.models.TemporalModel), Protocol #1 is the native mpjpe kernel.
"""
from __future__ import annotations

import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)

import time  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402

from vp3d_amd.checkpoint import load_checkpoint  # noqa: E402


def synthetic_dataset(args, normalize=None):
    """Seeded synthetic split (vp3d_amd.synth.synthetic_split) in run.py's per-view form;
    keypoints normalised on device by common.camera.normalize_screen_coordinates unless
    `normalize` is given."""
    from vp3d_amd import synth
    if normalize is None:
        from common.camera import normalize_screen_coordinates as normalize
    raw = synth.synthetic_split(args.synthetic_subjects, args.synthetic_actions,
                                args.synthetic_frames, args.joints, args.seed, normalize)
    return {s: {a: {k: [d[k]] for k in ("positions_3d", "keypoints", "cameras")} for a, d in acts.items()}
            for s, acts in raw.items()}


def load_data(args, stride=None):
    """The split run.py evaluates / trains on: synthetic or the reference's .npz files,
    every `stride`-th frame (default --downsample; 1 = undecimated)."""
    from vp3d_amd.datasets import downsample, load_dataset
    if args.dataset == "synthetic":
        data = synthetic_dataset(args)
    else:
        if args.trajectory and args.dataset == "humaneva":
            raise SystemExit("--trajectory needs camera intrinsics; HumanEva publishes none (humaneva_dataset.py)")
        _, data, _ = load_dataset(args.dataset, args.data_dir, args.keypoints)
    return downsample(data, args.downsample if stride is None else stride)


def deterministic_random(min_value, max_value, data):
    """Hash-seeded integer in [min_value, max_value) (reference common/utils.py:44-47)."""
    import hashlib
    digest = hashlib.sha256(data.encode()).digest()
    raw_value = int.from_bytes(digest[:4], byteorder='little', signed=False)
    return int(raw_value / (2 ** 32 - 1) * (max_value - min_value)) + min_value


def subset_views(cams, p3d, p2d, subset=1.0, stride=1):
    """The tail of the reference's fetch (run.py:168-180) on undecimated views: with
    subset < 1 every view keeps round(len // stride * subset) * stride frames starting at
    deterministic_random(0, len - n + 1, str(len)), every stride-th of them; otherwise
    every stride-th frame (--downsample).  The per-frame camera extrinsics are sliced with
    the poses -- the reference leaves camera params whole, which only its static-camera
    datasets tolerate; here K.E stays aligned with the frames it belongs to."""
    if subset >= 1 and stride <= 1:
        return cams, p3d, p2d
    cams, p3d, p2d = list(cams), list(p3d), list(p2d)
    for i in range(len(p2d)):
        if subset < 1:
            L = len(p2d[i])
            n = int(round(L // stride * subset) * stride)
            start = deterministic_random(0, L - n + 1, str(L))
            sl = slice(start, start + n, stride)
        else:
            sl = slice(None, None, stride)
        p2d[i] = p2d[i][sl]
        if p3d is not None:
            p3d[i] = p3d[i][sl]
        if cams is not None and "extrinsics" in cams[i]:
            c = dict(cams[i])
            c["extrinsics"] = c["extrinsics"][sl]
            cams[i] = c
    return cams, p3d, p2d


def joint_counts(data):
    """(2D joints, 3D joints) of a prepared split."""
    d = next(iter(next(iter(data.values())).values()))
    return int(d["keypoints"][0].shape[-2]), int(d["positions_3d"][0].shape[-2])


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
        gen = make_generator(*_views(data, seqs))
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


def _views(data, seqs):
    """(cameras, poses_3d, poses_2d) lists over every view of the (subject, action) pairs
    (run.py:879-904 fetch_actions)."""
    cams, p3d, p2d = [], [], []
    for s, a in seqs:
        d = data[s][a]
        assert len(d["positions_3d"]) == len(d["keypoints"]) == len(d["cameras"]), "Camera count mismatch"
        cams += d["cameras"]
        p3d += d["positions_3d"]
        p2d += d["keypoints"]
    return cams, p3d, p2d


SEQ_MODELS = ("Transformer", "LSTM-Coupled", "LSTM-Uncoupled")
SEQ_RECEPTIVE_FIELD = 243  # run.py:312 / :334 / :364


def build_seq_model(args, J, J_out, announce=True):
    """--use-model Transformer | LSTM-Coupled | LSTM-Uncoupled (reference run.py:311-393):
    the fork's trajectory lifters at the parsed hyper-parameters (2D keypoints in, the
    per-frame camera matrices taken separately by sliding_window).  Weights: the
    checkpoint's 'model_pos' (run.py:403-409, through the weights-only loader), or with
    --evaluate synthetic torch's default init under manual_seed(--seed)."""
    from common.models.CamLSTM import CoupledLSTM, UncoupledLSTM
    from common.models.CamTransformer import CoupledTransformer
    if args.model_name == "Transformer":
        model = CoupledTransformer(J, 2, J_out, 3, d_model=args.d_model, num_layers=args.num_layers,
                                   n_heads=args.n_heads, dim_feedforward=args.dim_feedforward,
                                   head_layers=[int(x) for x in args.transformer_head_architecture.split(",")],
                                   dropout=args.transformer_dropout)
    else:
        cls = CoupledLSTM if args.model_name == "LSTM-Coupled" else UncoupledLSTM
        model = cls(J, 2, J_out, 3, hidden_size=args.lstm_hidden_features, num_cells=args.lstm_cells,
                    head_layers=[int(x) for x in args.lstm_head_architecture.split(",")],
                    dropout=args.lstm_dropout)
    if announce:
        print('INFO: Trainable parameter count:', sum(p.numel() for p in model.parameters()))
    if args.evaluate and args.evaluate != "synthetic":
        path = os.path.join(args.checkpoint, args.evaluate)
        print('Loading checkpoint', path)
        ckpt = load_checkpoint(path, trust=args.trust_checkpoint)
        if "epoch" in ckpt:
            print('This model was trained for {} epochs'.format(ckpt["epoch"]))
        model.load_state_dict(ckpt["model_pos"])
    return model


def build_model(args, J, announce=True, J_out=None):
    from common.models.TemporalModel import TemporalModel
    from vp3d_amd import synth
    J_out = J if J_out is None else J_out
    if args.model_name in SEQ_MODELS:
        return build_seq_model(args, J, J_out, announce)
    fw = [int(x) for x in args.fcn_architecture.split(",")]
    jin = J + 6 if args.trajectory else J
    model = TemporalModel(jin, 2, J_out, filter_widths=fw, causal=args.causal, dropout=args.fcn_dropout,
                          channels=args.channels, dense=args.dense)
    if announce:
        print('INFO: Receptive field: {} frames'.format(model.receptive_field()))
        print('INFO: Trainable parameter count:', sum(p.numel() for p in model.parameters()))
    if args.evaluate == "synthetic" or not args.evaluate:
        sd = synth.lifter_state_dict([(k, tuple(v.shape)) for k, v in model.state_dict().items()],
                                     seed=args.seed)
        model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    else:
        path = os.path.join(args.checkpoint, args.evaluate)
        print('Loading checkpoint', path)
        ckpt = load_checkpoint(path, trust=args.trust_checkpoint)
        model.load_state_dict(ckpt["model_pos"])
    return model


def fetch(data, subjects, action_filter=None):
    """(cameras, poses_3d, poses_2d) lists over every view of the given subjects
    (run.py:126-182)."""
    seqs = [(s, a) for s in subjects for a in data[s]
            if action_filter is None or any(a.startswith(f) for f in action_filter)]
    return _views(data, seqs)


def train(args, n_epochs, train_generator, test_generator, model_pos_train, model_pos, optimizer,
          lr, lr_decay, save_state=True, resume=None, log=print):
    """The reference's epoch loop (run.py:424-590) for the temporal FCN: per batch the
    train-mode forward, mpjpe, backward and Adam step on the MI355X; per epoch the
    evaluation of the copied weights on the test generator, the exponential lr decay, the
    BatchNorm momentum decay 0.1 -> 0.001 and the checkpoint.  Returns the per-epoch
    (train, valid) losses in metres and the best validation error."""
    from common.loss import mpjpe

    losses_train, losses_valid = [], []
    epoch = 0
    initial_momentum, final_momentum = 0.1, 0.001
    if resume is not None:  # run.py:436-445
        epoch = resume["epoch"]
        if resume.get("optimizer") is not None:
            optimizer.load_state_dict(resume["optimizer"])
            train_generator.set_random_state(resume["random_state"])
        lr = resume["lr"]
    best = float("inf")
    while epoch < n_epochs:
        t0 = time.time()
        sum_train = 0.0
        N = 0
        model_pos_train.train()
        for batch_cam, batch_3d, batch_2d in train_generator.next_epoch():
            pred = model_pos_train(batch_2d)
            loss = mpjpe(pred, batch_3d)
            optimizer.zero_grad()
            loss.backward()
            optimizer.step()
            n = batch_3d.shape[0] * batch_3d.shape[1]
            sum_train += n * loss.item()
            N += n
        losses_train.append(sum_train / N)
        with torch.no_grad():
            model_pos.load_state_dict(model_pos_train.state_dict())
            model_pos.eval()
            if not args.no_eval:
                sum_valid = 0.0
                N = 0
                for batch_cam, batch_3d, batch_2d, _ in test_generator():
                    loss = mpjpe(model_pos(batch_2d), batch_3d)
                    n = batch_3d.shape[0] * batch_3d.shape[1]
                    sum_valid += n * loss.item()
                    N += n
                losses_valid.append(sum_valid / N)
                best = min(best, losses_valid[-1])
        elapsed = (time.time() - t0) / 60
        if args.no_eval:
            log('[%d] time %.2f lr %f 3d_train %f' % (epoch + 1, elapsed, lr, losses_train[-1] * 1000))
        else:
            log('[%d] time %.2f lr %f 3d_train %f 3d_valid %f' % (
                epoch + 1, elapsed, lr, losses_train[-1] * 1000, losses_valid[-1] * 1000))
        lr *= lr_decay
        for group in optimizer.param_groups:
            group["lr"] *= lr_decay
        epoch += 1
        momentum = initial_momentum * np.exp(-epoch / args.epochs * np.log(initial_momentum / final_momentum))
        model_pos_train.set_bn_momentum(momentum)
        if save_state and epoch % args.checkpoint_frequency == 0:
            os.makedirs(args.checkpoint, exist_ok=True)
            path = os.path.join(args.checkpoint, 'epoch_{}.bin'.format(epoch))
            log('Saving checkpoint to', path)
            torch.save({'epoch': epoch, 'lr': lr, 'random_state': train_generator.random_state(),
                        'optimizer': optimizer.state_dict(), 'model_pos': model_pos_train.state_dict()}, path)
    return {"train": losses_train, "valid": losses_valid, "best_valid": best}


def train_main(args, data):
    """`run.py` without --evaluate (run.py:653-673): ChunkedGenerator batches of
    batch_size // stride chunks of `stride` frames, Adam(lr, amsgrad=True), train()."""
    from common.generators import ChunkedGenerator, UnchunkedGenerator
    from vp3d_amd.train import Adam

    subjects = list(data.keys())
    subjects_train = subjects if args.subjects_train in (None, "*") else args.subjects_train.split(",")
    subjects_test = subjects if args.subjects_test in (None, "*") else args.subjects_test.split(",")
    action_filter = None if args.actions == "*" else args.actions.split(",")
    print("Training Subjects: ", ", ".join(subjects_train))
    print("Test Subjects: ", ", ".join(subjects_test))
    j2, j3 = joint_counts(data)
    model_pos_train = build_model(args, j2, J_out=j3).cuda()
    model_pos = build_model(args, j2, announce=False, J_out=j3).cuda()
    pad = (model_pos.receptive_field() - 1) // 2
    causal_shift = pad if args.causal else 0
    # `data` is undecimated here: the training views get the reference fetch's --subset /
    # --downsample rule (run.py:168-180, fetch(..., subset=args.subset) at :656), the test
    # views --downsample only (run.py:657)
    cams_tr, p3d_tr, p2d_tr = subset_views(*fetch(data, subjects_train, action_filter), subset=args.subset,
                                           stride=args.downsample)
    cams_te, p3d_te, p2d_te = subset_views(*fetch(data, subjects_test, action_filter), stride=args.downsample)
    resume = None
    if args.resume:
        path = os.path.join(args.checkpoint, args.resume)
        print('Loading checkpoint', path)
        # a run.py checkpoint holds the generator's numpy RandomState (run.py:566): the
        # weights-only loader admits exactly that (vp3d_amd.checkpoint)
        resume = load_checkpoint(path, trust=args.trust_checkpoint)
        model_pos_train.load_state_dict(resume["model_pos"])
    optimizer = Adam(model_pos_train.parameters(), lr=args.learning_rate, amsgrad=True)
    train_generator = ChunkedGenerator(args.batch_size // args.stride, cams_tr, p3d_tr, p2d_tr, args.stride,
                                       pad=pad, causal_shift=causal_shift, shuffle=True,
                                       trajectory=args.trajectory)

    def test_generator():
        return UnchunkedGenerator(cams_te, p3d_te, p2d_te, pad=pad, causal_shift=causal_shift,
                                  trajectory=args.trajectory).next_epoch()

    print('INFO: Training on {} frames'.format(sum(p.shape[0] for p in p2d_tr)))
    # Reference quirk kept for drop-in output: run.py:673 calls train() without lr /
    # lr_decay, so the optimiser starts at -lr but decays by train()'s default 0.95 (-lrd
    # is parsed and unused) and the logged lr starts at train()'s default 0.001.
    return train(args, args.epochs, train_generator, test_generator, model_pos_train, model_pos, optimizer,
                 0.001, 0.95, save_state=True, resume=resume)


def main(argv=None):
    from common.arguments import parse_args
    from common.generators import UnchunkedGenerator
    from vp3d_amd.evaluate import DeviceMetrics

    args = parse_args(argv)
    seq_model = args.model_name in SEQ_MODELS
    if args.model_name != "FCN" and not seq_model:
        if args.model_name == "StackedPoselifter":
            raise SystemExit("--use-model StackedPoselifter is outside the MI355X path (SURVEY.md §2)")
        raise KeyError('Invalid model name')  # run.py:392-393
    if not torch.cuda.is_available():
        raise SystemExit("run.py evaluates on the MI355X (no CPU fallback)")
    if seq_model and not args.evaluate:
        raise SystemExit(f"--use-model {args.model_name}: training the trajectory lifters is outside the "
                         "MI355X path (SURVEY.md §8(f)); --evaluate runs them")
    if seq_model and (args.trajectory or args.compute_dtype != "fp32"):
        raise SystemExit(f"--use-model {args.model_name} takes the camera matrices itself and runs in fp32 "
                         "(no --trajectory, --compute-dtype fp32)")
    if not args.evaluate:
        return train_main(args, load_data(args, stride=1))
    if args.subset < 1:
        # the reference's evaluation reads whole sequences; --subset only reaches fetch()
        # for the training views (run.py:217, :232, :656)
        print("INFO: --subset applies to training views only; evaluating whole sequences")
    data = load_data(args)
    subjects = list(data.keys()) if args.subjects_test in (None, "*") else args.subjects_test.split(",")
    j2, j3 = joint_counts(data)
    model = build_model(args, j2, J_out=j3).cuda().eval()
    if seq_model:
        receptive_field = SEQ_RECEPTIVE_FIELD
    else:
        model.set_compute_dtype(args.compute_dtype)
        receptive_field = model.receptive_field()
    pad = (receptive_field - 1) // 2
    causal_shift = pad if args.causal else 0

    def make_generator(cams, p3d, p2d):
        return UnchunkedGenerator(cams, p3d, p2d, pad=pad, causal_shift=causal_shift,
                                  trajectory=args.trajectory)

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
