#!/usr/bin/env python3
"""Generate the golden parity vectors by running the REFERENCE itself.

Run in the build container only (the reference is not on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py [/root/reference]

It imports the reference's own modules read-only (common.models.TemporalModel,
common.generators, common.camera, common.quaternion, common.loss), feeds them
synthetic inputs and weights from vp3d_amd.synth (seeded counter hash, so the
1024-channel weights are re-created by the tests instead of being stored), and
writes small .npz fixtures next to this script.  Nothing of the reference's code
is copied: the fixtures hold inputs and the reference's outputs only.
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
PKG = os.path.join(REPO, "dynamic-camera-augmented-videopose3d_amd")
REF = os.environ.get("VP3D_REFERENCE", "/root/reference")

# `common` must resolve to the reference (a namespace package there, so our
# regular package must not be on sys.path); vp3d_amd.synth is loaded by file path.
sys.path.insert(0, REF)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from common import camera as ref_camera  # noqa: E402
from common import generators as ref_gen  # noqa: E402
from common import loss as ref_loss  # noqa: E402
from common.models import TemporalModel as ref_tm  # noqa: E402
import importlib.util  # noqa: E402

_spec = importlib.util.spec_from_file_location("vp3d_synth", os.path.join(PKG, "vp3d_amd", "synth.py"))
synth = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(synth)

assert os.path.realpath(ref_tm.__file__).startswith(os.path.realpath(REF)), ref_tm.__file__

torch.set_num_threads(8)
MANIFEST = {}


def save(name, **arrays):
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **arrays)
    h = hashlib.sha256(open(path, "rb").read()).hexdigest()
    MANIFEST[name] = {"bytes": os.path.getsize(path), "sha256": h,
                      "arrays": {k: list(np.asarray(v).shape) for k, v in arrays.items()}}
    print(f"{name}: {os.path.getsize(path) / 1024:.1f} KiB")


def build_ref_model(strided, fw, causal=False, channels=1024, jin=17, jout=17, dense=False, seed=0):
    if strided:
        m = ref_tm.TemporalModelOptimized1f(jin, 2, jout, list(fw), causal=causal, channels=channels)
    else:
        m = ref_tm.TemporalModel(jin, 2, jout, list(fw), causal=causal, channels=channels, dense=dense)
    keys = [(k, tuple(v.shape)) for k, v in m.state_dict().items()]
    sd = synth.lifter_state_dict(keys, seed=seed)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    m.eval()
    return m, sd, keys


def model_case(name, strided, fw, B, T, causal=False, channels=1024, jin=17, dense=False,
               store_weights=False, seed=0):
    m, sd, keys = build_ref_model(strided, fw, causal, channels, jin=jin, dense=dense, seed=seed)
    x = synth.normalized_windows(seed + 1, name, B, T, n_joints=jin)
    with torch.no_grad():
        y = m(torch.from_numpy(x)).numpy()
    meta = dict(strided=strided, fw=list(fw), causal=causal, channels=channels, jin=jin,
                dense=dense, seed=seed, weights_sha256=synth.state_dict_sha256(sd),
                receptive_field=m.receptive_field(), total_causal_shift=m.total_causal_shift(),
                pad=list(m.pad), causal_shift=list(m.causal_shift),
                n_params=int(sum(p.numel() for p in m.parameters())),
                keys=[k for k, _ in keys], shapes=[list(s) for _, s in keys])
    arrays = dict(x=x, y=y, meta=np.array(json.dumps(meta)))
    if store_weights:
        for k, v in sd.items():
            arrays["w/" + k] = v
    save(name, **arrays)


def model_goldens():
    F3, F5 = (3, 3, 3), (3, 3, 3, 3, 3)
    model_case("opt1f_243_fp32", True, F5, 8, 243)
    model_case("opt1f_243_causal_fp32", True, F5, 4, 243, causal=True)
    model_case("seq_243_fp32", False, F5, 1, 400)
    model_case("seq_243_causal_fp32", False, F5, 1, 300, causal=True)
    model_case("seq_27_fp32", False, F3, 2, 300)
    model_case("traj46_243_fp32", True, F5, 4, 243, jin=23)
    model_case("small_dilated_c64", False, F3, 3, 60, channels=64, store_weights=True)
    model_case("small_opt1f_c64", True, F3, 5, 27, channels=64, store_weights=True)
    model_case("small_dense_c64", False, F3, 2, 50, channels=64, dense=True, store_weights=True)
    model_case("small_causal_c64", False, (3, 5, 3), 2, 80, channels=64, causal=True,
               store_weights=True)


def cams_for(name, T):
    E = synth.camera_extrinsics(2, name, T)
    return {"intrinsics": dict(synth.CMU_INTRINSICS),
            "extrinsics": E,
            "cam_velocity": np.array([0.1, 0.0, 0.0]),
            "cam_acceleration": np.array([0.0, 0.01, 0.0]),
            "cam_angular_velocity": np.array([0.0, 0.0, 0.2]),
            "cam_angular_acceleration": np.array([0.0, 0.0, 0.0])}


def generator_goldens():
    lens = [300, 90, 40]
    pad, B = 121, 8
    kps = [ref_camera.normalize_screen_coordinates(synth.keypoint_tracks(1, f"g{i}", n), 1280, 720)
           .astype(np.float32) for i, n in enumerate(lens)]
    p3d = [synth.gt_poses(3, f"g{i}", n) for i, n in enumerate(lens)]
    cams = [cams_for(f"g{i}", n) for i, n in enumerate(lens)]
    arrays = {}
    for i in range(len(lens)):
        arrays[f"kps{i}"] = kps[i]
        arrays[f"p3d{i}"] = p3d[i]
        arrays[f"extr{i}"] = cams[i]["extrinsics"]
    for causal in (0, 1):
        shift = pad if causal else 0
        gen = ref_gen.UnchunkedGenerator(cams, p3d, kps, pad=pad, causal_shift=shift)
        for j, (bc, b3, b2, info) in enumerate(gen.next_epoch()):
            arrays[f"unchunked_c{causal}_cam{j}"] = bc.astype(np.float32)
            arrays[f"unchunked_c{causal}_2d{j}"] = b2
        cg = ref_gen.ChunkedGenerator(B, cams, p3d, kps, 1, pad=pad, causal_shift=shift,
                                      shuffle=True, random_seed=1234)
        arrays[f"chunked_c{causal}_pairs"] = np.array(cg.next_pairs()[1], dtype=np.int64)
        # Q2: the generator yields its whole (reused) buffer; record the first two
        # batches and the last (partial, with stale rows) one
        cg2 = ref_gen.ChunkedGenerator(B, cams, p3d, kps, 1, pad=pad, causal_shift=shift,
                                       shuffle=True, random_seed=1234)
        for bi, (bc, b3, b2) in enumerate(cg2.next_epoch()):
            if bi in (0, 1, cg2.num_batches - 1):
                arrays[f"chunked_c{causal}_b{bi}_cam"] = bc.copy()
                arrays[f"chunked_c{causal}_b{bi}_3d"] = b3.copy()
                arrays[f"chunked_c{causal}_b{bi}_2d"] = b2.copy()
        arrays[f"chunked_c{causal}_num_batches"] = np.array(cg2.num_batches)
    arrays["meta"] = np.array(json.dumps(dict(lens=lens, pad=pad, batch_size=B, seed=1234)))
    save("generators", **arrays)


def camera_goldens():
    a = {}
    X = synth.keypoint_tracks(1, "cam", 64, 17)
    for (w, h) in ((1280, 720), (1000, 1002), (1000, 1000)):
        n = ref_camera.normalize_screen_coordinates(X, w, h)
        a[f"norm_in_{w}x{h}"] = X
        a[f"norm_out_{w}x{h}"] = n  # float64 (reference promotion, quirk Q6)
        a[f"img_out_{w}x{h}"] = ref_camera.image_coordinates(n.astype(np.float32), w, h)
    P = synth.normal(4, "w2c", (50, 17, 3), 1.0).astype(np.float32)
    q = synth.normal(4, "w2c/q", (4,), 1.0)
    q = (q / np.linalg.norm(q)).astype(np.float32)
    t = synth.normal(4, "w2c/t", (3,), 1.0).astype(np.float32)
    a["w2c_X"], a["w2c_R"], a["w2c_t"] = P, q, t
    a["w2c_out"] = ref_camera.world_to_camera(P, R=q, t=t)
    a["c2w_out"] = ref_camera.camera_to_world(a["w2c_out"].astype(np.float32), R=q, t=t)
    save("camera", **a)


def projection_goldens():
    """H36M projections (camera.py:37-67 with distortion, :69-90 linear): camera-space
    points (positive depth, some beyond the [-1, 1] clamp of X/Z) and H36M-style
    intrinsics [f(2), c(2), k(3), p(2)] per camera."""
    a = {}
    n_cam, n_pts = 6, 2 * 17
    X = synth.normal(6, "proj/X", (n_cam, n_pts, 3), 1.0).astype(np.float32)
    X[..., 2] = np.abs(X[..., 2]) * 2 + 0.2
    X[0, :4, 2] = 0.3  # |X/Z| > 1: exercises the clamp
    prm = np.concatenate([
        1.1 + 0.1 * synth.normal(6, "proj/f", (n_cam, 2), 1.0),
        0.05 * synth.normal(6, "proj/c", (n_cam, 2), 1.0),
        0.1 * synth.normal(6, "proj/k", (n_cam, 3), 1.0),
        0.01 * synth.normal(6, "proj/p", (n_cam, 2), 1.0)], axis=1).astype(np.float32)
    a["X"], a["params"] = X, prm
    a["proj"] = ref_camera.project_to_2d(torch.from_numpy(X), torch.from_numpy(prm)).numpy()
    a["proj_linear"] = ref_camera.project_to_2d_linear(torch.from_numpy(X), torch.from_numpy(prm)).numpy()
    save("projection", **a)


def loss_goldens():
    a = {}
    pred = synth.normal(5, "pred", (2, 40, 17, 3), 0.2).astype(np.float32)
    tgt = synth.normal(5, "tgt", (2, 40, 17, 3), 0.2).astype(np.float32)
    a["pred"], a["tgt"] = pred, tgt
    a["mpjpe"] = np.array(ref_loss.mpjpe(torch.from_numpy(pred), torch.from_numpy(tgt)).item())
    a["n_mpjpe"] = np.array(ref_loss.n_mpjpe(torch.from_numpy(pred), torch.from_numpy(tgt)).item())
    p2 = pred.reshape(-1, 17, 3)
    t2 = tgt.reshape(-1, 17, 3)
    a["p_mpjpe"] = np.array(ref_loss.p_mpjpe(p2.copy(), t2.copy()))
    a["mpjve"] = np.array(ref_loss.mean_velocity_error(p2, t2))
    save("loss", **a)


def run_eval_golden():
    """The reference's FCN --evaluate loop (run.py:697-771, 906-971) on the seeded
    synthetic split, 27-frame RF, 1024 channels (BASELINE config 1 shape)."""
    data = synth.synthetic_split(3, 3, 200, 17, 0, ref_camera.normalize_screen_coordinates)
    fw = [3, 3, 3]
    m, sd, keys = build_ref_model(False, fw, channels=1024, seed=0)
    pad = (m.receptive_field() - 1) // 2
    actions = {}
    for s in data:
        for a in data[s]:
            actions.setdefault(a.split(" ")[0], []).append((s, a))
    out = {}
    e1_seq, infos, motion = [], [], []
    for key, seqs in actions.items():
        cams = [data[s][a]["cameras"] for s, a in seqs]
        p3d = [data[s][a]["positions_3d"] for s, a in seqs]
        p2d = [data[s][a]["keypoints"] for s, a in seqs]
        gen = ref_gen.UnchunkedGenerator(cams, p3d, p2d, pad=pad, causal_shift=0)
        e1 = e2 = e3 = ev = 0.0
        N = 0
        with torch.no_grad():
            for bc, b3, b2, info in gen.next_epoch():
                x2 = torch.from_numpy(b2.astype("float32"))
                x3 = torch.from_numpy(b3.astype("float32"))
                pred = m(x2)
                err = ref_loss.mpjpe(pred, x3)
                n = x3.shape[0] * x3.shape[1]
                e3 += n * ref_loss.n_mpjpe(pred, x3).item()
                e1 += n * err.item()
                e1_seq.append(err.numpy())
                infos.append(info)
                pm = np.linalg.norm(np.diff(b3, axis=1), axis=-1)
                motion.append(np.mean(pm.squeeze(), axis=(0, 1)))
                N += n
                inp = x3.numpy().reshape(-1, 17, 3)
                pr = pred.numpy().reshape(-1, 17, 3)
                e2 += n * ref_loss.p_mpjpe(pr, inp)
                ev += n * ref_loss.mean_velocity_error(pr, inp)
        # run.py:762-765 evaluates (loss / N) * 1000 on the accumulators' own scalar types
        out[key] = np.array([(e1 / N) * 1000, (e2 / N) * 1000, (e3 / N) * 1000, (ev / N) * 1000])
    corr = np.corrcoef(np.stack([np.array(e1_seq)] + [
        np.linalg.norm(np.array([i[k] for i in infos]), axis=1)
        for k in ("cam_velocity", "cam_acceleration", "cam_angular_velocity", "cam_angular_acceleration")]
        + [np.array(motion)], axis=1))
    save("run_eval_27", actions=np.array(list(out.keys())), errors=np.stack(list(out.values())),
         pmcc=corr[0, 1:6], meta=np.array(json.dumps(dict(fw=fw, channels=1024, seed=0,
                                                           subjects=3, actions=3, frames=200))))


def train_case(name, strided, fw, B, T, causal=False, channels=64, dense=False, seed=0, steps=2):
    """Two reference training iterations (run.py:451-487 with TemporalModel in train mode,
    dropout 0): forward with BatchNorm batch statistics, mpjpe, backward,
    optim.Adam(amsgrad=True).step() (run.py:662).  Stores inputs, weights and per step
    the output, loss, every gradient, the running statistics and the updated weights."""
    m, sd, keys = build_ref_model(strided, fw, causal, channels, dense=dense, seed=seed)
    if strided:
        m = ref_tm.TemporalModelOptimized1f(17, 2, 17, list(fw), causal=causal, channels=channels,
                                            dropout=0.0)
    else:
        m = ref_tm.TemporalModel(17, 2, 17, list(fw), causal=causal, channels=channels, dense=dense,
                                 dropout=0.0)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    m.train()
    m.set_bn_momentum(0.1)
    opt = torch.optim.Adam(m.parameters(), lr=1e-3, amsgrad=True)
    arrays = {}
    for k, v in sd.items():
        arrays["w/" + k] = v
    T_out = None
    for it in range(steps):
        x = synth.normalized_windows(seed + 10 + it, name, B, T)
        y = m(torch.from_numpy(x))
        T_out = y.shape[1]
        tgt = synth.normal(seed + 20 + it, name + "/target", (B, T_out, 17, 3), std=0.2).astype(np.float32)
        loss = ref_loss.mpjpe(y, torch.from_numpy(tgt))
        opt.zero_grad()
        loss.backward()
        arrays[f"s{it}/x"] = x
        arrays[f"s{it}/target"] = tgt
        arrays[f"s{it}/y"] = y.detach().numpy()
        arrays[f"s{it}/loss"] = np.array(loss.item(), dtype=np.float32)
        for k, p in m.named_parameters():
            arrays[f"s{it}/grad/{k}"] = p.grad.numpy().copy()
        opt.step()
        for k, v in m.state_dict().items():
            arrays[f"s{it}/after/{k}"] = v.numpy().copy()
    meta = dict(strided=strided, fw=list(fw), causal=causal, channels=channels, dense=dense, seed=seed,
                B=B, T=T, T_out=int(T_out), steps=steps, lr=1e-3, amsgrad=True, momentum=0.1,
                keys=[k for k, _ in keys])
    arrays["meta"] = np.array(json.dumps(meta))
    save(name, **arrays)


def train_goldens():
    F3 = (3, 3, 3)
    train_case("train_dilated_c64", False, F3, 6, 31)           # chunk of 5 output frames
    train_case("train_opt1f_c64", True, F3, 8, 27)
    train_case("train_causal_c64", False, (3, 5, 3), 3, 80, causal=True)
    train_case("train_dense_c32", False, F3, 2, 40, channels=32, dense=True)


def _ref_seq_model(name, kind, seed):
    """The reference's CoupledTransformer / CoupledLSTM at the run.py defaults
    (arguments.py:41-54, run.py:311-363), torch's default init under manual_seed, the
    LSTM head's BN statistics randomised (eval mode)."""
    from common.models import CamLSTM as ref_lstm
    from common.models import CamTransformer as ref_tfm
    torch.manual_seed(seed)
    if kind == "transformer":
        m = ref_tfm.CoupledTransformer(17, 2, 17, 3, d_model=128, num_layers=2, n_heads=4, dim_feedforward=128,
                                       head_layers=[128, 128, 128], dropout=0.25)
    else:
        m = ref_lstm.CoupledLSTM(17, 2, 17, 3, hidden_size=128, num_cells=2, head_layers=[128, 128, 128],
                                 dropout=0.25)
        for i, bn in enumerate(m.bn_layers):
            n = bn.num_features
            bn.running_mean.copy_(torch.from_numpy(synth.uniform(seed + i, name + "/mu", (n,), -0.2, 0.2).astype(np.float32)))
            bn.running_var.copy_(torch.from_numpy(synth.uniform(seed + i, name + "/var", (n,), 0.5, 2.0).astype(np.float32)))
            bn.weight.data.copy_(torch.from_numpy(synth.uniform(seed + i, name + "/g", (n,), 0.5, 1.5).astype(np.float32)))
            bn.bias.data.copy_(torch.from_numpy(synth.uniform(seed + i, name + "/b", (n,), -0.1, 0.1).astype(np.float32)))
    return m.eval()


def seq_lifter_case(name, kind, B=6, L=260, seed=0):
    """Eval-mode CoupledTransformer / CoupledLSTM (CamTransformer.py:95-205,
    CamLSTM.py:47-129) at the run.py defaults (arguments.py:41-54): forward on B
    windows of 243 frames and sliding_window over one padded sequence of L frames
    (run.py:713).  Weights: torch's default init under manual_seed, BN statistics
    randomised; stored in the fixture."""
    m = _ref_seq_model(name, kind, seed)
    x2 = synth.normalized_windows(seed + 1, name, B, 243)
    xc = (synth.normal(seed + 2, name + "/cam", (B, 243, 3, 4), std=0.5)).astype(np.float32)
    s2 = synth.normalized_windows(seed + 3, name + "/seq", 1, L)
    sc = (synth.normal(seed + 4, name + "/seqcam", (1, L, 3, 4), std=0.5)).astype(np.float32)
    with torch.no_grad():
        y = m(torch.from_numpy(x2), torch.from_numpy(xc)).numpy()
        ys = m.sliding_window(torch.from_numpy(s2), torch.from_numpy(sc), 243).numpy()
    arrays = {"x2d": x2, "xcam": xc, "y": y, "seq2d": s2, "seqcam": sc, "yseq": ys}
    for k, v in m.state_dict().items():
        if not k.endswith(".pe"):  # the sinusoid table (5000 x d) is recomputed, not stored
            arrays["w/" + k] = v.numpy()
    meta = dict(kind=kind, B=B, L=L, window=243, seed=seed, keys=list(m.state_dict().keys()),
                d_model=128, num_layers=2, n_heads=4, dim_feedforward=128, hidden_size=128, num_cells=2,
                head_layers=[128, 128, 128])
    arrays["meta"] = np.array(json.dumps(meta))
    save(name, **arrays)


def seq_lifter_goldens():
    seq_lifter_case("cam_transformer", "transformer")
    seq_lifter_case("cam_lstm", "lstm")


def run_eval_seq_golden(kind, seed=0):
    """The reference's --evaluate loop with --use-model Transformer | LSTM-Coupled
    (run.py:311-363 construction, :697-771 evaluate with the sliding_window dispatch of
    :712-713 on the reference UnchunkedGenerator's camera matrices, :906-971
    run_evaluation) on the seeded synthetic split of run_eval_27 (3 subjects x 3
    actions, 200+ frames).  Weights stored in the fixture."""
    name = "run_eval_" + kind
    data = synth.synthetic_split(3, 3, 200, 17, 0, ref_camera.normalize_screen_coordinates)
    m = _ref_seq_model(name, kind, seed)
    pad = (243 - 1) // 2  # run.py:313-314 / :335-336
    actions = {}
    for s in data:
        for a in data[s]:
            actions.setdefault(a.split(" ")[0], []).append((s, a))
    out = {}
    e1_seq, infos, motion = [], [], []
    for key, seqs in actions.items():
        cams = [data[s][a]["cameras"] for s, a in seqs]
        p3d = [data[s][a]["positions_3d"] for s, a in seqs]
        p2d = [data[s][a]["keypoints"] for s, a in seqs]
        gen = ref_gen.UnchunkedGenerator(cams, p3d, p2d, pad=pad, causal_shift=0)
        e1 = e2 = e3 = ev = 0.0
        N = 0
        with torch.no_grad():
            for bc, b3, b2, info in gen.next_epoch():
                x2 = torch.from_numpy(b2.astype("float32"))
                x3 = torch.from_numpy(b3.astype("float32"))
                xc = torch.from_numpy(bc.astype("float32"))
                pred = m.sliding_window(x2, xc, gen.seq_length)
                err = ref_loss.mpjpe(pred, x3)
                n = x3.shape[0] * x3.shape[1]
                e3 += n * ref_loss.n_mpjpe(pred, x3).item()
                e1 += n * err.item()
                e1_seq.append(err.numpy())
                infos.append(info)
                pm = np.linalg.norm(np.diff(b3, axis=1), axis=-1)
                motion.append(np.mean(pm.squeeze(), axis=(0, 1)))
                N += n
                inp = x3.numpy().reshape(-1, 17, 3)
                pr = pred.numpy().reshape(-1, 17, 3)
                e2 += n * ref_loss.p_mpjpe(pr, inp)
                ev += n * ref_loss.mean_velocity_error(pr, inp)
        out[key] = np.array([(e1 / N) * 1000, (e2 / N) * 1000, (e3 / N) * 1000, (ev / N) * 1000])
    corr = np.corrcoef(np.stack([np.array(e1_seq)] + [
        np.linalg.norm(np.array([i[k] for i in infos]), axis=1)
        for k in ("cam_velocity", "cam_acceleration", "cam_angular_velocity", "cam_angular_acceleration")]
        + [np.array(motion)], axis=1))
    arrays = {"actions": np.array(list(out.keys())), "errors": np.stack(list(out.values())), "pmcc": corr[0, 1:6]}
    for k, v in m.state_dict().items():
        if not k.endswith(".pe"):
            arrays["w/" + k] = v.numpy()
    arrays["meta"] = np.array(json.dumps(dict(kind=kind, seed=seed, subjects=3, actions=3, frames=200,
                                              model={"transformer": "Transformer", "lstm": "LSTM-Coupled"}[kind])))
    save(name, **arrays)


def run_eval_seq_goldens():
    run_eval_seq_golden("transformer")
    run_eval_seq_golden("lstm")


DATASET_DIR = os.path.join(HERE, "datasets")
H36M_SUBJECTS = ("S1", "S5")
H36M_ACTIONS = ("Walking", "Walking 1", "Eating")
CMU_SUBJECTS = ("01", "02")
CMU_ACTIONS = ("walk_0", "jump_1")


def write_dataset_fixtures():
    """Small datasets in the reference's .npz layout (pickled dicts of arrays, as
    prepare_data_h36m.py / prepare_data_cmu_camera.py write them): H36M world-space
    32-joint mocap + per-camera 17-joint 2D tracks (some longer than the mocap, as in
    the real data), and the fork's CMU camera-space poses + per-frame extrinsics."""
    os.makedirs(DATASET_DIR, exist_ok=True)
    # ---- Human3.6M ----
    pos3, pos2 = {}, {}
    for si, subj in enumerate(H36M_SUBJECTS):
        pos3[subj], pos2[subj] = {}, {}
        for ai, act in enumerate(H36M_ACTIONS):
            T = 90 + 23 * ai + 11 * si
            key = f"h36m/{subj}/{act}"
            root = np.cumsum(synth.normal(11, key + "/root", (T, 1, 3), 0.01), axis=0) + np.array([0.0, 0.0, 0.9])
            body = synth.normal(11, key + "/body", (1, 32, 3), 0.25)
            jit = synth.normal(11, key + "/jit", (T, 32, 3), 0.005)
            pos3[subj][act] = (root + body + jit).astype(np.float32)
            pos2[subj][act] = [synth.keypoint_tracks(12, f"{key}/{c}", T + (3 if c == 1 else 0), 17, 1000, 1002)
                               for c in range(4)]
    meta = {"layout_name": "h36m", "num_joints": 17,
            "keypoints_symmetry": [[4, 5, 6, 11, 12, 13], [1, 2, 3, 14, 15, 16]]}
    np.savez_compressed(os.path.join(DATASET_DIR, "data_3d_h36m.npz"), positions_3d=pos3)
    np.savez_compressed(os.path.join(DATASET_DIR, "data_2d_h36m_gt.npz"), positions_2d=pos2, metadata=meta)
    # ---- CMU with procedural cameras ----
    pos3, seqs, pos2 = {}, {}, {}
    for si, subj in enumerate(CMU_SUBJECTS):
        pos3[subj], seqs[subj], pos2[subj] = {}, {}, {}
        for ai, act in enumerate(CMU_ACTIONS):
            T = 100 + 31 * ai + 7 * si
            key = f"cmu/{subj}/{act}"
            p = synth.gt_poses(13, key, T, 17) + np.array([0.0, 0.0, 4.0], dtype=np.float32)
            p = p + synth.normal(13, key + "/root", (T, 1, 3), 0.2).astype(np.float32)
            pos3[subj][act] = p.astype(np.float32)
            mot = synth.uniform(14, key, (4, 3), -1.0, 1.0)
            seqs[subj][act] = {"cam_extrinsic": synth.camera_extrinsics(15, key, T), "cam_velocity": mot[0],
                               "cam_acceleration": mot[1], "cam_angular_velocity": mot[2],
                               "cam_angular_acceleration": mot[3],
                               "pose_2d_flow": synth.normal(16, key, (T, 17, 2), 1.0).astype(np.float32)}
            pos2[subj][act] = synth.keypoint_tracks(17, key, T, 17)
    np.savez_compressed(os.path.join(DATASET_DIR, "data_3d_CMU.npz"), positions_3d=pos3, cam_seqs=seqs)
    np.savez_compressed(os.path.join(DATASET_DIR, "data_2d_CMU_gt.npz"), positions_2d=pos2, metadata=meta)


def _ref_eval(actions, fw, channels, seed, use_generator, jin=17, jout=17):
    """The reference's evaluate() numbers per action key (run.py:697-771)."""
    m, sd, keys = build_ref_model(False, fw, channels=channels, seed=seed, jin=jin, jout=jout)
    pad = (m.receptive_field() - 1) // 2
    out, e1_seq, infos, motion = {}, [], [], []
    for key, (cams, p3d, p2d) in actions.items():
        if use_generator:
            batches = ref_gen.UnchunkedGenerator(cams, p3d, p2d, pad=pad, causal_shift=0).next_epoch()
        else:
            # the H36M camera records crash the reference generator (quirk Q1): the same
            # batches, edge padding as generators.py:193-198
            batches = ((None, p[None], np.pad(k, ((pad, pad), (0, 0), (0, 0)), "edge")[None],
                        {"cam_velocity": np.zeros(3), "cam_acceleration": np.zeros(3),
                         "cam_angular_velocity": np.zeros(3), "cam_angular_acceleration": np.zeros(3)})
                       for p, k in zip(p3d, p2d))
        e1 = e2 = e3 = ev = 0.0
        N = 0
        with torch.no_grad():
            for bc, b3, b2, info in batches:
                x2 = torch.from_numpy(b2.astype("float32"))
                x3 = torch.from_numpy(b3.astype("float32"))
                pred = m(x2)
                err = ref_loss.mpjpe(pred, x3)
                n = x3.shape[0] * x3.shape[1]
                e3 += n * ref_loss.n_mpjpe(pred, x3).item()
                e1 += n * err.item()
                e1_seq.append(err.numpy())
                infos.append(info)
                motion.append(np.mean(np.linalg.norm(np.diff(b3, axis=1), axis=-1).squeeze(), axis=(0, 1)))
                N += n
                inp = x3.numpy().reshape(-1, x3.shape[-2], 3)
                pr = pred.numpy().reshape(-1, x3.shape[-2], 3)
                e2 += n * ref_loss.p_mpjpe(pr, inp)
                ev += n * ref_loss.mean_velocity_error(pr, inp)
        out[key] = np.array([(e1 / N) * 1000, (e2 / N) * 1000, (e3 / N) * 1000, (ev / N) * 1000])
    return out


def dataset_goldens():
    """The reference's data preparation (run.py:47-124) on the fixture datasets, then its
    evaluation loop: CMUMocapDataset + the reference generator as-is; H36M through the
    importable pieces (Human36mDataset without the crashing joint removal, quirk Q1; the
    reference Skeleton's remove_joints; world_to_camera; normalize_screen_coordinates)."""
    import copy
    from common.datasets import h36m_dataset as ref_h36m
    from common.datasets.CMUMocapDataset import CMUMocapDataset
    write_dataset_fixtures()
    fw, channels, seed = [3, 3, 3], 256, 0
    arrays = {}
    # ---- CMU ----
    ds = CMUMocapDataset(os.path.join(DATASET_DIR, "data_3d_CMU.npz"))
    kp = np.load(os.path.join(DATASET_DIR, "data_2d_CMU_gt.npz"), allow_pickle=True)["positions_2d"].item()
    for subj in ds.subjects():
        for act in ds[subj].keys():
            anim = ds[subj][act]
            pos = anim["positions"]
            pos -= pos[:, :1]
            anim["positions_3d"] = [pos]
    for subj in kp:
        for act in kp[subj]:
            k = kp[subj][act]
            intr = ds.cameras()[subj][act]["intrinsics"]
            k[..., :2] = ref_camera.normalize_screen_coordinates(k[..., :2], w=intr["res_w"], h=intr["res_h"])
            kp[subj][act] = [k]
    actions = {}
    for subj in ds.subjects():
        for act in ds[subj].keys():
            c, p3, p2 = actions.setdefault(act.split(" ")[0], ([], [], []))
            c.append(ds.cameras()[subj][act])
            p3 += ds[subj][act]["positions_3d"]
            p2 += kp[subj][act]
            arrays[f"cmu/{subj}/{act}/p3d"] = ds[subj][act]["positions_3d"][0]
            arrays[f"cmu/{subj}/{act}/kps"] = kp[subj][act][0]
    res = _ref_eval(actions, fw, channels, seed, use_generator=True)
    arrays["cmu_actions"] = np.array(list(res.keys()))
    arrays["cmu_errors"] = np.stack(list(res.values()))
    # ---- Human3.6M ----
    ds = ref_h36m.Human36mDataset(os.path.join(DATASET_DIR, "data_3d_h36m.npz"), remove_static_joints=False)
    sk = copy.deepcopy(ref_h36m.h36m_skeleton)
    kept = sk.remove_joints([4, 5, 9, 10, 11, 16, 20, 21, 22, 23, 24, 28, 29, 30, 31])
    kp = np.load(os.path.join(DATASET_DIR, "data_2d_h36m_gt.npz"), allow_pickle=True)["positions_2d"].item()
    actions = {}
    for subj in H36M_SUBJECTS:
        for act in H36M_ACTIONS:
            anim = ds[subj][act]
            views3, views2 = [], []
            for ci, cam in enumerate(anim["cameras"]):
                p = ref_camera.world_to_camera(anim["positions"][:, kept], R=cam["orientation"], t=cam["translation"])
                p[:, 1:] -= p[:, :1]
                k = kp[subj][act][ci][:p.shape[0]].copy()
                k[..., :2] = ref_camera.normalize_screen_coordinates(k[..., :2], w=cam["res_w"], h=cam["res_h"])
                views3.append(p)
                views2.append(k)
                arrays[f"h36m/{subj}/{act}/{ci}/p3d"] = p
                arrays[f"h36m/{subj}/{act}/{ci}/kps"] = k
            c, p3, p2 = actions.setdefault(act.split(" ")[0], ([], [], []))
            c += [None] * len(views3)
            p3 += views3
            p2 += views2
    res = _ref_eval(actions, fw, channels, seed, use_generator=False)
    arrays["h36m_actions"] = np.array(list(res.keys()))
    arrays["h36m_errors"] = np.stack(list(res.values()))
    for subj in H36M_SUBJECTS:
        for ci, cam in enumerate(ds.cameras()[subj]):
            for k in ("center", "focal_length", "translation", "orientation", "intrinsic"):
                arrays[f"h36m_cam/{subj}/{ci}/{k}"] = np.asarray(cam[k])
    arrays["h36m_skeleton_parents"] = np.asarray(sk.parents())
    arrays["h36m_kept_joints"] = np.asarray(kept)
    arrays["meta"] = np.array(json.dumps(dict(fw=fw, channels=channels, seed=seed,
                                              h36m_subjects=list(H36M_SUBJECTS), cmu_subjects=list(CMU_SUBJECTS))))
    save("run_eval_datasets", **arrays)


TDPW_SEQS = (("train", "courtyard_walk_00_0", 31, (1961.8529, 1969.2307, 540.0, 960.0)),
             ("train", "downtown_car_01_1", 37, (1972.5, 1968.25, 541.25, 959.5)),
             ("validation", "outdoors_turn_00_0", 29, (1961.8529, 1969.2307, 540.0, 960.0)))


def _upsample_linear(x, factor=4):
    """prepare_data_3dpw.py:29-37 (linear interpolation over time, float64 out)."""
    from scipy.interpolate import interp1d
    T = x.shape[0]
    return interp1d(np.arange(T), x, axis=0, kind="linear")(np.linspace(0, T - 1, factor * T))


def write_3dpw_fixture():
    """A small dataset in the layout prepare_data_3dpw.py:58-103 writes: keyframe camera
    poses (a yaw / pitch sweep and a walk) and SMPL joints upsampled 4x (so consecutive
    extrinsics are NOT exactly orthogonal, as in the real data), camera-space joints,
    float32 intrinsics (one with a non-integral principal point), float64 COCO 2D tracks."""
    pos3, seqs, intr, pos2 = {}, {}, {}, {}
    for subj, act, T0, (fx, fy, cx, cy) in TDPW_SEQS:
        key = f"3dpw/{subj}/{act}"
        for d in (pos3, seqs, intr, pos2):
            d.setdefault(subj, {})
        ang = np.cumsum(synth.uniform(21, key + "/ang", (T0, 3), -0.04, 0.04), axis=0)
        E = np.zeros((T0, 3, 4), np.float32)
        for t in range(T0):
            a, b, c = ang[t]
            Rz = np.array([[np.cos(a), -np.sin(a), 0], [np.sin(a), np.cos(a), 0], [0, 0, 1]])
            Ry = np.array([[np.cos(b), 0, np.sin(b)], [0, 1, 0], [-np.sin(b), 0, np.cos(b)]])
            Rx = np.array([[1, 0, 0], [0, np.cos(c), -np.sin(c)], [0, np.sin(c), np.cos(c)]])
            E[t, :, :3] = Rz @ Ry @ Rx
        E[:, :, 3] = (np.cumsum(synth.normal(21, key + "/walk", (T0, 3), 0.02), axis=0)
                      + np.array([0.0, 0.3, 3.5])).astype(np.float32)
        cam_seq = _upsample_linear(E)
        world = synth.gt_poses(22, key, T0, 24).astype(np.float32) * 2 + np.array([0.0, 0.0, 0.5], np.float32)
        world = _upsample_linear(world.reshape(-1, 24, 3))
        hom = np.concatenate([world, np.ones(world.shape[:2] + (1,), np.float32)], axis=2)
        pos3[subj][act] = np.einsum("tij,tnj->tni", cam_seq, hom)
        seqs[subj][act] = cam_seq
        intr[subj][act] = np.array([[fx, 0, cx], [0, fy, cy], [0, 0, 1]], np.float32)
        trk = synth.keypoint_tracks(23, key, T0, 18, int(2 * cx), int(2 * cy))
        pos2[subj][act] = _upsample_linear(np.asarray(trk, np.float32))
    meta = {"layout_name": "coco", "num_joints": 18,
            "keypoints_symmetry": [[2, 3, 4, 8, 9, 10, 14, 16], [5, 6, 7, 11, 12, 13, 15, 17]]}
    np.savez_compressed(os.path.join(DATASET_DIR, "data_3d_3DPW.npz"), positions_3d=pos3, cam_seqs=seqs,
                        cam_intrinsics=intr)
    np.savez_compressed(os.path.join(DATASET_DIR, "data_2d_3DPW_gt.npz"), positions_2d=pos2, metadata=meta)


def dataset_3dpw_goldens():
    """The reference's ThreeDPWDataset (ThreeDPWDataset.py:24-117, scipy logm) and run.py's
    preparation (:65-124) on the 3DPW fixture, then its evaluation loop (generator as-is)."""
    from common.datasets.ThreeDPWDataset import ThreeDPWDataset
    os.makedirs(DATASET_DIR, exist_ok=True)
    write_3dpw_fixture()
    fw, channels, seed = [3, 3, 3], 256, 0
    arrays = {}
    ds = ThreeDPWDataset(os.path.join(DATASET_DIR, "data_3d_3DPW.npz"))
    kp = np.load(os.path.join(DATASET_DIR, "data_2d_3DPW_gt.npz"), allow_pickle=True)["positions_2d"].item()
    for subj in ds.subjects():
        for act in ds[subj].keys():
            anim = ds[subj][act]
            pos = anim["positions"]
            pos -= pos[:, :1]
            anim["positions_3d"] = [pos]
            cam = ds.cameras()[subj][act]
            for k in ("cam_velocity", "cam_acceleration", "cam_angular_velocity", "cam_angular_acceleration"):
                arrays[f"3dpw/{subj}/{act}/{k}"] = np.asarray(cam[k])
            for k in ("center", "focal_length"):
                arrays[f"3dpw/{subj}/{act}/{k}"] = np.asarray(cam["intrinsics"][k])
            arrays[f"3dpw/{subj}/{act}/res"] = np.array([cam["intrinsics"]["res_w"], cam["intrinsics"]["res_h"]])
    for subj in kp:
        for act in kp[subj]:
            k = kp[subj][act]
            intr = ds.cameras()[subj][act]["intrinsics"]
            k[..., :2] = ref_camera.normalize_screen_coordinates(k[..., :2], w=intr["res_w"], h=intr["res_h"])
            kp[subj][act] = [k]
    actions = {}
    for subj in ds.subjects():
        for act in ds[subj].keys():
            c, p3, p2 = actions.setdefault(act.split(" ")[0], ([], [], []))
            c.append(ds.cameras()[subj][act])
            p3 += ds[subj][act]["positions_3d"]
            p2 += kp[subj][act]
            arrays[f"3dpw/{subj}/{act}/p3d"] = ds[subj][act]["positions_3d"][0]
            arrays[f"3dpw/{subj}/{act}/kps"] = kp[subj][act][0]
    res = _ref_eval(actions, fw, channels, seed, use_generator=True, jin=18, jout=24)
    arrays["3dpw_actions"] = np.array(list(res.keys()))
    arrays["3dpw_errors"] = np.stack(list(res.values()))
    arrays["meta"] = np.array(json.dumps(dict(fw=fw, channels=channels, seed=seed,
                                              seqs=[[s_, a_] for s_, a_, _, _ in TDPW_SEQS])))
    save("run_eval_3dpw", **arrays)


HE_SEQS = (("Train/S1", "Walk 1 chunk0", 83), ("Train/S2", "Jog 1 chunk0", 71), ("Validate/S3", "Box 1 chunk1", 77))


def write_humaneva_fixture():
    """A small dataset in the upstream HumanEva layout (prepare_data_humaneva.py): world
    15-joint mocap per (split/subject, action), three camera tracks of 2D keypoints
    (640 x 480 pixels, one longer than the mocap)."""
    pos3, pos2 = {}, {}
    for subj, act, T in HE_SEQS:
        key = f"he/{subj}/{act}"
        root = np.cumsum(synth.normal(31, key + "/root", (T, 1, 3), 0.01), axis=0) + np.array([0.5, -0.2, 0.9])
        body = synth.normal(31, key + "/body", (1, 15, 3), 0.25)
        jit = synth.normal(31, key + "/jit", (T, 15, 3), 0.005)
        pos3.setdefault(subj, {})[act] = (root + body + jit).astype(np.float32)
        pos2.setdefault(subj, {})[act] = [synth.keypoint_tracks(32, f"{key}/{c}", T + (2 if c == 2 else 0), 15, 640, 480)
                                          for c in range(3)]
    meta = {"layout_name": "humaneva15", "num_joints": 15,
            "keypoints_symmetry": [[2, 3, 4, 8, 9, 10], [5, 6, 7, 11, 12, 13]]}
    np.savez_compressed(os.path.join(DATASET_DIR, "data_3d_humaneva.npz"), positions_3d=pos3)
    np.savez_compressed(os.path.join(DATASET_DIR, "data_2d_humaneva_gt.npz"), positions_2d=pos2, metadata=meta)


def dataset_humaneva_goldens():
    """The reference's HumanEvaDataset (humaneva_dataset.py:90-120) and run.py's
    preparation of a calibrated multi-view dataset (:65-124: world_to_camera per camera,
    root-relative joints, 2D cut to the mocap length and normalised per camera), then its
    evaluation loop on edge-padded whole sequences (the reference's fetch_actions indexes
    the per-subject camera list by action name and crashes, quirk Q1, as for H36M)."""
    from common.datasets.humaneva_dataset import HumanEvaDataset
    os.makedirs(DATASET_DIR, exist_ok=True)
    write_humaneva_fixture()
    fw, channels, seed = [3, 3, 3], 256, 0
    arrays = {}
    ds = HumanEvaDataset(os.path.join(DATASET_DIR, "data_3d_humaneva.npz"))
    kp = np.load(os.path.join(DATASET_DIR, "data_2d_humaneva_gt.npz"), allow_pickle=True)["positions_2d"].item()
    actions = {}
    for subj, act, _ in HE_SEQS:
        anim = ds[subj][act]
        views3, views2 = [], []
        for ci, cam in enumerate(anim["cameras"]):
            p = ref_camera.world_to_camera(anim["positions"], R=cam["orientation"], t=cam["translation"])
            p[:, 1:] -= p[:, :1]
            k = kp[subj][act][ci][:p.shape[0]].copy()
            k[..., :2] = ref_camera.normalize_screen_coordinates(k[..., :2], w=cam["res_w"], h=cam["res_h"])
            views3.append(p)
            views2.append(k)
            arrays[f"he/{subj}/{act}/{ci}/p3d"] = p
            arrays[f"he/{subj}/{act}/{ci}/kps"] = k
        c, p3, p2 = actions.setdefault(act.split(" ")[0], ([], [], []))
        c += [None] * len(views3)
        p3 += views3
        p2 += views2
    res = _ref_eval(actions, fw, channels, seed, use_generator=False, jin=15, jout=15)
    arrays["he_actions"] = np.array(list(res.keys()))
    arrays["he_errors"] = np.stack(list(res.values()))
    arrays["meta"] = np.array(json.dumps(dict(fw=fw, channels=channels, seed=seed,
                                              seqs=[[s_, a_] for s_, a_, _ in HE_SEQS])))
    save("run_eval_humaneva", **arrays)


GROUPS = {"run_eval": run_eval_golden, "dataset": dataset_goldens, "dataset_3dpw": dataset_3dpw_goldens,
          "dataset_humaneva": dataset_humaneva_goldens, "model": model_goldens, "generator": generator_goldens,
          "camera": camera_goldens, "projection": projection_goldens, "loss": loss_goldens,
          "train": train_goldens, "seq_lifter": seq_lifter_goldens, "run_eval_seq": run_eval_seq_goldens}

if __name__ == "__main__":
    # python make_golden.py [group ...]  (default: every group); the manifest is merged
    todo = sys.argv[1:] or list(GROUPS)
    for g in todo:
        GROUPS[g]()
    env = dict(torch=torch.__version__, numpy=np.__version__, python=sys.version.split()[0],
               reference=REF)
    mpath = os.path.join(HERE, "MANIFEST.json")
    fixtures = {}
    if os.path.exists(mpath) and sys.argv[1:]:
        with open(mpath) as f:
            fixtures = json.load(f).get("fixtures", {})
    fixtures.update(MANIFEST)
    MANIFEST = fixtures
    with open(mpath, "w") as f:
        json.dump({"environment": env, "fixtures": MANIFEST}, f, indent=1, sort_keys=True)
    print("total KiB", sum(v["bytes"] for v in MANIFEST.values()) / 1024)
