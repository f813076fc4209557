"""run.py flags and checkpoint loading (CPU)."""
import os

import numpy as np
import pytest
import torch

from common.arguments import parse_args


def test_reference_training_command_parses():
    # a reference-style training command with the long spellings (reference arguments.py:24-38)
    a = parse_args(["--dataset", "CMU", "--keypoints", "gt", "--resume", "epoch_10.bin", "--epochs", "80",
                    "--learning-rate", "0.0005", "--lr-decay", "0.9", "--batch-size", "512",
                    "--fcn-architecture", "3,3,3", "--channels", "256", "--stride", "2",
                    "--checkpoint-frequency", "5", "--use-model", "FCN", "--hidden-features", "64",
                    "--n_heads", "8", "--viz-subject", "S1", "--subset", "0.5"])
    assert (a.dataset, a.resume, a.epochs, a.learning_rate, a.lr_decay) == ("CMU", "epoch_10.bin", 80, 5e-4, 0.9)
    assert (a.batch_size, a.fcn_architecture, a.channels, a.stride) == (512, "3,3,3", 256, 2)
    assert a.lstm_hidden_features == 64 and a.n_heads == 8 and a.subset == 0.5
    b = parse_args(["-d", "h36m", "-r", "x.bin", "-e", "3", "-lr", "0.01", "-lrd", "0.5", "-b", "64", "-s", "1",
                    "-ch", "128", "-str", "S1,S5", "-te", "4"])
    assert (b.dataset, b.resume, b.epochs, b.learning_rate, b.lr_decay, b.channels) == ("h36m", "x.bin", 3, 0.01,
                                                                                          0.5, 128)
    assert b.subjects_train == "S1,S5" and b.tuning_epochs == 4


def test_reference_defaults():
    a = parse_args([])
    assert (a.epochs, a.batch_size, a.learning_rate, a.lr_decay, a.stride) == (60, 1024, 0.001, 0.95, 1)
    assert (a.fcn_architecture, a.channels, a.fcn_dropout, a.checkpoint_frequency) == ("3,3,3,3,3", 1024, 0.25, 10)


def test_invalid_combinations():
    with pytest.raises(SystemExit):
        parse_args(["--resume", "a.bin", "--evaluate", "b.bin"])
    with pytest.raises(SystemExit):
        parse_args(["--export-training-curves", "--no-eval"])
    with pytest.raises(SystemExit):
        parse_args(["-d", "nonsense"])


def test_checkpoint_loader_admits_run_checkpoint_only(tmp_path):
    from vp3d_amd.checkpoint import load_checkpoint
    rs = np.random.RandomState(1234)
    rs.permutation(100)
    path = os.path.join(tmp_path, "epoch_1.bin")
    sd = {"w": torch.arange(6.0)}
    torch.save({"epoch": 1, "lr": 0.001, "random_state": rs, "optimizer": {"state": {}, "param_groups": []},
                "model_pos": sd}, path)
    ck = load_checkpoint(path)
    assert ck["epoch"] == 1 and torch.equal(ck["model_pos"]["w"], sd["w"])
    assert ck["random_state"].randint(0, 1 << 30) == rs.randint(0, 1 << 30)

    class Evil:
        def __reduce__(self):
            return (os.system, ("echo pwned",))
    bad = os.path.join(tmp_path, "evil.bin")
    torch.save({"model_pos": sd, "x": Evil()}, bad)
    with pytest.raises(RuntimeError, match="trust-checkpoint"):
        load_checkpoint(bad)


def test_subset_views_matches_reference_fetch():
    """--subset / --downsample on the training views (reference run.py:168-180): the trimmed
    lengths and start frames.  The starts are the reference's own deterministic_random
    (common/utils.py:44-47) values, pinned by importing it in the build container."""
    import run
    want_start = {1000: 411, 2048: 1008, 517: 345, 300: 22}  # deterministic_random(0, L - n + 1, str(L))
    for L, n in ((1000, 100), (2048, 204), (517, 50), (300, 30)):
        assert run.deterministic_random(0, L - n + 1, str(L)) == want_start[L]
    lens = [1000, 2048, 517]
    p2d = [np.arange(L * 2, dtype=np.float32).reshape(L, 1, 2) for L in lens]
    p3d = [np.arange(L * 3, dtype=np.float32).reshape(L, 1, 3) for L in lens]
    cams = [{"intrinsics": {}, "extrinsics": np.arange(L * 12, dtype=np.float64).reshape(L, 3, 4)} for L in lens]
    for subset, stride in ((0.1, 1), (0.1, 2), (1.0, 3), (0.5, 3)):
        c2, q3, q2 = run.subset_views(cams, p3d, p2d, subset=subset, stride=stride)
        for i, L in enumerate(lens):
            if subset < 1:
                n = int(round(L // stride * subset) * stride)
                start = run.deterministic_random(0, L - n + 1, str(L))
                idx = np.arange(start, start + n, stride)
            else:
                idx = np.arange(0, L, stride)
            assert q2[i].shape[0] == q3[i].shape[0] == c2[i]["extrinsics"].shape[0] == len(idx)
            np.testing.assert_array_equal(q2[i][:, 0, 0], 2 * idx)
            np.testing.assert_array_equal(q3[i][:, 0, 0], 3 * idx)
            np.testing.assert_array_equal(c2[i]["extrinsics"][:, 0, 0], 12 * idx)
    # the inputs are untouched
    assert p2d[0].shape[0] == 1000 and cams[0]["extrinsics"].shape[0] == 1000
    c2, q3, q2 = run.subset_views(cams, p3d, p2d)  # subset 1, stride 1: the views as they are
    assert q2 is p2d and q3 is p3d and c2 is cams


def test_downsample_slices_extrinsics_with_poses():
    """--downsample 2 on a CMU-style split: 2D, 3D and per-frame extrinsics keep equal
    lengths (the documented divergence from the reference, which leaves K.E undecimated)."""
    from vp3d_amd.datasets import downsample
    data = {"01": {"walk_0": {"positions_3d": [np.zeros((301, 17, 3), np.float32)],
                              "keypoints": [np.zeros((301, 17, 2), np.float32)],
                              "cameras": [{"intrinsics": {}, "extrinsics": np.zeros((301, 3, 4))}]}}}
    d = downsample(data, 2)["01"]["walk_0"]
    assert d["positions_3d"][0].shape[0] == d["keypoints"][0].shape[0] == 151
    assert d["cameras"][0]["extrinsics"].shape[0] == 151
    assert downsample(data, 1) is data
