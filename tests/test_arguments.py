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
