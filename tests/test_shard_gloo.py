"""Multi-rank sharding rehearsed on CPU with the gloo backend,
world_size 2: window shards and halo'd time shards reassemble the unsharded
output exactly, and the single end-of-run all_reduce gives the global MPJPE.
The per-shard compute here is the CPU oracle (test infrastructure); on the GPU
node the same shard arithmetic feeds libvp3d (bench.py under torchrun)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from vp3d_amd import shard, synth

FW = [3, 3, 3]
RF = 27


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _state():
    from common.models.TemporalModel import TemporalModel
    m = TemporalModel(17, 2, 17, FW, channels=32)
    return synth.lifter_state_dict([(k, tuple(v.shape)) for k, v in m.state_dict().items()], seed=5)


def _worker(rank, world, port, outdir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle.temporal_ref import lifter_forward
    sd = _state()
    win = torch.from_numpy(synth.normalized_windows(6, "shardwin", 11, RF))
    y_w = shard.forward_sharded_windows(lambda x: lifter_forward(sd, x, FW, strided=True), win, rank, world)
    seq = torch.from_numpy(synth.normalized_windows(6, "shardseq", 1, 200))
    y_s = shard.forward_sharded_sequence(lambda x: lifter_forward(sd, x, FW), seq, RF, rank, world)
    gt = torch.from_numpy(synth.gt_poses(3, "shardgt", 11, 17)).view(11, 1, 17, 3)
    s, e = shard.shard_range(11, rank, world)
    err = torch.linalg.norm(y_w - gt[s:e], dim=-1)
    g = shard.reduce_mpjpe(float(err.sum()), float(err.numel()))
    np.savez(os.path.join(outdir, f"r{rank}.npz"), y_w=y_w.numpy(), y_s=y_s.numpy(), g=g)
    dist.barrier()
    dist.destroy_process_group()


def test_shard_ranges():
    assert [shard.shard_range(10, r, 3) for r in range(3)] == [(0, 4), (4, 7), (7, 10)]
    assert [shard.shard_range(2, r, 4) for r in range(4)] == [(0, 1), (1, 2), (2, 2), (2, 2)]
    o0, o1, i0, i1 = shard.time_shard(100, 1, 2, 243)
    assert (o0, o1, i0, i1) == (50, 100, 50, 342)
    with pytest.raises(ValueError):
        shard.shard_range(10, 2, 2)


def test_gloo_world2(tmp_path):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    from oracle.temporal_ref import lifter_forward
    sd = _state()
    win = torch.from_numpy(synth.normalized_windows(6, "shardwin", 11, RF))
    y_full = lifter_forward(sd, win, FW, strided=True).numpy()
    seq = torch.from_numpy(synth.normalized_windows(6, "shardseq", 1, 200))
    ys_full = lifter_forward(sd, seq, FW).numpy()
    parts = [np.load(os.path.join(tmp_path, f"r{r}.npz")) for r in range(world)]
    assert np.array_equal(np.concatenate([p["y_w"] for p in parts]), y_full)
    assert np.allclose(np.concatenate([p["y_s"] for p in parts], axis=1), ys_full, atol=1e-6)
    gt = synth.gt_poses(3, "shardgt", 11, 17).reshape(11, 1, 17, 3)
    want = float(np.mean(np.linalg.norm(y_full.astype(np.float64) - gt, axis=-1)))
    for p in parts:
        assert abs(float(p["g"]) - want) < 1e-6


def _grad_worker(rank, world, port, outdir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(100 + rank)
    params = [torch.nn.Parameter(torch.zeros(s)) for s in [(7, 3), (11,), (2, 5, 4)]]
    for p in params:
        p.grad = torch.randn(p.shape)
    mine = [p.grad.clone() for p in params]
    flat = shard.allreduce_gradients(params)
    flat2 = shard.allreduce_gradients(params, flat)  # reuses the bucket
    assert flat2 is flat
    np.savez(os.path.join(outdir, f"g{rank}.npz"), *[m.numpy() for m in mine],
             *[p.grad.numpy() for p in params])
    dist.destroy_process_group()


def test_allreduce_gradients_gloo_world2(tmp_path):
    """Data-parallel training's gradient averaging (one flat-bucket all_reduce per step):
    after two calls every rank holds the mean of the ranks' gradients (the second call
    averages identical values, so it is idempotent)."""
    port = _free_port()
    mp.spawn(_grad_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    g = [np.load(os.path.join(tmp_path, f"g{r}.npz")) for r in range(2)]
    for i in range(3):
        want = (g[0][f"arr_{i}"] + g[1][f"arr_{i}"]) / 2
        for r in range(2):
            np.testing.assert_allclose(g[r][f"arr_{i + 3}"], want, rtol=1e-6, atol=1e-7)
