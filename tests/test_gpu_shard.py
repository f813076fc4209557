"""Config 4's sharded path through libvp3d: two ranks of the bench's
strong-scaling step, started as fresh processes (torch.multiprocessing spawn; the test
process is never exec-replaced), sharing the one GPU over gloo.  Each rank takes
vp3d_amd.shard.window_shard of the same seeded global window set -- the function
bench.py's windows_main shards with -- and runs lifter.forward_windows (the window gather
fused into the expand conv, then the stack) on its slice.  The concatenated shards must
be bit-equal to the unsharded forward of the whole set, and the global MPJPE from the
single end-of-run all_reduce must equal the unsharded one."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

FW = [3, 3, 3, 3, 3]
G = 65536  # config 4's global batch


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _setup(dev):
    from common.models.TemporalModel import TemporalModelOptimized1f
    from vp3d_amd import synth
    from vp3d_amd.pipeline import SyntheticWindowPool
    model = TemporalModelOptimized1f(17, 2, 17, FW, channels=1024)
    sd = synth.lifter_state_dict([(k, tuple(v.shape)) for k, v in model.state_dict().items()], seed=0)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    model.eval().cuda(dev)
    pool = SyntheticWindowPool(1000, dev)  # the bench's window source
    return model, pool


def _run_shard(rank, world, dev, dtype):
    from vp3d_amd.shard import window_shard
    model, pool = _setup(dev)
    pairs, s, e = window_shard(pool, G, rank, world, dev)
    lifter = model.native_lifter(dev)
    RF = model.receptive_field()
    y = torch.empty((e - s, 1, 17, 3), device=dev)
    with torch.no_grad():
        lifter.forward_windows(pool.seqs, pairs, RF, (RF - 1) // 2, concat_cams=False, dtype=dtype, out=y)
    torch.cuda.synchronize()
    return y, s, e


def _worker(rank, world, port, outdir, dtype):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from vp3d_amd import shard, synth
    y, s, e = _run_shard(rank, world, torch.device("cuda", 0), dtype)
    gt = torch.from_numpy(synth.gt_poses(3, "shard_gt", G, 17).reshape(G, 1, 17, 3)[s:e]).cuda()
    err = torch.linalg.norm(y.double() - gt.double(), dim=-1)
    g = shard.reduce_mpjpe(float(err.sum()), float(err.numel()))
    np.savez(os.path.join(outdir, f"r{rank}.npz"), y=y.cpu().numpy(), s=s, e=e, g=g)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("dtype", ["bf16", "f16x3"])
def test_config4_two_ranks_bit_equal(tmp_path, dtype):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), dtype), nprocs=world, join=True)
    parts = [np.load(os.path.join(tmp_path, f"r{r}.npz")) for r in range(world)]
    assert [(int(p["s"]), int(p["e"])) for p in parts] == [(0, G // 2), (G // 2, G)]
    y_full, _, _ = _run_shard(0, 1, torch.device("cuda", 0), dtype)
    y_full = y_full.cpu().numpy()
    y_cat = np.concatenate([p["y"] for p in parts])
    assert y_cat.shape == y_full.shape == (G, 1, 17, 3)
    assert np.array_equal(y_cat, y_full)
    from vp3d_amd import synth
    gt = synth.gt_poses(3, "shard_gt", G, 17).reshape(G, 1, 17, 3)
    want = float(np.mean(np.linalg.norm(y_full.astype(np.float64) - gt, axis=-1)))
    for p in parts:
        assert abs(float(p["g"]) - want) <= 1e-12 * max(1.0, want)


@pytest.mark.parametrize("dtype", ["f16x3", "fp32"])
def test_config4_eight_shards_bit_equal(dtype):
    """Config 4 at N = 8 (8,192 windows per rank), the shards run one after another on the one
    GPU: their concatenation is bit-equal to the unsharded 65,536-window forward.  At 8,192
    windows every conv leaves a partial last round (128 tiles past the whole rounds), which
    runs as 256 x 128 half-N tiles in the whole tile's K order (conv_gemm_a4 HN) -- not as
    split-K chains, which gave up bit identity across shard sizes; layers under 384 tiles run
    on q64 (a4's K order) and the exact f32 shrink is the same bits narrow or tiled.  (The
    16-bit dtypes' shrink is not: its narrow kernel for < 32,768 rows sums K in another order
    than the tile kernel)"""
    dev = torch.device("cuda", 0)
    y_full, _, _ = _run_shard(0, 1, dev, dtype)
    parts = [_run_shard(r, 8, dev, dtype) for r in range(8)]
    assert [(s, e) for _, s, e in parts] == [(r * G // 8, (r + 1) * G // 8) for r in range(8)]
    y_cat = torch.cat([y for y, _, _ in parts]).cpu().numpy()
    assert np.array_equal(y_cat, y_full.cpu().numpy())
