"""Embarrassingly parallel sharding of the lifter over ranks (one process per GPU).

SURVEY.md §8(e): windows (Optimized1f) are independent, so a global batch of B
windows is split into contiguous per-rank shards with no data-path collective;
long sequences (dilated TemporalModel) split by time with a read-only input halo
of receptive_field - 1 frames per shard (no exchange).  The only collective is
the end-of-run metric reduction: (sum of per-joint errors, count) — 16 bytes per
rank — reduced once with all_reduce.

Training (run.py:451-487) is data-parallel the usual way: each rank trains on its own
shard of the batch and the gradients are averaged with ONE all_reduce of a flat
bucket per step (`allreduce_gradients`; 68 MB at 1024 channels, far below the
xGMI-ring sweet spot, so one bucket beats per-tensor calls).  BatchNorm statistics
stay per rank (no SyncBN), as under torch DDP.

The helpers here are pure index arithmetic plus those reductions, so they are
exercised on CPU with the gloo backend (tests/test_shard_gloo.py) and run
unchanged over RCCL on the GPU node.
"""
from __future__ import annotations

from typing import Callable, Tuple

import torch
import torch.distributed as dist


def shard_range(total: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous [start, end) of `total` items owned by `rank`; sizes differ by <= 1."""
    if world <= 0 or not (0 <= rank < world):
        raise ValueError(f"bad rank/world {rank}/{world}")
    base, extra = divmod(total, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def time_shard(T_out: int, rank: int, world: int, receptive_field: int) -> Tuple[int, int, int, int]:
    """Output frames [o0, o1) of a sequence with T_out outputs owned by `rank`, and the
    input frames [i0, i1) they need (T_in = T_out + rf - 1; output t reads inputs
    t .. t + rf - 1).  Neighbouring shards overlap by rf - 1 input frames (the halo)."""
    o0, o1 = shard_range(T_out, rank, world)
    return o0, o1, o0, o1 + receptive_field - 1


def window_shard(pool, G: int, rank: int, world: int, device) -> Tuple[torch.Tensor, int, int]:
    """This rank's slice of a global window set of G (sequence, start) pairs drawn from
    `pool` (vp3d_amd.pipeline.SyntheticWindowPool or anything with global_pairs(G)):
    the pair rows [s, e) on `device`, and s, e.  The config-4 bench and its multi-rank
    GPU test shard through this one function."""
    s, e = shard_range(G, rank, world)
    pairs_all = pool.global_pairs(G)
    return torch.from_numpy(pairs_all[s:e]).to(device), s, e


def forward_sharded_windows(fn: Callable[[torch.Tensor], torch.Tensor], windows: torch.Tensor,
                            rank: int, world: int) -> torch.Tensor:
    """Run `fn` on this rank's contiguous shard of a (B, T, J, F) window batch."""
    s, e = shard_range(int(windows.shape[0]), rank, world)
    return fn(windows[s:e])


def forward_sharded_sequence(fn: Callable[[torch.Tensor], torch.Tensor], seq: torch.Tensor,
                             receptive_field: int, rank: int, world: int) -> torch.Tensor:
    """Run a dilated-model `fn` on this rank's time shard of a padded (1, T_in, J, F)
    sequence; returns the (1, o1 - o0, J_out, 3) slice of the full output."""
    T_out = int(seq.shape[1]) - receptive_field + 1
    o0, o1, i0, i1 = time_shard(T_out, rank, world, receptive_field)
    if o1 <= o0:
        return seq.new_zeros((1, 0) + tuple(seq.shape[2:3]) + (3,))
    return fn(seq[:, i0:i1])


def reduce_mpjpe(err_sum: float, count: float, device=None) -> float:
    """Global MPJPE from per-rank (sum of errors, count) with one all_reduce
    (identity when torch.distributed is not initialised)."""
    t = torch.tensor([float(err_sum), float(count)], dtype=torch.float64,
                     device=device if device is not None else "cpu")
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t[0] / t[1]) if t[1] > 0 else float("nan")


def allreduce_gradients(params, flat: torch.Tensor | None = None) -> torch.Tensor | None:
    """Average the .grad of `params` over all ranks with a single all_reduce of one flat
    bucket (RCCL on the GPU node, gloo in the CPU tests).  Returns the bucket so the
    caller can pass it back next step (no re-allocation); no-op when not distributed."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return flat
    grads = [p.grad for p in params if p.grad is not None]
    n = sum(g.numel() for g in grads)
    if flat is None or flat.numel() != n or flat.device != grads[0].device:
        flat = torch.empty(n, dtype=grads[0].dtype, device=grads[0].device)
    torch.cat([g.reshape(-1) for g in grads], out=flat)
    dist.all_reduce(flat, op=dist.ReduceOp.SUM)
    flat.div_(dist.get_world_size())
    o = 0
    for g in grads:
        g.copy_(flat[o:o + g.numel()].view_as(g))
        o += g.numel()
    return flat
