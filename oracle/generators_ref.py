"""ORACLE (test infrastructure only): numpy restatement of the reference batching.

Follows reference common/generators.py:
  ChunkedGenerator.__init__   :30-71   (pairs :39-45, buffers :50-52, RandomState :56)
  ChunkedGenerator.pad_chunk  :92-100  ('edge' padding of out-of-range frames)
  ChunkedGenerator.next_epoch :102-137 (window bounds :109-110, K @ E :115-125,
                                        whole reused buffers yielded: quirk Q2)
  UnchunkedGenerator          :140-205 (edge pad (pad+shift, pad-shift) :193-198, K @ E :180-190)
"""
from __future__ import annotations

import numpy as np


def intrinsic_matrix(intr) -> np.ndarray:
    """3x3 float32 K from an intrinsics dict (generators.py:116-123)."""
    fx, fy = intr["focal_length"]
    cx, cy = intr["center"]
    return np.array([[fx, 0, cx], [0, fy, cy], [0, 0, 1]], dtype=np.float32)


def chunk_pairs(seq_lengths, chunk_length=1):
    """(seq, start_3d, end_3d) triples in the reference's order (generators.py:39-45)."""
    out = []
    for i, n in enumerate(seq_lengths):
        n_chunks = (n + chunk_length - 1) // chunk_length
        offset = (n_chunks * chunk_length - n) // 2
        b = np.arange(n_chunks + 1) * chunk_length - offset
        out.extend((i, int(b[k]), int(b[k + 1])) for k in range(n_chunks))
    return out


def shuffled_pairs(seq_lengths, chunk_length=1, seed=1234):
    """RandomState(seed).permutation of the pair list (generators.py:56, :85)."""
    return np.random.RandomState(seed).permutation(chunk_pairs(seq_lengths, chunk_length))


def edge_slice(arr, start, end):
    """Frames [start, end) of arr with out-of-range frames replaced by the nearest
    valid frame (np.pad 'edge', generators.py:92-100)."""
    idx = np.clip(np.arange(start, end), 0, arr.shape[0] - 1)
    return arr[idx]


def chunked_batches(cams, poses_3d, poses_2d, batch_size, chunk_length, pad, causal_shift,
                    shuffle=True, seed=1234, random=None):
    """Yields (batch_cam, batch_3d, batch_2d) exactly as ChunkedGenerator.next_epoch does,
    including the reuse of one float64 buffer per array (stale rows in the last batch).
    `random`: the generator's RandomState carried across epochs (generators.py:56, :85;
    each epoch draws the next permutation from it); default a fresh RandomState(seed)."""
    lengths = [p.shape[0] for p in poses_2d]
    if not shuffle:
        pairs = np.array(chunk_pairs(lengths, chunk_length))
    elif random is not None:
        pairs = random.permutation(chunk_pairs(lengths, chunk_length))
    else:
        pairs = shuffled_pairs(lengths, chunk_length, seed)
    L = chunk_length + 2 * pad
    bcam = np.empty((batch_size, L, 3, 4))
    b3d = np.empty((batch_size, chunk_length) + poses_3d[0].shape[-2:])
    b2d = np.empty((batch_size, L) + poses_2d[0].shape[-2:])
    n_batches = (len(pairs) + batch_size - 1) // batch_size
    for bi in range(n_batches):
        for i, (s, a, b) in enumerate(pairs[bi * batch_size:(bi + 1) * batch_size]):
            lo, hi = a - pad - causal_shift, b + pad - causal_shift
            b2d[i] = edge_slice(poses_2d[s], lo, hi)
            bcam[i] = intrinsic_matrix(cams[s]["intrinsics"]) @ edge_slice(cams[s]["extrinsics"], lo, hi)
            b3d[i] = edge_slice(poses_3d[s], a, b)
        yield bcam, b3d, b2d


def unchunked_sequences(cams, poses_3d, poses_2d, pad, causal_shift):
    """Yields (batch_cam, batch_3d, batch_2d) per sequence with 'edge' padding of
    (pad + shift) frames before and (pad - shift) after (generators.py:178-205)."""
    for cam, p3, p2 in zip(cams, poses_3d, poses_2d):
        n = p2.shape[0]
        idx = np.clip(np.arange(-(pad + causal_shift), n + pad - causal_shift), 0, n - 1)
        camseq = intrinsic_matrix(cam["intrinsics"]) @ cam["extrinsics"]
        yield camseq[idx][None], (None if p3 is None else p3[None]), p2[idx][None]
