#!/usr/bin/env python3
"""Per-layer HBM traffic of the lifter forward from rocprofv3 PMC passes.

    python tools/traffic.py gpurun_out/TAG [--batch 8192] [--dtype bf16] [--out profiles/traffic_bf16_b8192.json]

Reads the FETCH_SIZE and WRITE_SIZE passes (`tools/pmc_pass.sh TAG FETCH_SIZE WRITE_SIZE`
over a `bench.py` run), orders the dispatches by Dispatch_Id and splits them into
forwards: a forward starts at the expand-conv dispatch of the bench batch (grid =
ceil(B*81/256) or ceil(B*81/128) workgroups of 256 threads for the fused expand
kernel) and is followed by the 9 conv-GEMM dispatches
of blocks 1-4 and the shrink, in layer order.

Units and corrections (MI355X_MICROARCH.md, "HBM"): FETCH_SIZE and WRITE_SIZE
are KiB; on gfx950 FETCH_SIZE tallies each 128-byte read request as 64 bytes, so
the read side is doubled.  WRITE_SIZE is exact for 16-byte-per-lane stores.
"""
import argparse
import sys
import csv
import glob
import json
import os
from collections import defaultdict

LAYERS = ["expand", "block1_k3", "block1_1x1", "block2_k3", "block2_1x1", "block3_k3",
          "block3_1x1", "block4_k3", "block4_1x1", "shrink"]


def read_counter(d, name, prefix="pmc"):
    rows = {}
    for f in glob.glob(os.path.join(d, prefix + "*", "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if r["Counter_Name"] != name:
                    continue
                rows[int(r["Dispatch_Id"])] = (r["Kernel_Name"], int(r["Grid_Size"]), float(r["Counter_Value"]))
    return rows


def forwards(rows, B):
    """Yield lists of (layer, value) per forward of batch B."""
    ids = sorted(rows)
    # the fused expand kernel runs 256 rows per workgroup (RB = 4) or 128 (RB = 2, the
    # camera concat): grid in threads = workgroups x 256
    expand_grids = {((B * 81 + 255) // 256) * 256, ((B * 81 + 127) // 128) * 256}
    # other expand forms (f16x3: two workgroups per CU): the largest expand grid in the trace
    expand_grids.add(max((g for n, g, _ in rows.values() if "expand_gemm" in n), default=0))
    # the fp32 path: the expand conv on the 128 x 128 f32 tile kernel (1024 channels)
    f32_expand = ((B * 81 + 127) // 128) * 8 * 256
    i = 0
    while i < len(ids):
        name, grid, _ = rows[ids[i]]
        start = ("expand_gemm" in name and grid in expand_grids) or ("conv_gemm_f32" in name and grid == f32_expand)
        if not start:
            i += 1
            continue
        # a layer starts at a conv_gemm dispatch; split-K tail dispatches (tail_split_kernel,
        # tail_reduce_*) add to the layer before them, except the f16x3 shrink's (round 6): a
        # tail_split_kernel followed by shrink_reduce_x3_kernel is the shrink layer itself
        seq = [["expand", rows[ids[i]][2]]]
        last_split = 0.0
        j = i + 1
        while j < len(ids):
            n2, g2, v2 = rows[ids[j]]
            if "conv_gemm" in n2:
                if len(seq) == len(LAYERS):
                    break
                seq.append([LAYERS[len(seq)], v2])
                last_split = 0.0
            elif "tail_split_kernel" in n2 and len(seq) > 1:
                seq[-1][1] += v2
                last_split = v2
            elif "shrink_reduce" in n2 and len(seq) == len(LAYERS) - 1:
                seq[-1][1] -= last_split
                seq.append([LAYERS[len(seq)], last_split + v2])
                last_split = 0.0
            elif "reduce" in n2 and len(seq) > 1:
                seq[-1][1] += v2
            elif "expand_gemm" in n2:
                break
            j += 1
        if len(seq) == len(LAYERS):
            yield [tuple(x) for x in seq]
        i = j


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--dominant", default="block1_k3")
    ap.add_argument("--out")
    ap.add_argument("--prefix", default="pmc", help="PMC pass directories under DIR (pmc*, traj_pmc*)")
    a = ap.parse_args()
    acc = {c: defaultdict(list) for c in ("FETCH_SIZE", "WRITE_SIZE")}
    for c in acc:
        for seq in forwards(read_counter(a.dir, c, a.prefix), a.batch):
            for layer, v in seq:
                acc[c][layer].append(v)
    per_layer = {}
    for layer in LAYERS:
        f, w = acc["FETCH_SIZE"].get(layer), acc["WRITE_SIZE"].get(layer)
        if not f or not w:
            continue
        rd = 2.0 * 1024.0 * sum(f) / len(f)
        wr = 1024.0 * sum(w) / len(w)
        per_layer[layer] = {"read_bytes": rd, "write_bytes": wr, "hbm_bytes": rd + wr,
                            "launches": min(len(f), len(w))}
    import subprocess
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "dynamic-camera-augmented-videopose3d_amd"))
    from vp3d_amd import build as _build
    try:
        commit = subprocess.run(["git", "rev-parse", "--short", "HEAD"], capture_output=True, text=True).stdout.strip()
    except OSError:
        commit = None
    out = {"batch": a.batch, "dtype": a.dtype, "dominant": a.dominant,
           "build_hash": _build.source_hash(), "git_commit": commit or None,
           "hbm_bytes_per_launch": per_layer.get(a.dominant, {}).get("hbm_bytes"),
           "per_layer": per_layer,
           "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes in {a.dir}/{a.prefix}*; "
                     "FETCH_SIZE x 2 (gfx950 128-B requests tallied as 64 B), KiB -> B"}
    s = json.dumps(out, indent=1)
    print(s)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(s + "\n")


if __name__ == "__main__":
    main()
