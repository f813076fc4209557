#!/usr/bin/env python3
"""One-line digest of a bench.py JSON line: value, ms/step, dominant-kernel TF/s, per-layer ms."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().split("\n")[-1])
r = d["roofline"]
print(f"{d['value']:.0f} {d['unit']} {d['dtype']} {d['ms_per_step']:.3f} ms/step | "
      f"{r['kernel']} {r['achieved']:.0f}/{r['peak']:.0f} {r['unit']} | "
      + " ".join(f"{k}={v:.3f}" for k, v in d["per_layer_ms"].items()))
