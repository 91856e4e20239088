"""Compare two tools/frame_dump.py outputs: bit-identity and the max difference per array."""
import sys

import torch

a, b = (torch.load(p, weights_only=True) for p in sys.argv[1:3])
for k in ("out12", "tile"):
    x, y = a[k], b[k]
    same = torch.equal(x, y)
    d = float((x - y).abs().max()) if x.shape == y.shape else float("nan")
    print(f"{k}: identical={same} max|d|={d:.3e} differing={int((x != y).sum()) if x.shape == y.shape else -1}")
