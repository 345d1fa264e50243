"""Diagnostic: per-launch phase stamps of one 2^30 select (KTH_STAMPS=1 build
path of libkth.so prints them to stderr after each select)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mpi-k-selection_amd"))
import torch  # noqa: E402

import kselect  # noqa: E402

log2n = int(sys.argv[1]) if len(sys.argv) > 1 else 30
fam = sys.argv[2] if len(sys.argv) > 2 else "uniform_half"
n = 1 << log2n
sel = kselect.Selector(0)
keys = torch.empty(n, dtype=torch.int32, device="cuda")
sel.fill(keys, n, fam)
out = torch.zeros(4, dtype=torch.int32, device="cuda")
for i in range(4):
    print(f"--- select {i}", file=sys.stderr, flush=True)
    sel.select_async(keys, n, n // 2, out[i:i + 1])
sel.sync()
print(out.tolist(), sel.stats()["path"], flush=True)
