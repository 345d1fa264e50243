"""Diagnostic: one top-k on the window path with KTH_TOPK_DEBUG=1 (tile counts vs a host recount)."""
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mpi-k-selection_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import kselect  # noqa: E402

n = (1 << 22) + 5
a = np.random.default_rng(n).integers(-2 ** 31, 2 ** 31, size=n, dtype=np.int64).astype(np.int32)
d = torch.from_numpy(a).cuda()
sel = kselect.Selector(0)
for k in (n // 2, n // 1024 + 1):
    vals = torch.empty(k, dtype=torch.int32, device="cuda")
    idx = torch.empty(k, dtype=torch.int64, device="cuda")
    sel.topk(d, n, k, vals, idx)
    sel.sync()
    print("k", k, "stats", sel.stats(), "select", sel.select(d, k), "true", int(np.sort(a)[k - 1]), flush=True)
