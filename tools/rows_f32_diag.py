"""Diagnostic: the full-shape f32 rows case of tests/test_gpu_parity.py::test_rows_full_shape;
prints mismatching rows and dumps a few to gpurun_out/ for offline analysis."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mpi-k-selection_amd"))
import kselect  # noqa: E402

sel = kselect.Selector(0)
R, C = 65536, 4096
g = torch.Generator(device="cuda")
g.manual_seed(123)
m = torch.rand((R, C), generator=g, device="cuda") * 2 - 1
m[::7] = torch.round(m[::7] * 8) / 8
srt = torch.sort(m, dim=1).values
out = torch.empty(R, dtype=m.dtype, device="cuda")
os.makedirs("gpurun_out", exist_ok=True)
for k in (1, 64, 2048, 4096):
    sel.rows(m, R, C, k, out, f32=True)
    sel.sync()
    bad = torch.nonzero(out != srt[:, k - 1]).flatten()
    print(f"k={k}: {bad.numel()} bad rows; first {bad[:10].tolist()}", flush=True)
    for r in bad[:3].tolist():
        row = m[r].cpu().numpy()
        print(f"  row {r}: got {out[r].item()!r} want {srt[r, k - 1].item()!r} min {row.min()!r} max {row.max()!r} "
              f"distinct {np.unique(row).size}", flush=True)
        row.tofile(f"gpurun_out/badrow_k{k}_r{r}.bin")
