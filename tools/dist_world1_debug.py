"""Diagnostic: the sharded protocol at world 1 (RCCL), stats after each select."""
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mpi-k-selection_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import kselect  # noqa: E402
from kselect.dist import DistSelector, HipBackend  # noqa: E402

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29541")
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
n = 1 << 23
gen = kselect.Selector(0)
b = HipBackend(0)
ds = DistSelector(b)
for fam in ("uniform_full", "few_distinct", "sorted_desc"):
    keys = torch.empty(n, dtype=torch.int32, device="cuda")
    gen.fill(keys, n, fam, seed=0x5EED0001, param=7)
    gen.sync()
    srt = np.sort(keys.cpu().numpy())
    for k in (1, n // 2, n, n // 2, 1):
        got = int(ds.select(keys, n, n, k).item())
        st = b.sel.stats()
        print(fam, "k", k, "got", got, "want", int(srt[k - 1]), "ok", got == int(srt[k - 1]), st, flush=True)
ds.close()
dist.destroy_process_group()
