"""Diagnostic: the sharded protocol with one rank vs the single-GPU select."""
import os
import socket
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mpi-k-selection_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import kselect  # noqa: E402
from kselect.dist import DistSelector, HipBackend  # noqa: E402

s = socket.socket()
s.bind(("127.0.0.1", 0))
os.environ["MASTER_ADDR"] = "127.0.0.1"
os.environ["MASTER_PORT"] = str(s.getsockname()[1])
s.close()
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
ds = DistSelector(HipBackend(0))
sel = kselect.Selector(0)
for fam in ("uniform_full", "few_distinct", "sorted_desc"):
    n = 1 << 23
    keys = torch.empty(n, dtype=torch.int32, device="cuda")
    sel.fill(keys, n, fam)
    sel.sync()
    srt = np.sort(keys.cpu().numpy())
    for k in (1, n // 2, n):
        got = int(ds.select(keys, n, n, k).item())
        st = ds.b.sel.stats()
        one = sel.select(keys, k)
        print(fam, k, "dist", got, "single", one, "true", int(srt[k - 1]), "ok" if got == srt[k - 1] else "BAD", st)
dist.destroy_process_group()
