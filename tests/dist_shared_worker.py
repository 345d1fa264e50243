"""One rank of the sharded select with every rank on GPU 0 (KTH_SHARE_GPU=1 test
mode; run by tests/test_gpu_shared.py, one process per rank).

The product's multi-process path end to end -- file rendezvous, one libkth ctx
per process, DistSelector(HipBackend) with the early result and the DistStatus
read -- with the collectives staged through host memory over gloo
(kselect.rccl.HostComm) instead of RCCL, which refuses two ranks on one device.
The reference's own launch and collectives this replaces:
TODO-kth-problem-cgm.c:53-61 (mpirun ranks), :103 (Scatterv), :135-190
(Gather / Bcast / Allreduce of the weighted-median rounds).

Env: RANK, WORLD_SIZE, KTH_RDV_FILE (FileStore path).  Prints ONE JSON line:
{"rank": r, "golden": [[case, answer, error], ...], "synthetic": [[fam, n, k,
answer, error, want], ...]} (want only on rank 0, which generates the whole
input to compute it).
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from conftest import load_input  # noqa: E402 -- also puts kselect on sys.path


def main():
    import numpy as np
    import torch
    import torch.distributed as dist

    import kselect
    from kselect.dist import DistSelector, HipBackend, shard_bounds

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", init_method="file://" + os.environ["KTH_RDV_FILE"], rank=rank,
                            world_size=world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.cuda.set_stream(torch.cuda.Stream(dev))
    sel = kselect.Selector(0)
    ds = DistSelector(HipBackend(0, sel))
    assert type(ds.comm).__name__ == "HostComm" and ds.comm.world == world, ds.comm
    res = {"rank": rank, "golden": [], "synthetic": []}
    try:
        with open(os.path.join(HERE, "golden", "expected.json")) as f:
            golden = json.load(f)
        for i, c in enumerate(golden["cases"]):
            a = load_input(c["input"])
            start, cnt = shard_bounds(a.size, rank, world)  # TODO-kth-problem-cgm.c:81-100
            shard = torch.from_numpy(np.ascontiguousarray(a[start:start + cnt])).to(dev)
            out = ds.select(shard, cnt, a.size, c["k"])
            res["golden"].append([i, int(out.item()), ds.error()])
        for fam in ("uniform_full", "few_distinct", "sorted_desc"):
            n = (1 << 24) + 5
            start, cnt = shard_bounds(n, rank, world)
            shard = torch.empty(cnt, dtype=torch.int32, device=dev)
            sel.fill(shard, cnt, fam, param=7, offset=start, n_total=n)
            srt = None
            if rank == 0:
                whole = torch.empty(n, dtype=torch.int32, device=dev)
                sel.fill(whole, n, fam, param=7)
                srt = torch.sort(whole).values.cpu()
                del whole
            for k in (1, n // 3, n // 2, n):
                out = ds.select(shard, cnt, n, k)
                res["synthetic"].append([fam, n, k, int(out.item()), ds.error(),
                                         int(srt[k - 1]) if srt is not None else None])
    finally:
        ds.close()
        sel.close()
        dist.destroy_process_group()
    sys.stdout.write(json.dumps(res) + "\n")
    sys.stdout.flush()


if __name__ == "__main__":
    main()
