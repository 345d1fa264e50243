"""Host cost of the sharded protocol's Python path (kselect.dist.DistSelector
over a one-rank RCCL group): wall time per select() call, split at the host's
wait on level 0's status, at a size where the device finishes first.  Design
probe, not part of the product.  Usage: python tools/dist_host_probe.py [log2n=24] [reps=200]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-k-selection_amd"))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import kselect  # noqa: E402
from kselect.dist import DistSelector, HipBackend  # noqa: E402


def main():
    log2n = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    n = 1 << log2n
    dev = torch.device("cuda", 0)
    torch.cuda.set_stream(torch.cuda.Stream(dev))
    dist.init_process_group("nccl", device_id=dev, store=dist.HashStore(), rank=0, world_size=1)
    sel = kselect.Selector(0)
    sel.set_stream(torch.cuda.current_stream(dev))
    keys = torch.empty(n, dtype=torch.int32, device=dev)
    sel.fill(keys, n, kselect.FAMILIES["uniform_half"], 12345)
    ds = DistSelector(HipBackend(0, sel))
    outs = torch.zeros(reps, dtype=torch.int32, device=dev)
    views = [outs[i:i + 1] for i in range(reps)]
    for i in range(20):
        ds.select(keys, n, n, n // 2, out=views[i])
    torch.cuda.synchronize()
    # time each step of the protocol generator on the host
    acc = {}
    t_all = time.perf_counter()
    for i in range(reps):
        t = time.perf_counter()
        gen = ds.steps(keys, n, n, n // 2, views[i])
        while True:
            try:
                op = next(gen)
            except StopIteration:
                break
            t2 = time.perf_counter()
            acc.setdefault("steps", []).append(t2 - t)
            if op[0] == "all_gather":
                ds.comm.all_gather(op[1], op[2])
            else:
                ds.comm.all_reduce_sum_(op[1])
            t = time.perf_counter()
            acc.setdefault(op[0], []).append(t - t2)
        acc.setdefault("tail", []).append(time.perf_counter() - t)
    torch.cuda.synchronize()
    total = (time.perf_counter() - t_all) / reps
    print(f"n=2^{log2n}: {total * 1e6:.1f} us per select (host loop incl. device waits)")
    for k, v in acc.items():
        v = sorted(v)
        print(f"  {k:10s} calls {len(v):5d} median {v[len(v) // 2] * 1e6:8.1f} us  p90 {v[int(len(v) * 0.9)] * 1e6:8.1f} us")
    ok = len(set(outs.cpu().tolist())) == 1
    print("answers agree:", ok)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
