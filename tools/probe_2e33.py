"""BASELINE config 3's size on one MI355X: kth_select_i32 over 2^33 int32 keys
(32 GiB) in one array, k in {1, 2^32, n}, each answer checked with the exact
rank certificate #(<v) < k <= #(<=v) counted on the device (in 2^30-key
chunks).  Prints one JSON line per k with the select time (synchronised,
median of reps) and the path stats."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mpi-k-selection_amd"))


def certificate(keys, v):
    import torch
    lt = le = 0
    for c in torch.split(keys, 1 << 30):
        lt += int((c < v).sum())
        le += int((c <= v).sum())
    return lt, le


def main():
    import torch

    import kselect

    log2n = int(sys.argv[1]) if len(sys.argv) > 1 else 33
    family = sys.argv[2] if len(sys.argv) > 2 else "uniform_half"
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    sel = kselect.Selector(0, stream=stream)
    n = 1 << log2n
    keys = torch.empty(n, dtype=torch.int32, device=dev)
    sel.fill(keys, n, family, param=7)
    sel.reserve(n)
    out = torch.zeros(1, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    for k in (1, n // 2, n):
        times = []
        for _ in range(reps):
            t0 = time.perf_counter()
            sel.select_async(keys, n, k, out)
            torch.cuda.synchronize()
            times.append((time.perf_counter() - t0) * 1e3)
        v = int(out.item())
        st = sel.stats()
        lt, le = certificate(keys, v)
        times.sort()
        ms = times[len(times) // 2]
        print(json.dumps({"n": n, "log2n": log2n, "family": family, "k": k, "answer": v, "ok": lt < k <= le,
                          "lt": lt, "le": le, "ms_median": ms, "ms_all": [round(t, 3) for t in times],
                          "gkeys_s": n / ms / 1e6, "path": st["path"], "candidates": st["candidates"],
                          "capacity": st["capacity"], "error": st["error"]}), flush=True)
        if not lt < k <= le:
            return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
