"""Where does a short warmup lose time?  Per-select host times of the first
selects on a fresh process (each synchronised), then back-to-back blocks of 20
selects, then the same after an idle second -- 2^30 uniform_half, k = n/2, no
timing events on the stream.  Prints one JSON line per phase."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mpi-k-selection_amd"))


def main():
    import torch

    import kselect

    log2n = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    sel = kselect.Selector(0, stream=stream)
    n = 1 << log2n
    k = n // 2
    keys = torch.empty(n, dtype=torch.int32, device=dev)
    sel.fill(keys, n, "uniform_half")
    sel.reserve(n)
    out = torch.zeros(1, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()

    single = []
    for _ in range(40):
        t0 = time.perf_counter()
        sel.select_async(keys, n, k, out)
        torch.cuda.synchronize()
        single.append((time.perf_counter() - t0) * 1e3)
    print(json.dumps({"phase": "synced_each", "ms": [round(x, 4) for x in single]}), flush=True)

    def block(m):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(m):
            sel.select_async(keys, n, k, out)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3 / m

    print(json.dumps({"phase": "blocks_of_20", "ms_per_select": [round(block(20), 4) for _ in range(8)]}), flush=True)
    time.sleep(1.0)
    print(json.dumps({"phase": "after_idle_1s", "ms_per_select": [round(block(20), 4) for _ in range(4)]}), flush=True)
    time.sleep(1.0)
    first = []
    for _ in range(10):
        t0 = time.perf_counter()
        sel.select_async(keys, n, k, out)
        torch.cuda.synchronize()
        first.append((time.perf_counter() - t0) * 1e3)
    print(json.dumps({"phase": "synced_each_after_idle", "ms": [round(x, 4) for x in first]}), flush=True)
    sel.close()


if __name__ == "__main__":
    main()
