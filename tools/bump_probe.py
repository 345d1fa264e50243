"""Is the slowdown of the ~5th-12th selects after a start (or an idle pause)
ours or the device's?  Per-iteration event times of 40 back-to-back
iterations of: the select (2^30, k = n/2), torch's sum of the same 4 GiB (a
plain HBM-bound read), and the select again -- each phase after a 2 s idle
pause.  Prints one JSON line per phase."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mpi-k-selection_amd"))


def main():
    import torch

    import kselect

    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    sel = kselect.Selector(0, stream=stream)
    n = 1 << 30
    family = sys.argv[1] if len(sys.argv) > 1 else "uniform_half"
    with_sum = len(sys.argv) > 2 and sys.argv[2] == "sum"
    keys = torch.empty(n, dtype=torch.int32, device=dev)
    sel.fill(keys, n, family, param=7)
    sel.reserve(n)
    out = torch.zeros(1, dtype=torch.int32, device=dev)
    acc = torch.zeros(1, dtype=torch.int64, device=dev)
    sel.select_async(keys, n, n // 2, out)  # first-launch costs out of the way
    torch.sum(keys, dim=0, dtype=torch.int64, out=acc[0])
    torch.cuda.synchronize()

    def phase(name, fn, m=40):
        time.sleep(2.0)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(m + 1)]
        torch.cuda.synchronize()
        ev[0].record(stream)
        for i in range(m):
            fn()
            ev[i + 1].record(stream)
        torch.cuda.synchronize()
        ms = [ev[i].elapsed_time(ev[i + 1]) for i in range(m)]
        print(json.dumps({"phase": name, "ms": [round(x, 4) for x in ms],
                          "first10": round(sum(ms[:10]) / 10, 4), "last20": round(sum(ms[-20:]) / 20, 4)}), flush=True)

    for rep in range(2):
        phase(f"select_{family}_{os.environ.get('KTH_COOP', 'coop')}_{rep}", lambda: sel.select_async(keys, n, n // 2, out))
        if with_sum:
            phase(f"torch_sum_{rep}", lambda: torch.sum(keys, dim=0, dtype=torch.int64, out=acc[0]))
    sel.close()


if __name__ == "__main__":
    main()
