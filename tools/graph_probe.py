"""Launch-gap probe: the same 2^30-key selects enqueued eagerly on a created
stream, eagerly on the null stream, and replayed from one captured HIP graph
(torch.cuda.CUDAGraph over kth_select_i32_async on the ctx stream), the three
interleaved round by round after a long warmup.  Prints ms per select for each
and whether every answer agrees.  Design probe, not part of the product.
Usage: python tools/graph_probe.py [log2n=30] [reps=20] [rounds=6] [order=eager,null,graph]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-k-selection_amd"))
import torch  # noqa: E402

import kselect  # noqa: E402


def main():
    log2n = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 6
    order = sys.argv[4].split(",") if len(sys.argv) > 4 else ["eager", "null", "graph"]
    n, k = 1 << log2n, 1 << (log2n - 1)
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(dev)
    sel = kselect.Selector(0, stream=s)
    keys = torch.empty(n, dtype=torch.int32, device=dev)
    sel.fill(keys, n, kselect.FAMILIES["uniform_half"], 12345)
    sel.reserve(n)
    outs = {m: torch.zeros(2 * reps, dtype=torch.int32, device=dev) for m in ("eager", "null", "graph")}

    def eager(out):
        for i in range(2 * reps):  # an even count: the ctx's alternating slot sets come back to the start
            sel.select_async(keys, n, k, out[i:i + 1])

    torch.cuda.synchronize()
    with torch.cuda.stream(s):
        for _ in range(5):  # warmup (and the clocks' transient)
            eager(outs["eager"])
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            eager(outs["graph"])
    torch.cuda.synchronize()
    res = {}
    for _ in range(rounds):
        for m in order:
            sel.set_stream(None if m == "null" else s)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if m == "graph":
                g.replay()
            elif m == "null":
                eager(outs[m])
            else:
                with torch.cuda.stream(s):
                    eager(outs[m])
            torch.cuda.synchronize()
            res.setdefault(m, []).append((time.perf_counter() - t0) * 1e3 / (2 * reps))
    ans = {m: o.cpu().tolist() for m, o in outs.items()}
    ok = len(set(ans["eager"])) == 1 and all(ans[m] == ans["eager"] for m in order)
    for m, v in res.items():
        med = sorted(v)[len(v) // 2]
        print(f"{m:6s} ms/select " + " ".join(f"{x:.4f}" for x in v) +
              f"  median {med:.4f} ({n / (med * 1e-3) / 1e9:.1f} Gkeys/s)")
    print("answers agree:", ok, ans["eager"][0])
    sel.close()


if __name__ == "__main__":
    main()
