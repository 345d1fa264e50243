"""Host enqueue cost of the single-process sharded select (kth_sharded_*).

Prints, for a ShardedSelector over the given devices and 2^log2n keys per
device, the host microseconds one kth_sharded_select_i32 spends enqueueing
(kth_sharded_enqueue_us) next to its wall time per select.  DESIGN.md cites
this for VERDICT r2 item 3 (enqueue per device-step vs the 50 us bar)."""
import argparse
import json
import sys
import time

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0] + "/mpi-k-selection_amd")
import torch  # noqa: E402

import kselect  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--devices", default="0")
    ap.add_argument("--log2n", type=int, default=30)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    devs = [int(x) for x in a.devices.split(",")]
    n = 1 << a.log2n
    shards = []
    for d in devs:
        s = kselect.Selector(d)
        t = torch.empty(n, dtype=torch.int32, device=f"cuda:{d}")
        s.fill(t, n, "uniform_half", offset=d * n, n_total=n * len(devs))
        s.sync()
        s.close()
        shards.append(t)
    sh = kselect.ShardedSelector(devs)
    k = n * len(devs) // 2
    for _ in range(3):
        sh.select(shards, k)
    enq, wall = [], []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        sh.select(shards, k)
        wall.append((time.perf_counter() - t0) * 1e6)
        enq.append(sh.enqueue_us())
    enq.sort()
    wall.sort()
    # device-steps per select: begin+sample, window+scan, 3 levels, result; plus 5 collectives
    print(json.dumps({"devices": devs, "keys_per_device": n, "enqueue_us_median": enq[len(enq) // 2],
                      "enqueue_us_min": enq[0], "wall_us_median": wall[len(wall) // 2],
                      "enqueue_us_per_device": enq[len(enq) // 2] / len(devs)}))
    sh.close()


if __name__ == "__main__":
    main()
