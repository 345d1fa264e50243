#!/usr/bin/env python3
"""bench.py -- exact k-th selection on MI355X (BASELINE.json metric).

One step = one exact selection of the k-th smallest of n int32 keys already
resident in HBM (k = n/2, the median, as in the reference's k = n/2 variants
kth-problem-seq.c~:24 and TODO-kth-problem-cgm.c~:48).

  N = 1 : BASELINE config 2 -- 2^30 keys on one GPU (kth_select_i32_async).
  N > 1 : BASELINE config 3 -- 2^30 keys per GPU (weak scaling, 2^33 at N = 8),
          one process per GPU, RCCL collectives through torch.distributed
          (kselect.dist.DistSelector); value = all ranks' keys / max-over-ranks time.

Input: counter-based synthetic keys generated on the device (family
uniform_half = [-2^30, 2^30), the reference's well-defined domain, so the CPU
baselines are correct runs of the reference).  The answer of every run is
verified on the device with an exact rank certificate (#<v < k <= #<=v).

Extra fields: "roofline" (streaming kernel k_main: 4 B/key algorithmic bytes /
its HIP-event-timed duration vs 8 TB/s; traffic from profiles/pmc_traffic.json
when present) and "cpu_baseline" (rank 0, N = 1: the reference's own seq select
block, vector.c compiled from /root/reference into oracle/_ref, on a bounded
sample of the same family).
"""
import argparse
import ctypes
import json
import os
import platform
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "mpi-k-selection_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak, /opt/skills/guides/MI355X_MICROARCH.md


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


class _IntVector(ctypes.Structure):  # reference vector.h:7-11
    _fields_ = [("size", ctypes.c_int), ("capacity", ctypes.c_int), ("data", ctypes.POINTER(ctypes.c_int))]


def cpu_baseline(keys_np, family):
    """The reference's seq select block (kth-problem-seq.c:30-35: VecQuickSort + VecGet
    on one core) timed on this host on a bounded sample of the workload."""
    import numpy as np

    n = keys_np.size
    k = n // 2
    ref = os.path.join(REPO, "oracle", "_ref", "libvector_ref.so")
    buf = np.array(keys_np, dtype=np.int32, copy=True)
    if os.path.exists(ref):
        lib = ctypes.CDLL(ref)
        lib.VecGet.restype = ctypes.c_int
        v = _IntVector(n, n, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_int)))
        t0 = time.perf_counter()
        lib.VecQuickSort(ctypes.byref(v))
        ans = lib.VecGet(ctypes.byref(v), ctypes.c_int(k - 1))
        dt = time.perf_counter() - t0
        kind = "reference"
        what = "reference vector.c (oracle/_ref/libvector_ref.so): VecQuickSort + VecGet(k-1)"
    else:
        lib = ctypes.CDLL(os.path.join(REPO, "oracle", "liboracle.so"))
        lib.ko_seq_ref_inplace.restype = ctypes.c_int32
        lib.ko_seq_ref_inplace.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64]
        t0 = time.perf_counter()
        ans = lib.ko_seq_ref_inplace(buf.ctypes.data, n, k)
        dt = time.perf_counter() - t0
        kind = "port"
        what = "oracle restatement ko_seq_ref_inplace (qsort + VecGet)"
    return {
        "value": n / dt / 1e9,
        "unit": "Gkeys/s",
        "cores": 1,
        "kind": kind,
        "sample": f"seq select block, {what}, on 2^{n.bit_length() - 1} keys of {family}, k=n/2, "
                  f"{dt:.2f} s; host {cpu_model()} ({os.cpu_count()} cpus visible)",
        "seconds": dt,
        "answer": int(ans),
    }


def cpu_baseline_cgm(keys_np, procs, timeout=120):
    """The reference CGM program (TODO-kth-problem-cgm.c, n/k parameterised) under mpirun."""
    binary = os.path.join(REPO, "oracle", "_ref", "cgm_param")
    mpirun = "/opt/conda/bin/mpirun"
    if not (os.path.exists(binary) and os.path.exists(mpirun)):
        return None
    n = keys_np.size
    with tempfile.NamedTemporaryFile(suffix=".bin", delete=False) as f:
        keys_np.astype("<i4").tofile(f)
        path = f.name
    try:
        env = dict(os.environ, KO_N=str(n), KO_K=str(n // 2), KO_TIME="1", KO_INPUT=path)
        p = subprocess.run([mpirun, "-n", str(procs), binary], env=env, capture_output=True, text=True,
                           timeout=timeout)
        import re

        m = re.search(r"kth element[= ]\s*(-?\d+)\s*\n\s*time:\s*([0-9.]+)", p.stdout)
        if not m:
            return {"error": (p.stdout + p.stderr)[-300:]}
        t = float(m.group(2))
        return {"value": n / t / 1e9, "unit": "Gkeys/s", "cores": procs, "kind": "reference",
                "sample": f"mpirun -n {procs} CGM (oracle/_ref/cgm_param) on 2^{n.bit_length() - 1} keys, k=n/2, "
                          f"MPI_Wtime {t:.3f} s (TODO-kth-problem-cgm.c:76,279)",
                "answer": int(m.group(1))}
    except subprocess.TimeoutExpired:
        return {"error": f"timeout {timeout}s"}
    finally:
        os.unlink(path)


def rows_main(args):
    """BASELINE config 5: out[r] = k-th smallest of row r of a rows x cols matrix
    (kth_select_rows_{i32,f32}); one step = one call over the whole matrix.
    N > 1: independent replicas (each rank its own matrix, weak scaling)."""
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local_rank = int(os.environ.get("LOCAL_RANK", 0))
    import torch
    import torch.distributed as dist

    import kselect

    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    sel = kselect.Selector(local_rank, stream=stream)
    R, C = args.rows, args.cols
    k = args.k or C // 2
    f32 = args.rows_dtype == "f32"
    g = torch.Generator(device=dev)
    g.manual_seed(args.seed + rank)
    if f32:
        m = torch.rand((R, C), generator=g, device=dev, dtype=torch.float32) * 2 - 1
        out = torch.empty(R, dtype=torch.float32, device=dev)
    else:
        m = torch.randint(-2 ** 31, 2 ** 31, (R, C), generator=g, device=dev, dtype=torch.int64).to(torch.int32)
        out = torch.empty(R, dtype=torch.int32, device=dev)

    if args.topk:
        vals = torch.empty((R, k), dtype=m.dtype, device=dev)
        cols_out = torch.empty((R, k), dtype=torch.int32, device=dev)

        def step():
            sel.topk_rows(m, R, C, k, vals, cols_out, largest=True, f32=f32)
    else:
        def step():
            sel.rows(m, R, C, k, out, f32=f32)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(2 * args.steps)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        evs[2 * i].record(stream)
        step()
        evs[2 * i + 1].record(stream)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    kern_ms = sum(evs[2 * i].elapsed_time(evs[2 * i + 1]) for i in range(args.steps)) / args.steps
    # exact check on a slice of rows against torch's sort (total order; no NaNs here)
    chk = min(R, 4096)
    if args.topk:  # same value multiset as torch.topk (order and tie choice differ by contract)
        want = torch.sort(torch.topk(m[:chk], k, dim=1).values, dim=1).values
        verified = bool(torch.equal(torch.sort(vals[:chk], dim=1).values, want))
    else:
        want = torch.sort(m[:chk], dim=1).values[:, k - 1]
        verified = bool(torch.equal(out[:chk], want))
    keys_total = R * C * world
    value = keys_total / (elapsed / args.steps) / 1e9
    achieved = 4.0 * R * C / (kern_ms * 1e-3) / 1e9
    rows_traffic = None  # PMC HBM bytes per launch (tools/gpu_profiles.sh), for this exact workload
    tpath = os.path.join(REPO, "profiles", f"pmc_traffic_rows_{args.rows_dtype}.json")
    if os.path.exists(tpath) and not args.topk and (R, C, k) == (65536, 4096, 64):
        try:
            rows_traffic = json.load(open(tpath)).get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            rows_traffic = None
    res = {
        "metric": ("Gkeys/s batched top-k (largest) per row" if args.topk else "Gkeys/s batched k-th per row")
                  + " (65536 x 4096, BASELINE config 5)",
        "value": value, "unit": "Gkeys/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed * 1e3 / args.steps, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32" if f32 else "int32",
        "data": "synthetic (torch.rand / torch.randint on device)",
        "config": {"workload": f"{'top-k' if args.topk else 'k-th'} per row of a {R} x {C} "
                               f"{'f32' if f32 else 'int32'} matrix, k={k}",
                   "rows": R, "cols": C, "k": k, "parallelism": f"replicas{world}" if world > 1 else "single"},
        "roofline": {"bound": "hbm", "kernel": "kth::k_rows_reg" if C <= 4096 else "kth::k_rows",
                     "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": rows_traffic,
                     "algorithmic_bytes_per_launch": 4 * R * C, "avg_launch_ms": kern_ms},
        "verified": verified,
    }
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0 if verified else 1


def topk_main(args):
    """top-k (k smallest, int64 indices, index order) of one
    2^log2n int32 array (kth_topk_i32 = select + count pass + ordered
    compaction); one step = one call.  N > 1: independent replicas."""
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local_rank = int(os.environ.get("LOCAL_RANK", 0))
    import torch
    import torch.distributed as dist

    import kselect

    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    sel = kselect.Selector(local_rank, stream=stream)
    n = 1 << args.log2n
    k = args.k or 1024
    keys = torch.empty(n, dtype=torch.int32, device=dev)
    sel.fill(keys, n, args.family, seed=args.seed + rank, param=7)
    sel.reserve(n)
    vals = torch.empty(k, dtype=torch.int32, device=dev)
    idx = torch.empty(k, dtype=torch.int64, device=dev)
    for _ in range(args.warmup):
        sel.topk(keys, n, k, vals, idx)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(2 * args.steps)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        evs[2 * i].record(stream)
        sel.topk(keys, n, k, vals, idx)
        evs[2 * i + 1].record(stream)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    call_ms = sum(evs[2 * i].elapsed_time(evs[2 * i + 1]) for i in range(args.steps)) / args.steps
    # exact check: same values as torch.topk (smallest), indices point at them, index order
    want = torch.sort(torch.topk(keys, k, largest=False).values).values
    verified = bool(torch.equal(torch.sort(vals).values, want) and torch.equal(keys[idx], vals)
                    and bool((idx[1:] > idx[:-1]).all()))
    achieved = 4.0 * n / (call_ms * 1e-3) / 1e9
    res = {
        "metric": "Gkeys/s top-k (smallest, values + int64 indices) of one int32 array",
        "value": n * world / (elapsed / args.steps) / 1e9, "unit": "Gkeys/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed * 1e3 / args.steps,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "int32",
        "data": "synthetic (device counter-based generator, splitmix64)",
        "config": {"workload": f"top-{k} of 2^{args.log2n} int32 keys, {args.family}", "n": n, "k": k,
                   "parallelism": f"replicas{world}" if world > 1 else "single"},
        "roofline": {"bound": "hbm", "kernel": "whole kth_topk_i32 call (select + k_topk_count + scan + write)",
                     "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                     "traffic": None, "algorithmic_bytes_per_launch": 4 * n, "avg_launch_ms": call_ms},
        "verified": verified,
    }
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0 if verified else 1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--log2n", type=int, default=30, help="keys per GPU = 2^log2n")
    ap.add_argument("--family", default="uniform_half")
    ap.add_argument("--seed", type=lambda s: int(s, 0), default=0x5EED0001)
    ap.add_argument("--k", type=int, default=0, help="global 1-based rank (default n_total/2)")
    ap.add_argument("--cpu-log2n", type=int, default=25)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dist", action="store_true",
                    help="run the sharded (kth_dist_* + RCCL) protocol even on one GPU")
    ap.add_argument("--workload", choices=["select", "rows", "topk"], default="select",
                    help="select: BASELINE config 2/3 (the metric); rows: config 5, batched k-th per row; "
                         "topk: top-k of one array (--k, default 1024)")
    ap.add_argument("--rows", type=int, default=65536)
    ap.add_argument("--cols", type=int, default=4096)
    ap.add_argument("--rows-dtype", choices=["i32", "f32"], default="i32")
    ap.add_argument("--topk", action="store_true", help="rows workload: top-k (largest) values + columns per row")
    args = ap.parse_args()
    if args.workload == "rows":
        return rows_main(args)
    if args.workload == "topk":
        return topk_main(args)

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local_rank = int(os.environ.get("LOCAL_RANK", 0))

    import torch
    import torch.distributed as dist

    import kselect
    from kselect.dist import DistSelector, HipBackend

    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    # one explicit stream for everything (torch ops, the selector, RCCL): the
    # legacy null stream would add implicit synchronisation to every launch
    torch.cuda.set_stream(torch.cuda.Stream(dev))
    sharded = world > 1 or args.dist
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    elif args.dist:  # the sharded protocol on one GPU: a one-rank RCCL group
        dist.init_process_group("nccl", device_id=dev, store=dist.HashStore(), rank=0, world_size=1)

    def barrier():
        if world > 1:
            dist.barrier()

    sel = kselect.Selector(local_rank)
    sel.set_stream(torch.cuda.current_stream(dev))
    n_local = 1 << args.log2n
    n_total = n_local * world
    k = args.k or n_total // 2
    family = kselect.FAMILIES[args.family]
    keys = torch.empty(n_local, dtype=torch.int32, device=dev)
    sel.fill(keys, n_local, family, args.seed, offset=rank * n_local, n_total=n_total)
    out = torch.zeros(args.warmup + args.steps, dtype=torch.int32, device=dev)

    if not sharded:
        sel.reserve(n_local)

        def step(i):
            sel.select_async(keys, n_local, k, out[i:i + 1])
    else:
        ds = DistSelector(HipBackend(local_rank, sel))

        def step(i):
            ds.select(keys, n_local, n_total, k, out=out[i:i + 1])

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    barrier()
    sel.enable_timing(True)
    torch.cuda.synchronize()
    barrier()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    barrier()
    n_sel, main_ms, total_ms = sel.take_timing()
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # exact rank certificate of every answer (device-side integer counts)
    answers = out.cpu().tolist()
    v = answers[args.warmup]
    cnt = torch.stack([(keys < v).sum(), (keys <= v).sum()]).to(torch.int64)
    if world > 1:
        dist.all_reduce(cnt)
    lt, le = (int(x) for x in cnt.tolist())
    verified = (lt < k <= le) and all(a == v for a in answers)
    stats = sel.stats() if not sharded else None

    ms_per_step = elapsed * 1e3 / args.steps
    value = n_total / (elapsed / args.steps) / 1e9
    avg_main_ms = main_ms / max(1, n_sel)
    achieved = 4.0 * n_local / (avg_main_ms * 1e-3) / 1e9 if avg_main_ms > 0 else None
    traffic = None
    tpath = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if os.path.exists(tpath):
        try:
            tj = json.load(open(tpath))
            if tj.get("log2n") == args.log2n and tj.get("family") == args.family:
                traffic = tj.get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            traffic = None

    res = {
        "metric": "Gkeys/s exact k-th select, 2^30 int32 (1 GPU) / 2^33 (8 GPU); % HBM roofline",
        "value": value,
        "unit": "Gkeys/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic (device counter-based generator, splitmix64)",
        "config": {
            "workload": f"exact k-th select (median) of 2^{args.log2n} int32 keys per GPU, {args.family}",
            "n_total": n_total,
            "k": k,
            "keys_per_gpu": n_local,
            "family": args.family,
            "parallelism": f"shards{world}" if sharded else "single",
        },
        "roofline": {
            "bound": "hbm",
            "kernel": "kth::k_main (streaming pass)",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": (achieved / HBM_PEAK_GBS) if achieved else None,
            "traffic": traffic,
            "algorithmic_bytes_per_launch": 4 * n_local,
            "avg_launch_ms": avg_main_ms,
        },
        "verified": bool(verified),
        "answer": v,
        "whole_select_ms_events": total_ms / max(1, n_sel) if not sharded else None,
    }
    if stats:
        res["path"] = {1: "lds", 2: "radix", 3: "window", 4: "window_fallback"}.get(stats["path"], "?")
        res["candidates"] = stats["candidates"]

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        nc = 1 << args.cpu_log2n
        tmp = torch.empty(nc, dtype=torch.int32, device=dev)
        sel.fill(tmp, nc, family, args.seed, offset=0, n_total=nc)
        keys_np = tmp.cpu().numpy()
        del tmp
        try:
            res["cpu_baseline"] = cpu_baseline(keys_np, args.family)
            cg = cpu_baseline_cgm(keys_np, min(8, os.cpu_count() or 1))
            if cg:
                res["cpu_baseline_cgm"] = cg
        except Exception as e:  # noqa: BLE001 -- baseline is informational
            res["cpu_baseline"] = {"error": repr(e)}

    if rank == 0:
        print(json.dumps(res), flush=True)
    if sharded:
        dist.destroy_process_group()
    return 0 if verified else 1


if __name__ == "__main__":
    sys.exit(main())
