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
CPU_SHARE = int(os.environ.get("KTH_CPU_SHARE", "16"))  # host CPUs granted per GPU job on the GPU box


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def emit(obj):
    """One JSON result line in ONE write(2): rank processes share the parent's
    stdout, and print() writes the text and the newline separately, so two
    ranks' lines could interleave."""
    sys.stdout.flush()
    data = (json.dumps(obj) + "\n").encode()
    while data:
        data = data[os.write(1, data):]


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


RDV_ENV = "KTH_RDV_FILE"  # launch_ranks' file rendezvous (no TCP port to probe and race for)
# TEST MODE, not a scaling point: every rank on GPU 0, the collectives staged
# through host memory over gloo (RCCL refuses two ranks on one device).  It runs
# everything the multi-GPU launch depends on -- launcher, rendezvous, one ctx
# per process, the sharded protocol with its early result and DistStatus read --
# except RCCL's transport, on the one-GPU pool.
SHARE_ENV = "KTH_SHARE_GPU"


def shared_gpu():
    return os.environ.get(SHARE_ENV, "0") not in ("", "0")


def init_group(dev, backend="nccl"):
    """The ranks' process group: under torchrun (the driver's launch) env://
    with the launcher's store; under launch_ranks a FileStore at $KTH_RDV_FILE.
    Ranks sharing one GPU (KTH_SHARE_GPU=1) form a gloo group."""
    import torch.distributed as dist

    if shared_gpu():
        backend, dev = "gloo", None
    path = os.environ.get(RDV_ENV)
    if path:
        dist.init_process_group(backend, device_id=dev, init_method="file://" + path,
                                rank=int(os.environ["RANK"]), world_size=int(os.environ["WORLD_SIZE"]))
    else:
        dist.init_process_group(backend, device_id=dev)


def coll_device(dev):
    """Where the bench's own small collectives (timing max, certificate counts)
    take tensors: host memory when the ranks share a GPU (gloo group)."""
    import torch

    return torch.device("cpu") if shared_gpu() else dev


def launch_ranks(n, argv):
    """`bench.py --gpus N` without a launcher: start N rank processes of this
    script (RANK / LOCAL_RANK / WORLD_SIZE set, one GPU each, rendezvous through
    a FileStore file named by $KTH_RDV_FILE: no port is probed, so none can be
    taken between the probe and the bind), replacing the reference's
    `mpirun -n P` launch (TODO-kth-problem-cgm.c:53-61).  This parent never
    imports torch or touches a GPU; it forwards the ranks' output, stops every
    rank when one fails, and exits with the first failing rank's code."""
    rdv_dir = tempfile.mkdtemp(prefix="kth_rdv_")
    rdv = os.path.join(rdv_dir, "store")
    log(f"bench: launching {n} ranks (one per GPU), rendezvous file://{rdv}")
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", **{RDV_ENV: rdv})
        env.pop("MASTER_PORT", None)
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__), *argv], env=env))
    rc = 0
    live = list(enumerate(procs))
    while live:
        time.sleep(0.2)
        for item in list(live):
            r, p = item
            code = p.poll()
            if code is None:
                continue
            live.remove(item)
            if code != 0:
                log(f"bench: rank {r} exited with code {code}; stopping the other ranks")
                rc = rc or code
                for _, q in live:
                    q.terminate()
    for f in os.listdir(rdv_dir):
        os.unlink(os.path.join(rdv_dir, f))
    os.rmdir(rdv_dir)
    return rc


def need_gpu(local_rank):
    """Fail loudly (there is no CPU fallback) unless GPU `local_rank` is visible
    (GPU 0 for every rank when they share one, KTH_SHARE_GPU=1)."""
    import torch

    if shared_gpu():
        local_rank = 0
    ndev = torch.cuda.device_count() if torch.cuda.is_available() else 0
    if local_rank >= ndev:
        raise SystemExit(f"bench: rank needs GPU {local_rank} but {ndev} GPU(s) are visible (no CPU fallback)")
    torch.cuda.set_device(local_rank)
    return torch.device("cuda", local_rank)


class _IntVector(ctypes.Structure):  # reference vector.h:7-11
    _fields_ = [("size", ctypes.c_int), ("capacity", ctypes.c_int), ("data", ctypes.POINTER(ctypes.c_int))]


def cpu_host():
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count()
    return {"cpu_model": cpu_model(), "nproc": os.cpu_count(), "affinity_cpus": aff}


def cpu_baseline(keys_np, family, min_seconds=5.0, max_reps=50):
    """The reference's seq select block (kth-problem-seq.c:30-35: VecQuickSort +
    VecGet(k-1) on one core), timed on this host.  BASELINE config 1: 2^20 keys,
    k = n/2.  Each repetition sorts a fresh copy; reported: median over the
    repetitions of the monotonic time and of the CPU time (clock(), what the
    reference prints, kth-problem-seq.c:30,35)."""
    import numpy as np

    n = keys_np.size
    k = n // 2
    ref = os.path.join(REPO, "oracle", "_ref", "libvector_ref.so")
    if os.path.exists(ref):
        lib = ctypes.CDLL(ref)
        lib.VecGet.restype = ctypes.c_int
        kind = "reference"
        what = "reference vector.c compiled from its own source (oracle/_ref/libvector_ref.so): VecQuickSort + VecGet(k-1)"

        def run(buf):
            v = _IntVector(n, n, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_int)))
            lib.VecQuickSort(ctypes.byref(v))
            return lib.VecGet(ctypes.byref(v), ctypes.c_int(k - 1))
    else:
        lib = ctypes.CDLL(os.path.join(REPO, "oracle", "liboracle.so"))
        lib.ko_seq_ref_inplace.restype = ctypes.c_int32
        lib.ko_seq_ref_inplace.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64]
        kind = "port"
        what = "oracle restatement ko_seq_ref_inplace (qsort with the reference comparator + VecGet)"

        def run(buf):
            return lib.ko_seq_ref_inplace(buf.ctypes.data, n, k)
    mono, cpu, answers = [], [], set()
    while len(mono) < 3 or (sum(mono) < min_seconds and len(mono) < max_reps):
        buf = np.array(keys_np, dtype=np.int32, copy=True)
        c0, t0 = time.thread_time(), time.monotonic()
        answers.add(int(run(buf)))
        t1, c1 = time.monotonic(), time.thread_time()
        mono.append(t1 - t0)
        cpu.append(c1 - c0)
    dt, dc = float(np.median(mono)), float(np.median(cpu))
    want = int(np.partition(keys_np, k - 1)[k - 1])
    return {
        "value": n / dt / 1e9,
        "unit": "Gkeys/s",
        "cores": 1,
        "kind": kind,
        "sample": f"BASELINE config 1: seq select block, {what}, 2^{n.bit_length() - 1} keys of {family}, k=n/2; "
                  f"median of {len(mono)} runs: {dt * 1e3:.1f} ms monotonic, {dc * 1e3:.1f} ms clock()",
        "n": n,
        "reps": len(mono),
        "seconds_monotonic": dt,
        "seconds_clock": dc,
        "answer": answers.pop() if len(answers) == 1 else sorted(answers),
        "want": want,
    }


def cpu_baseline_cgm(keys_np, procs, reps=3, timeout=120):
    """The reference CGM program (TODO-kth-problem-cgm.c compiled from its own
    source, n/k read from the environment: oracle/_ref/cgm_param) under
    `mpirun -n procs`; its own MPI_Wtime from before the Scatterv to the answer
    (:76, :279).  Median of `reps` runs; `wall_s` is the whole mpirun (rank 0's
    key generation -- the input file read through the VecAdd shim -- included).
    Raises on any failure."""
    import re

    import numpy as np

    binary = os.path.join(REPO, "oracle", "_ref", "cgm_param")
    mpirun = "/opt/conda/bin/mpirun"
    for f in (binary, mpirun):
        if not os.path.exists(f):
            raise RuntimeError(f"CGM baseline: {f} missing")
    n = keys_np.size
    with tempfile.NamedTemporaryFile(suffix=".bin", delete=False) as f:
        keys_np.astype("<i4").tofile(f)
        path = f.name
    times, answers, walls = [], set(), []
    try:
        env = dict(os.environ, KO_N=str(n), KO_K=str(n // 2), KO_TIME="1", KO_INPUT=path)
        for _ in range(reps):
            w0 = time.monotonic()
            p = subprocess.run([mpirun, "-n", str(procs), binary], env=env, capture_output=True, text=True,
                               timeout=timeout, stdin=subprocess.DEVNULL)
            walls.append(time.monotonic() - w0)
            m = re.search(r"kth element[= ]\s*(-?\d+)\s*\n\s*time:\s*([0-9.]+)", p.stdout)
            if not m:
                raise RuntimeError(f"CGM baseline P={procs}: no answer line (rc {p.returncode}): "
                                   f"{(p.stdout + p.stderr)[-300:]!r}")
            answers.add(int(m.group(1)))
            times.append(float(m.group(2)))
    finally:
        os.unlink(path)
    t = float(np.median(times))
    return {"value": n / t / 1e9, "unit": "Gkeys/s", "cores": procs, "procs": procs, "kind": "reference",
            "sample": f"mpirun -n {procs} reference CGM (oracle/_ref/cgm_param) on 2^{n.bit_length() - 1} keys, "
                      f"k=n/2, median MPI_Wtime of {reps} runs {t * 1e3:.1f} ms (TODO-kth-problem-cgm.c:76,279)",
            "seconds": t, "reps": reps, "n": n, "wall_s": float(np.median(walls)),
            "answer": answers.pop() if len(answers) == 1 else sorted(answers)}


def cpu_baselines(keys_np, family):
    """Every CPU baseline of BASELINE.md on this host, errors collected rather
    than swallowed: (cpu_baseline, cpu_baseline_cgm list, errors)."""
    import numpy as np

    want = int(np.partition(keys_np, keys_np.size // 2 - 1)[keys_np.size // 2 - 1])
    errors, seq, cgm = [], None, []
    try:
        seq = cpu_baseline(keys_np, family)
        seq["answer_ok"] = seq["answer"] == want
        if not seq["answer_ok"]:
            errors.append(f"seq baseline answered {seq['answer']}, true k-th is {want}")
    except Exception as e:  # noqa: BLE001 -- reported at the top level of the line
        errors.append(f"seq baseline: {e!r}")
    host = cpu_host()
    # BASELINE.md asks for P in {2, 4, 8, all cores}.  "All cores" is this job's
    # CPU share, not the machine: the GPU box exposes every host CPU (nproc,
    # affinity 256) but grants one GPU's job a share of 16 (its OMP_NUM_THREADS /
    # MAX_JOBS), and more MPI ranks than that would oversubscribe the share
    share = min(CPU_SHARE, host["affinity_cpus"] or 1)
    for P in sorted({2, 4, 8, share}):
        try:
            r = cpu_baseline_cgm(keys_np, P)
            if P == share:
                r["sample"] += (f"; all cores of this job's CPU share: {share} of the host's {host['nproc']} "
                                f"CPUs ({CPU_SHARE} per GPU on the GPU box)")
            r["answer_ok"] = r["answer"] == want
            if not r["answer_ok"]:
                errors.append(f"CGM baseline P={P} answered {r['answer']}, true k-th is {want}")
            cgm.append(r)
        except Exception as e:  # noqa: BLE001
            errors.append(f"CGM baseline P={P}: {e!r}")
    if seq is not None:
        seq.pop("want", None)
        seq["sample"] += f"; host {host['cpu_model']}, nproc {host['nproc']}, affinity {host['affinity_cpus']} cpus"
    return seq, cgm, errors, host


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

    dev = need_gpu(local_rank)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    if world > 1:
        init_group(dev)
    sel = kselect.Selector(dev.index, stream=stream)
    R, C = args.rows, args.cols
    k = args.k or C // 2
    f32 = args.rows_dtype == "f32"
    g = torch.Generator(device=dev)
    g.manual_seed(args.seed + rank)
    dup = args.rows_input == "dup"
    if f32:
        m = torch.rand((R, C), generator=g, device=dev, dtype=torch.float32) * 2 - 1
        if dup:  # duplicate-heavy: 17 distinct values per row
            m = torch.round(m * 8) / 8
        out = torch.empty(R, dtype=torch.float32, device=dev)
    else:
        lo, hi = (-3, 4) if dup else (-2 ** 31, 2 ** 31)  # duplicate-heavy: 7 distinct values
        m = torch.randint(lo, hi, (R, C), generator=g, device=dev, dtype=torch.int64).to(torch.int32)
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
        t = torch.tensor([elapsed], dtype=torch.float64, device=coll_device(dev))
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
    # algorithmic bytes of a launch: the keys read, the outputs written (top-k:
    # a value and an int32 column per kept key; k-th: one value per row)
    algo_bytes = 4 * R * C + (8 * R * k if args.topk else 4 * R)
    achieved = algo_bytes / (kern_ms * 1e-3) / 1e9
    rows_traffic, rows_note = None, "no PMC measurement for this workload"
    if not dup and (R, C, k) == (65536, 4096, 64):
        rows_traffic, rows_note = pmc_traffic(
            f"pmc_traffic_rows_{'topk_' if args.topk else ''}{args.rows_dtype}.json", None, None)
    res = {
        "metric": ("Gkeys/s batched top-k (largest) per row" if args.topk else "Gkeys/s batched k-th per row")
                  + " (65536 x 4096, BASELINE config 5)",
        "value": value, "unit": "Gkeys/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed * 1e3 / args.steps, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32" if f32 else "int32",
        "data": "synthetic (torch.rand / torch.randint on device)" + (
            ", duplicate-heavy: f32 round(u*8)/8 (17 values), int32 randint[-3, 3] (7 values)" if dup else ""),
        "config": {"workload": f"{'top-k' if args.topk else 'k-th'} per row of a {R} x {C} "
                               f"{'f32' if f32 else 'int32'} matrix, k={k}" + (", duplicate-heavy" if dup else ""),
                   "input": args.rows_input,
                   "rows": R, "cols": C, "k": k, "parallelism": f"replicas{world}" if world > 1 else "single"},
        "roofline": {"bound": "hbm", "kernel": "kth::k_rows_reg" if C <= 4096 else "kth::k_rows",
                     "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": rows_traffic, "traffic_source": rows_note,
                     "algorithmic_bytes_per_launch": algo_bytes, "avg_launch_ms": kern_ms},
        "verified": verified,
    }
    if rank == 0:
        emit(res)
    if world > 1:
        dist.destroy_process_group()
    return 0 if verified else 1


def pmc_traffic(name, log2n, family, field="hbm_bytes_per_launch"):
    """HBM bytes per launch of the dominant kernel from profiles/<name> (two
    rocprofv3 --pmc passes, tools/pmc_traffic.py), used only when it was
    measured on the libkth.so build loaded now (kth_build_id) and on this
    workload; otherwise (None, reason)."""
    import kselect
    path = os.path.join(REPO, "profiles", name)
    try:
        tj = json.load(open(path))
    except (OSError, ValueError):
        return None, f"profiles/{name} missing or unreadable"
    here = kselect.LIB.kth_build_id().decode()
    if tj.get("build_id") != here:
        return None, f"profiles/{name} was measured on libkth build {tj.get('build_id')}, loaded build is {here}"
    if log2n is not None and (tj.get("log2n"), tj.get("family")) != (log2n, family):
        return None, f"profiles/{name} is for 2^{tj.get('log2n')} {tj.get('family')}, not this workload"
    return tj.get(field), f"profiles/{name} (PMC FETCH_SIZE/WRITE_SIZE, build {here}; {tj.get('correction', '')})"


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

    dev = need_gpu(local_rank)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    if world > 1:
        init_group(dev)
    sel = kselect.Selector(dev.index, stream=stream)
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
        t = torch.tensor([elapsed], dtype=torch.float64, device=coll_device(dev))
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    call_ms = sum(evs[2 * i].elapsed_time(evs[2 * i + 1]) for i in range(args.steps)) / args.steps
    # exact check: same values as torch.topk (smallest), indices point at them, index order
    want = torch.sort(torch.topk(keys, k, largest=False).values).values
    verified = bool(torch.equal(torch.sort(vals).values, want) and torch.equal(keys[idx], vals)
                    and bool((idx[1:] > idx[:-1]).all()))
    # algorithmic bytes: the input read once + the k (value, int64 index) pairs written
    alg_bytes = 4 * n + 12 * k
    traffic, traffic_note = pmc_traffic(f"pmc_traffic_topk_k{k}.json", args.log2n, args.family,
                                        field="hbm_bytes_per_call")
    achieved = alg_bytes / (call_ms * 1e-3) / 1e9
    res = {
        "metric": "Gkeys/s top-k (smallest, values + int64 indices) of one int32 array",
        "value": n * world / (elapsed / args.steps) / 1e9, "unit": "Gkeys/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed * 1e3 / args.steps,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "int32",
        "data": "synthetic (device counter-based generator, splitmix64)",
        "config": {"workload": f"top-{k} of 2^{args.log2n} int32 keys, {args.family}", "n": n, "k": k,
                   "parallelism": f"replicas{world}" if world > 1 else "single"},
        "roofline": {"bound": "hbm", "kernel": "whole kth_topk_i32 call (select + count + scan + write)",
                     "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                     "traffic": traffic, "traffic_source": traffic_note,
                     "algorithmic_bytes_per_launch": alg_bytes, "avg_launch_ms": call_ms},
        "verified": verified,
    }
    if rank == 0:
        emit(res)
    if world > 1:
        dist.destroy_process_group()
    return 0 if verified else 1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--log2n", type=int, default=30, help="keys per GPU = 2^log2n")
    ap.add_argument("--family", default="uniform_half")
    ap.add_argument("--seed", type=lambda s: int(s, 0), default=0x5EED0001)
    ap.add_argument("--k", type=int, default=0, help="global 1-based rank (default n_total/2)")
    ap.add_argument("--cpu-log2n", type=int, default=20, help="CPU baseline size (BASELINE config 1: 2^20)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-cpu-full", action="store_true",
                    help="skip the reference CGM leg at the GPU workload's own size (config 2: 2^30, ~45 s)")
    ap.add_argument("--local-shards", type=int, default=1,
                    help="P > 1: P shards of 2^log2n keys on this one GPU through kth_sharded_* (config 3 on one GPU)")
    ap.add_argument("--dist", action="store_true",
                    help="run the sharded (kth_dist_* + RCCL) protocol even on one GPU")
    ap.add_argument("--workload", choices=["select", "rows", "topk"], default="select",
                    help="select: BASELINE config 2/3 (the metric); rows: config 5, batched k-th per row; "
                         "topk: top-k of one array (--k, default 1024)")
    ap.add_argument("--rows", type=int, default=65536)
    ap.add_argument("--cols", type=int, default=4096)
    ap.add_argument("--rows-dtype", choices=["i32", "f32"], default="i32")
    ap.add_argument("--topk", action="store_true", help="rows workload: top-k (largest) values + columns per row")
    ap.add_argument("--rows-input", choices=["uniform", "dup"], default="uniform",
                    help="rows workload input: uniform (f32 U(-1,1), int32 full range) or dup (duplicate-heavy)")
    ap.add_argument("--probe-launch", action="store_true",
                    help="(tests) each rank prints its launch environment as JSON and exits before touching a GPU")
    ap.add_argument("--probe-rendezvous", action="store_true",
                    help="(tests) the ranks meet as a gloo group through the launch's rendezvous, all-reduce their "
                         "ranks and print the sum; no GPU is touched")
    args = ap.parse_args()
    if args.gpus < 1:
        log(f"bench: --gpus {args.gpus} must be >= 1")
        return 2
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch_ranks(args.gpus, sys.argv[1:])
    world = int(os.environ.get("WORLD_SIZE", 1))
    if world != args.gpus:
        log(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}: refusing to report a {world}-rank run as {args.gpus}")
        return 2
    if args.probe_rendezvous:
        import torch
        import torch.distributed as dist

        init_group(None, backend="gloo")
        t = torch.tensor([int(os.environ.get("RANK", 0))])
        dist.all_reduce(t)
        emit({"rank": dist.get_rank(), "world": dist.get_world_size(), "rank_sum": int(t.item())})
        dist.destroy_process_group()
        return 0
    if args.probe_launch:
        emit({k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", RDV_ENV)})
        return 0
    if args.workload == "rows":
        return rows_main(args)
    if args.workload == "topk":
        return topk_main(args)

    rank = int(os.environ.get("RANK", 0))
    local_rank = int(os.environ.get("LOCAL_RANK", 0))

    import torch
    import torch.distributed as dist

    import kselect
    from kselect.dist import DistSelector, HipBackend

    dev = need_gpu(local_rank)
    # one explicit stream for everything (torch ops, the selector, RCCL): the
    # legacy null stream would add implicit synchronisation to every launch
    torch.cuda.set_stream(torch.cuda.Stream(dev))
    sharded = world > 1 or args.dist
    if world > 1:
        init_group(dev)
    elif args.dist:  # the sharded protocol on one GPU: a one-rank RCCL group
        dist.init_process_group("nccl", device_id=dev, store=dist.HashStore(), rank=0, world_size=1)

    def barrier():
        if world > 1:
            dist.barrier()

    sel = kselect.Selector(dev.index)
    sel.set_stream(torch.cuda.current_stream(dev))
    P = args.local_shards
    if P > 1 and sharded:
        raise SystemExit("bench: --local-shards runs on one GPU without --dist / WORLD_SIZE > 1")
    n_local = 1 << args.log2n
    n_total = n_local * world * P
    k = args.k or n_total // 2
    family = kselect.FAMILIES[args.family]
    keys = torch.empty(n_local * P, dtype=torch.int32, device=dev)
    sel.fill(keys, n_local * P, family, args.seed, offset=rank * n_local, n_total=n_total)
    out = torch.zeros(args.warmup + args.steps, dtype=torch.int32, device=dev)
    outv = [out[i:i + 1] for i in range(args.warmup + args.steps)]  # (views made before any timing)
    comm_world = None
    local_answers = [0] * (args.warmup + args.steps)

    if P > 1:
        # BASELINE config 3's shards on ONE GPU: P shards of 2^log2n keys
        # through kth_sharded_* with the device repeated (the local
        # transport: the same per-shard steps, the all-reduces a device-side
        # slot sum).  kth_sharded_select_i32 is synchronous: each step ends
        # with the answer on the host.
        views = [keys[i * n_local:(i + 1) * n_local] for i in range(P)]
        sh = kselect.ShardedSelector([dev.index] * P)
        sizes = [n_local] * P

        def step(i):
            local_answers[i] = sh.select(views, k, sizes)
    elif not sharded:
        sel.reserve(n_local)

        def step(i):
            sel.select_async(keys, n_local, k, outv[i])
    else:
        ds = DistSelector(HipBackend(dev.index, sel))
        comm_world = getattr(ds.comm, "world", None)
        if comm_world != world:
            raise SystemExit(f"bench: RCCL communicator spans {comm_world} ranks, WORLD_SIZE is {world}")

        def step(i):
            ds.select(keys, n_local, n_total, k, out=outv[i])

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    barrier()
    # the timed region: exactly K steps, no HIP timing events on the stream
    # (events switch the queue to timestamped dispatches, ~10 us a select)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    barrier()
    # then the same K steps once more with events around the streaming pass
    # and each whole select: roofline.avg_launch_ms (not the value)
    sel.enable_timing(True)
    torch.cuda.synchronize()
    barrier()
    t2 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i)
    torch.cuda.synchronize()
    elapsed_ev = time.perf_counter() - t2
    barrier()
    n_sel, main_ms, total_ms = sel.take_timing()
    sel.enable_timing(False)
    if world > 1:
        t = torch.tensor([elapsed, elapsed_ev], dtype=torch.float64, device=coll_device(dev))
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, elapsed_ev = (float(x) for x in t.tolist())

    # exact rank certificate of every answer (device-side integer counts)
    answers = local_answers if P > 1 else out.cpu().tolist()
    v = answers[args.warmup]
    cnt = torch.zeros(2, dtype=torch.int64, device=dev)
    for c in torch.split(keys, 1 << 30):  # (bounded temporaries at 2^33)
        cnt += torch.stack([(c < v).sum(), (c <= v).sum()]).to(torch.int64)
    if world > 1:
        cnt = cnt.to(coll_device(dev))
        dist.all_reduce(cnt)
    lt, le = (int(x) for x in cnt.tolist())
    verified = (lt < k <= le) and all(a == v for a in answers)
    stats = sel.stats() if not sharded and P == 1 else None

    ms_per_step = elapsed * 1e3 / args.steps
    value = n_total / (elapsed / args.steps) / 1e9
    avg_main_ms = main_ms / max(1, n_sel)
    achieved = 4.0 * n_local / (avg_main_ms * 1e-3) / 1e9 if avg_main_ms > 0 else None
    kernel = "kth::k_main (streaming pass)"
    if P > 1:  # the shards' ctxs are internal to the handle: the whole select, host-timed
        avg_main_ms = ms_per_step
        achieved = 4.0 * n_local * P / (ms_per_step * 1e-3) / 1e9
        kernel = f"whole sharded select ({P} shards on one GPU, host-timed, synchronous)"
    traffic, traffic_note = pmc_traffic("pmc_traffic.json", args.log2n, args.family)
    if P > 1:
        traffic, traffic_note = None, "PMC traffic is measured per k_main launch (one shard), not per sharded select"

    shared = shared_gpu() and world > 1
    res = {
        "metric": "Gkeys/s exact k-th select, 2^30 int32 (1 GPU) / 2^33 (8 GPU); % HBM roofline",
        "value": value,
        "unit": "Gkeys/s",
        "n_gpus": 1 if shared else world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic (device counter-based generator, splitmix64)",
        "config": {
            "workload": (f"exact k-th select (median) of 2^{args.log2n} int32 keys per GPU, {args.family}" if P == 1 else
                         f"BASELINE config 3 on one GPU: exact k-th select (median) of {P} shards x 2^{args.log2n} "
                         f"int32 keys (kth_sharded local transport), {args.family}"),
            "n_total": n_total,
            "k": k,
            "keys_per_gpu": n_local,
            "family": args.family,
            "parallelism": "shared-gpu-host-comm" if shared else (
                f"shards{world}" if sharded else (f"local_shards{P}" if P > 1 else "single")),
            "ranks": world,
            "rccl_world": None if shared else (comm_world if sharded else None),
        },
        "roofline": {
            "bound": "hbm",
            "kernel": kernel,
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": (achieved / HBM_PEAK_GBS) if achieved else None,
            "traffic": traffic,
            "traffic_source": traffic_note,
            "algorithmic_bytes_per_launch": 4 * n_local * P,
            "avg_launch_ms": avg_main_ms,
        },
        "verified": bool(verified),
        "answer": v,
        "whole_select_ms_events": total_ms / max(1, n_sel) if not sharded else None,
        "ms_per_step_events": elapsed_ev * 1e3 / args.steps,
    }
    if shared:
        res["scaling_point"] = False
        res["note"] = (f"TEST MODE (KTH_SHARE_GPU=1): {world} rank processes share GPU 0 and stage the collectives "
                       "through host memory over gloo; not a scaling point (the host waits at every collective)")
    if stats:
        res["path"] = {1: "lds", 2: "radix", 3: "window", 4: "window_fallback"}.get(stats["path"], "?")
        res["candidates"] = stats["candidates"]

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        nc = 1 << args.cpu_log2n
        tmp = torch.empty(nc, dtype=torch.int32, device=dev)
        sel.fill(tmp, nc, family, args.seed, offset=0, n_total=nc)
        keys_np = tmp.cpu().numpy()
        del tmp
        seq, cgm, errors, host = cpu_baselines(keys_np, args.family)
        res["cpu_baseline"] = seq
        res["cpu_baseline_cgm"] = cgm
        res["cpu_baseline_errors"] = errors
        res["cpu_host"] = host
        if not args.no_cpu_full and P == 1 and args.log2n == 30:
            # BASELINE config 2 "vs mpirun CGM on host cores" at config 2's own
            # size, in this run: the reference CGM on the very keys the GPU
            # selected (its answer must be the certified GPU answer)
            share = min(CPU_SHARE, host["affinity_cpus"] or 1)
            log(f"bench: reference CGM under mpirun -n {share} on the 2^30 GPU input (one run, ~45 s)")
            try:
                full = cpu_baseline_cgm(keys.cpu().numpy(), share, reps=1, timeout=600)
                full["answer_ok"] = full["answer"] == v and bool(verified)
                full["sample"] = (f"BASELINE config 2 at its own size: the reference CGM (oracle/_ref/cgm_param) under "
                                  f"mpirun -n {share} (all cores of this job's CPU share) on the same 2^30 "
                                  f"{args.family} keys the GPU selected, k=n/2, one run: MPI_Wtime "
                                  f"{full['seconds']:.2f} s (TODO-kth-problem-cgm.c:76,279), {full['wall_s']:.1f} s "
                                  f"wall with rank 0's key generation")
                if not full["answer_ok"]:
                    errors.append(f"CGM 2^30 P={share} answered {full['answer']}, the GPU's certified answer is {v}")
                res["cpu_baseline_cgm_full"] = full
            except Exception as e:  # noqa: BLE001 -- reported at the top level of the line
                errors.append(f"CGM baseline 2^30 P={share}: {e!r}")

    if rank == 0:
        emit(res)
    if sharded:
        dist.destroy_process_group()
    return 0 if verified else 1


if __name__ == "__main__":
    sys.exit(main())
