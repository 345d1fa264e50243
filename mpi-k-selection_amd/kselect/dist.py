"""Sharded exact k-th selection, one process per GPU.

Replaces the CGM driver of the reference (TODO-kth-problem-cgm.c:76-278):

  reference (per round, ~10-12 rounds)           here (once per selection)
  -------------------------------------          -----------------------------------
  :103 MPI_Scatterv of 4n bytes from rank 0      shards already resident per GPU
  :115 local qsort (88% of CGM time)             --
  :125-131 local median                          local sample (chunks of kth_sample_chunk() keys)
  :135-136 2x MPI_Gather (median, n_i)           all_gather of the samples
  :139-165 weighted median on rank 0             every rank derives the same window
  :168 MPI_Bcast of the pivot                    -- (deterministic, no broadcast)
  :171-185 3-way count L/E/G                     ONE streaming pass per shard
  :190 MPI_Allreduce(3 ints)                     all_reduce of the counts
  :194-225 discard via VecErase                  local candidate compaction
  :242-270 Gather sizes + Barrier + Gatherv      the counts' all_reduce carries the candidates'
  :277-278 rank-0 qsort + VecGet(k-1)            first 12-bit digit; one more all_reduce for the
                                                 second (windows <= 2^24 values wide)

Every rank ends with the same answer (the reference prints it on rank 0 only).
On GPUs the collectives go through a direct RCCL communicator on the
selector's own stream (kselect.rccl: torch's ProcessGroupNCCL would fence every
collective with a hop to its internal stream), so enqueueing them never makes
the host wait.  The host waits ONCE per selection: kth_dist_level(1) waits for
level 0's kernel to learn from its DistStatus how many levels follow (by then
the device has the second all-reduce, and with the early result the usual last
step, queued behind it); the protocol is a loop over kth_dist_level until it
returns KTH_DIST_DONE (at most KTH_DIST_MAX_LEVELS slots).  Ranks that share
one GPU (KTH_SHARE_GPU=1, tests) stage the collectives through host memory over
gloo (kselect.rccl.HostComm); CPU tests use torch.distributed ops directly.
The per-rank device work is a ``backend``: ``HipBackend`` (libkth.so) in the
product; tests plug in a CPU restatement to exercise this orchestration on gloo.
"""
import os

import torch
import torch.distributed as dist

from . import KTH_DIST_DONE, KTH_DIST_MAX_LEVELS, KTH_EINTERNAL, KTH_STATS_WORDS, LIB as _lib, KthError, Selector, check, \
    check_single_runtime
from .rccl import HostComm, RcclComm, TorchComm

SMALL_PER_RANK = 64  # below this many keys per rank: all-gather and select locally


def shard_bounds(n, rank, world):
    """Block partition of TODO-kth-problem-cgm.c:81-100: sizev[i] = n/P + (i < n%P)."""
    size, rem = divmod(n, world)
    start = rank * size + min(rank, rem)
    return start, size + (1 if rank < rem else 0)


class HipBackend:
    """Per-rank device steps through the kth_dist_* entry points of libkth.so."""

    def __init__(self, device, selector=None):
        check_single_runtime()  # torch's streams and RCCL must share libkth.so's HIP runtime
        self.device = torch.device("cuda", device)
        self.sel = selector or Selector(device)
        self.stream = torch.cuda.current_stream(self.device)
        self.sel.set_stream(self.stream)
        self.ctx = self.sel.handle

    def make_comm(self, group=None):
        """RCCL on this backend's stream for an "nccl" group (KTH_DIST_COMM=torch
        forces torch.distributed collectives instead); a CPU (gloo) group --
        ranks sharing one GPU -- stages the device tensors through host memory."""
        if dist.get_backend(group) != "nccl":
            return HostComm(group)
        if os.environ.get("KTH_DIST_COMM", "rccl") != "torch":
            return RcclComm(self.device.index, self.stream, group)
        return TorchComm(group)

    def sample_size(self, n_local):
        return int(_lib.kth_dist_sample_size(int(n_local)))

    def alloc_slots(self):
        return torch.zeros((3, KTH_STATS_WORDS), dtype=torch.int64, device=self.device)

    def alloc_sample(self, s):
        return torch.empty(s, dtype=torch.int32, device=self.device)

    def begin(self, slots, n_total, k):
        check(_lib.kth_dist_begin(self.ctx, slots.data_ptr(), int(n_total), int(k)), "kth_dist_begin")

    def sample(self, shard, n_local, out, s_local):
        check(_lib.kth_dist_sample(self.ctx, shard.data_ptr(), int(n_local), out.data_ptr(), int(s_local)),
              "kth_dist_sample")

    def window(self, sample_all, s_total):
        check(_lib.kth_dist_window(self.ctx, sample_all.data_ptr(), int(s_total)), "kth_dist_window")

    def scan(self, shard, n_local):
        r = _lib.kth_dist_scan(self.ctx, shard.data_ptr(), int(n_local))
        if r < 0:
            check(r, "kth_dist_scan")
        return r

    def level(self, shard, n_local, level):
        r = _lib.kth_dist_level(self.ctx, shard.data_ptr(), int(n_local), int(level))
        if r < 0:
            check(r, "kth_dist_level")
        return r

    def result(self, out):
        check(_lib.kth_dist_result(self.ctx, out.data_ptr()), "kth_dist_result")

    def select_rccl(self, comm, shard, n_local, n_total, k, slots, sample, gathered, s_local, out, early):
        """The whole protocol in one call over an RcclComm (kth_dist_select_rccl)."""
        c, ar, ag = comm.entry_points()
        r = _lib.kth_dist_select_rccl(self.ctx, ar, ag, c, comm.world, shard.data_ptr(), n_local, n_total, k,
                                      slots.data_ptr(), sample.data_ptr(), gathered.data_ptr(), s_local,
                                      out.data_ptr(), early)
        if r:
            check(r, "kth_dist_select_rccl")

    def result_early(self, out):
        """The result enqueued before level 1 looks at level 0's status (a
        no-op on the device unless level 0 was the last); result() closes."""
        check(_lib.kth_dist_result_early(self.ctx, out.data_ptr()), "kth_dist_result_early")

    def alloc_out(self):
        return torch.empty(1, dtype=torch.int32, device=self.device)

    def error(self):
        """The last selection's device error word (kth_ctx_last_stats; synchronises)."""
        return int(self.sel.stats()["error"])

    def select_all(self, keys, n, k, out):
        """k-th smallest of keys[0..n) on this GPU (the small-input path)."""
        self.sel.select_async(keys, n, k, out)


class DistSelector:
    """k-th smallest of the union of every rank's shard (global 1-based k)."""

    def __init__(self, backend, group=None, comm=None, world=None):
        self.b = backend
        self.group = group
        self.world = dist.get_world_size(group) if world is None else int(world)
        if comm is None and world is None:
            comm = backend.make_comm(group) if hasattr(backend, "make_comm") else TorchComm(group)
        self.comm = comm
        self.slots = backend.alloc_slots()
        self.out = backend.alloc_out()
        self._sample = None
        self._gathered = None
        self._checked = None  # last (n_local, n_total, k) every rank agreed on
        self._s_local_for, self._s_local, self._sample_n = None, 0, -1
        self._one_call, self._early = None, 1  # (decided at the first select)

    def s_local(self, n_total):
        """Sample keys per rank: the window needs ~sample_size(n_total) keys in
        all (what one GPU would take), not that many per rank, so the
        all-gather stays ~4 MiB.  (Cached per n_total: the host's path between
        two selects is what the device waits on when a select is short.)"""
        if self._s_local_for != n_total:
            self._s_local = max(64, (self.b.sample_size(n_total) // self.world) & ~63)
            self._s_local_for = n_total
        return self._s_local

    def steps(self, shard, n_local, n_total, k, out):
        """The per-rank protocol as a generator: the device steps run in the
        generator, each collective is yielded to the caller, who performs it
        across the ranks before resuming -- ("all_gather", dst, src) or
        ("all_reduce", t), SUM in place (select() runs them over self.comm;
        lockstep() performs them for P selectors in one process)."""
        b = self.b
        s_local = self.s_local(n_total)
        if self._sample is None or self._sample_n != s_local:
            self._sample = b.alloc_sample(s_local)
            self._gathered = b.alloc_sample(s_local * self.world)
            self._sample_n = s_local
        b.begin(self.slots, n_total, k)
        b.sample(shard, n_local, self._sample, s_local)
        yield ("all_gather", self._gathered, self._sample)
        b.window(self._gathered, s_local * self.world)
        i = b.scan(shard, n_local)  # counts + the candidates' first digit
        yield ("all_reduce", self.slots[i])
        for level in range(KTH_DIST_MAX_LEVELS + 1):  # usually one level: two all-reduces in all
            if level == 1 and hasattr(b, "result_early") and os.environ.get("KTH_DIST_EARLY", "1") != "0":
                # before level 1 waits for level 0's status on the host, so the
                # device runs the (usual) last step right after the all-reduce
                b.result_early(out)
            i = b.level(shard, n_local, level)
            if i == KTH_DIST_DONE:
                break
            yield ("all_reduce", self.slots[i])
        else:
            raise KthError(KTH_EINTERNAL, "kth_dist_level never returned KTH_DIST_DONE")
        b.result(out)

    def select(self, shard, n_local, n_total, k, out=None):
        """Enqueue one selection; returns the device (or CPU, for gloo) int32[1]
        answer tensor (``out`` if given, else a buffer reused by every call).
        Asynchronous: a device-side failure (e.g. a timed-out grid barrier)
        leaves ``out`` unwritten -- ``error()`` / ``value()`` report it.

        n_total must be the sum of n_local over ranks and k in [1, n_total];
        every rank must pass the same (n_total, k).  Shards are expected to be
        balanced (every n_local >= n_total // world, as the block partition of
        shard_bounds gives); below SMALL_PER_RANK keys per rank the shards are
        all-gathered and every rank selects from the union."""
        out = self.out if out is None else out
        if self.comm is None:
            raise RuntimeError("this DistSelector was built for lockstep() (world=P, no communicator); "
                               "select() needs a process group")
        if n_total // self.world < SMALL_PER_RANK:
            if not (1 <= k <= n_total):
                raise ValueError(f"k={k} outside [1, {n_total}]")
            return self._select_small(shard, n_local, n_total, k, out)
        if self._checked != (n_local, n_total, k):
            self._check_args(n_local, n_total, k, self.s_local(n_total))
        if self._one_call is None:
            # over RCCL: every step and collective in one library call (the
            # host's per-step round trips through the bindings are ~35 us a
            # select); KTH_DIST_PY=1 keeps the scripted steps
            self._one_call = (isinstance(self.comm, RcclComm) and hasattr(self.b, "select_rccl")
                              and os.environ.get("KTH_DIST_PY") != "1")
            self._early = 1 if os.environ.get("KTH_DIST_EARLY", "1") != "0" else 0
        if self._one_call:
            s_local = self.s_local(n_total)
            if self._sample_n != s_local:
                self._sample = self.b.alloc_sample(s_local)
                self._gathered = self.b.alloc_sample(s_local * self.world)
                self._sample_n = s_local
            self.b.select_rccl(self.comm, shard, n_local, n_total, k, self.slots, self._sample, self._gathered,
                               s_local, out, self._early)
            return out
        for op in self.steps(shard, n_local, n_total, k, out):
            if op[0] == "all_gather":
                self.comm.all_gather(op[1], op[2])
            else:
                self.comm.all_reduce_sum_(op[1])
        return out

    def error(self):
        """The device error word of this rank's last selection (0 = none;
        synchronises).  A nonzero word means the answer tensor was NOT written."""
        return self.b.error() if hasattr(self.b, "error") else 0

    def value(self, shard, n_local, n_total, k):
        """select() + wait: the answer as an int, KthError(KTH_EINTERNAL) when
        the device reports an error (the answer buffer would hold a stale value)."""
        out = self.select(shard, n_local, n_total, k)
        err = self.error()
        if err:
            raise KthError(KTH_EINTERNAL, f"sharded select: device error {err}")
        return int(out.item())

    def _coll_device(self):
        """Where this group's own torch.distributed collectives take tensors:
        host memory for a CPU (gloo) group, else the answer's device."""
        return torch.device("cpu") if dist.get_backend(self.group) == "gloo" else self.out.device

    def _check_args(self, n_local, n_total, k, s_local):
        """Validate the arguments across ranks (two small collectives, once per
        distinct (n_local, n_total, k)), so that every rank raises together
        instead of one rank raising while the others wait in a collective."""
        dev = self._coll_device()
        mx = torch.tensor([n_total, -n_total, k, -k, 0 if n_local >= s_local else 1], dtype=torch.int64, device=dev)
        dist.all_reduce(mx, op=dist.ReduceOp.MAX, group=self.group)
        tot = torch.tensor([n_local], dtype=torch.int64, device=dev)
        dist.all_reduce(tot, op=dist.ReduceOp.SUM, group=self.group)
        mx, tot = mx.tolist(), int(tot.item())
        if mx[0] != -mx[1] or mx[2] != -mx[3]:
            raise ValueError(f"ranks disagree on n_total / k (n_total in [{-mx[1]}, {mx[0]}], "
                             f"k in [{-mx[3]}, {mx[2]}])")
        if tot != n_total:
            raise ValueError(f"shard sizes sum to {tot}, not n_total={n_total}")
        if not (1 <= k <= n_total):
            raise ValueError(f"k={k} outside [1, {n_total}]")
        if mx[4]:
            raise ValueError(f"some shard is smaller than the per-rank sample ({s_local} keys); "
                             "use balanced shards (kselect.dist.shard_bounds)")
        self._checked = (n_local, n_total, k)

    def _select_small(self, shard, n_local, n_total, k, out):
        """Tiny inputs (cf. the reference's final Gatherv + solve on one rank,
        TODO-kth-problem-cgm.c:235-278): all-gather the shards, select locally."""
        dev = self._coll_device()
        sizes = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(self.world)]
        dist.all_gather(sizes, torch.tensor([n_local], dtype=torch.int64, device=dev), group=self.group)
        sizes = [int(x.item()) for x in sizes]
        if sum(sizes) != n_total:
            raise ValueError(f"shard sizes {sizes} do not sum to n_total={n_total}")
        m = max(sizes)
        padded = torch.zeros(m, dtype=torch.int32, device=dev)
        padded[:n_local] = shard[:n_local]
        gathered = torch.empty(m * self.world, dtype=torch.int32, device=dev)
        dist.all_gather_into_tensor(gathered, padded, group=self.group)
        union = torch.cat([gathered[r * m:r * m + sizes[r]] for r in range(self.world)])
        self.b.select_all(union.to(self.out.device), n_total, k, out)
        return out

    def close(self):
        if self.comm is not None:  # (lockstep selectors have none)
            self.comm.close()


def lockstep(selectors, shards, n_locals, k, outs=None, observe=None):
    """P selectors of one process, one shard each, run the protocol in
    lockstep: every selector's steps up to its next collective, then the
    collective performed here -- the all-gather as a concatenation of the P
    samples, the all-reduce as the SUM of the P slots written back to each.
    The Python mirror of kth_sharded's local transport (P shards on one
    device; also P CPU backends in tests).  Returns the P answer tensors.
    ``observe(kind, tensors)`` sees every collective's result."""
    P = len(selectors)
    if not (len(shards) == len(n_locals) == P) or P < 1:
        raise ValueError("one shard and one size per selector")
    n_total = int(sum(int(n) for n in n_locals))
    if not (1 <= k <= n_total):
        raise ValueError(f"k={k} outside [1, {n_total}]")
    if any(s.world != P for s in selectors):
        raise ValueError(f"selectors built for world {[s.world for s in selectors]}, lockstep runs {P}")
    s_local = selectors[0].s_local(n_total)
    if min(int(n) for n in n_locals) < s_local:
        raise ValueError(f"some shard is smaller than the per-rank sample ({s_local} keys)")
    outs = [s.out for s in selectors] if outs is None else outs
    gens = [s.steps(sh, int(n), n_total, k, o) for s, sh, n, o in zip(selectors, shards, n_locals, outs)]
    while True:
        ops = [next(g, None) for g in gens]
        if all(op is None for op in ops):
            return outs
        if any(op is None for op in ops) or len({op[0] for op in ops}) != 1:
            raise RuntimeError(f"selectors out of step: {[op and op[0] for op in ops]}")
        if ops[0][0] == "all_gather":
            cat = torch.cat([op[2] for op in ops])
            for op in ops:
                op[1].copy_(cat)
            res = cat
        else:
            total = ops[0][1].clone()
            for op in ops[1:]:
                total += op[1]
            for op in ops:
                op[1].copy_(total)
            res = total
        if observe:
            observe(ops[0][0], res)
