"""The multi-process sharded path on ONE GPU (KTH_SHARE_GPU=1 test mode).

The driver's N-GPU run launches `bench.py --gpus N` as N rank processes, each
with its own libkth ctx, meeting through a rendezvous and running
kselect.dist.DistSelector(HipBackend) -- the early result, the DistStatus read,
one all-gather and two all-reduces per select.  On the one-GPU pool every part
of that runs here except RCCL's transport: the ranks share GPU 0 and stage the
collectives through host memory over gloo (kselect.rccl.HostComm), as
apps/kth_cgm.c --comm mpi does.  Replaces the reference's launch and
collectives TODO-kth-problem-cgm.c:53-61, :103, :135-190.

* bench.py --gpus 2 with KTH_SHARE_GPU=1 at 2^24 keys per rank: launcher, file
  rendezvous, the timed protocol, the device-side rank certificate; its line
  says it is not a scaling point.
* The reference's golden fixtures split 2 ways by its block partition
  (TODO-kth-problem-cgm.c:81-100): every answer equals the true order
  statistic and every terminating `mpirun -n 2` CGM-ref answer, on both ranks.
"""
import json
import os
import subprocess
import sys
import tempfile

import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _env(extra):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_PORT", "KTH_RDV_FILE")}
    env.update(extra)
    return env


def test_bench_shared_gpu_two_ranks():
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--log2n", "24", "--steps", "3", "--warmup", "1",
                        "--no-cpu-baseline"], cwd=REPO, capture_output=True, text=True, timeout=240,
                       env=_env({"KTH_SHARE_GPU": "1"}), stdin=subprocess.DEVNULL)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout  # rank 0 only
    line = lines[0]
    assert line["verified"] is True, line
    assert line["n_gpus"] == 1 and line["config"]["ranks"] == 2, line
    assert line["config"]["parallelism"] == "shared-gpu-host-comm" and line["config"]["rccl_world"] is None, line
    assert line["scaling_point"] is False and "not a scaling point" in line["note"], line
    assert line["config"]["n_total"] == 2 << 24 and line["config"]["k"] == 1 << 24, line


def _run_workers(world, timeout=240):
    rdv_dir = tempfile.mkdtemp(prefix="kth_rdv_")
    rdv = os.path.join(rdv_dir, "store")
    procs = []
    try:
        for r in range(world):
            env = _env({"RANK": str(r), "WORLD_SIZE": str(world), "KTH_RDV_FILE": rdv})
            procs.append(subprocess.Popen([sys.executable, "-u", os.path.join(HERE, "dist_shared_worker.py")],
                                          env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                                          stdin=subprocess.DEVNULL))
        outs = []
        for p in procs:
            try:
                so, se = p.communicate(timeout=timeout)
            except subprocess.TimeoutExpired:
                for q in procs:
                    q.kill()
                raise
            assert p.returncode == 0, se[-3000:]
            outs.append(json.loads([ln for ln in so.splitlines() if ln.startswith("{")][-1]))
        return {o["rank"]: o for o in outs}
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
        for f in os.listdir(rdv_dir):
            os.unlink(os.path.join(rdv_dir, f))
        os.rmdir(rdv_dir)


def test_shared_gpu_golden_split_p2(golden):
    """Two rank processes on GPU 0: the golden fixtures by the reference's
    block partition (shards under 64 keys take the gather-to-every-rank path),
    then 2^24 + 5 keys of three families, k in {1, n/3, n/2, n}."""
    res = _run_workers(2)
    assert sorted(res) == [0, 1]
    cases = golden["cases"]
    g0, g1 = res[0]["golden"], res[1]["golden"]
    assert len(g0) == len(g1) == len(cases)
    checked_cgm = 0
    for (i, a0, e0), (j, a1, e1) in zip(g0, g1):
        c = cases[i]
        assert i == j and e0 == e1 == 0, (c, e0, e1)
        assert a0 == a1 == c["true"], (c, a0, a1)
        v = c["cgm_ref"].get("2")
        if v is not None and v != "livelock":
            assert a0 == v, (c, a0)
            checked_cgm += 1
    assert checked_cgm > 100  # (57 of the 190 P = 2 reference runs livelock)
    s0, s1 = res[0]["synthetic"], res[1]["synthetic"]
    assert len(s0) == len(s1) == 12
    for (fam, n, k, a0, e0, want), (_, _, _, a1, e1, _) in zip(s0, s1):
        assert e0 == e1 == 0 and a0 == a1 == want, (fam, n, k, a0, a1, want)
