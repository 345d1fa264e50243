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
* The reference's golden fixtures split 2 and 3 ways by its block partition
  (TODO-kth-problem-cgm.c:81-100): every answer equals the true order
  statistic and every terminating `mpirun -n 2` / `-n 3` CGM-ref answer, on
  every rank.
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


@pytest.mark.parametrize("world", [2, 3])
def test_shared_gpu_golden_split(golden, world):
    """world rank processes on GPU 0: the golden fixtures by the reference's
    block partition (shards under 64 keys take the gather-to-every-rank path),
    every answer equal on every rank, to the true value and to every
    terminating `mpirun -n world` CGM-ref run; then 2^24 + 5 keys of three
    families (uneven shards at world 3), k in {1, n/3, n/2, n}."""
    res = _run_workers(world)
    assert sorted(res) == list(range(world))
    cases = golden["cases"]
    gs = [res[r]["golden"] for r in range(world)]
    assert all(len(g) == len(cases) for g in gs)
    checked_cgm = 0
    for rows in zip(*gs):
        i = rows[0][0]
        c = cases[i]
        assert all(r[0] == i and r[2] == 0 for r in rows), (c, rows)
        assert {r[1] for r in rows} == {c["true"]}, (c, rows)
        v = c["cgm_ref"].get(str(world))
        if v is not None and v != "livelock":
            assert rows[0][1] == v, (c, rows[0][1])
            checked_cgm += 1
    assert checked_cgm > 100  # (57 of the 190 P = 2 reference runs livelock)
    ss = [res[r]["synthetic"] for r in range(world)]
    assert all(len(x) == 12 for x in ss)
    for rows in zip(*ss):
        fam, n, k, _, _, want = rows[0]
        assert all(r[4] == 0 and r[3] == want for r in rows), (fam, n, k, rows)
