"""bench.py's launch contract (CPU, no GPU needed).

`bench.py --gpus N` must run N ranks: under torchrun (WORLD_SIZE set) it must
agree with WORLD_SIZE, and without a launcher it starts the N rank processes
itself (replacing the reference's `mpirun -n P`, TODO-kth-problem-cgm.c:53-61)
without touching a GPU in the parent.  It must never print a result line for
fewer ranks than asked, and it fails loudly where a GPU is missing.
"""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _run(args, env_extra=None, timeout=180):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_PORT", "KTH_RDV_FILE")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH, *args], capture_output=True, text=True, timeout=timeout, env=env,
                          cwd="/tmp")


@pytest.mark.parametrize("n", [2, 3])
def test_launcher_spawns_n_ranks(n):
    r = _run(["--gpus", str(n), "--probe-launch"])
    assert r.returncode == 0, r.stderr
    ranks = [json.loads(line) for line in r.stdout.splitlines() if line.startswith("{")]
    assert sorted(int(x["RANK"]) for x in ranks) == list(range(n))
    assert {x["WORLD_SIZE"] for x in ranks} == {str(n)}
    assert sorted(int(x["LOCAL_RANK"]) for x in ranks) == list(range(n))
    assert {x["MASTER_ADDR"] for x in ranks} == {"127.0.0.1"}
    # one shared FileStore rendezvous, no probed TCP port (round 4's EADDRINUSE)
    assert {x["MASTER_PORT"] for x in ranks} == {None}
    rdv = {x["KTH_RDV_FILE"] for x in ranks}
    assert len(rdv) == 1 and rdv.pop().startswith("/")
    assert f"launching {n} ranks" in r.stderr


@pytest.mark.parametrize("n", [2, 4])
def test_launcher_rendezvous(n):
    """The ranks launch_ranks starts really meet through its file rendezvous
    (the same init_group the nccl ranks use, on gloo here) and all-reduce."""
    r = _run(["--gpus", str(n), "--probe-rendezvous"])
    assert r.returncode == 0, r.stderr
    out = [json.loads(line) for line in r.stdout.splitlines() if line.startswith("{")]
    assert sorted(x["rank"] for x in out) == list(range(n))
    assert {(x["world"], x["rank_sum"]) for x in out} == {(n, n * (n - 1) // 2)}


def test_world_size_mismatch_refused():
    r = _run(["--gpus", "8", "--probe-launch"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "refusing" in r.stderr
    assert '"n_gpus"' not in r.stdout


def test_torchrun_style_env_accepted():
    r = _run(["--gpus", "2", "--probe-launch"], {"WORLD_SIZE": "2", "RANK": "1", "LOCAL_RANK": "1",
                                                 "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": "29511"})
    assert r.returncode == 0, r.stderr
    assert json.loads(r.stdout.strip())["RANK"] == "1"


def test_no_gpu_fails_loudly():
    """Without a GPU every rank exits non-zero and no result line is printed
    (there is no CPU fallback)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    for gpus in ("1", "2"):
        r = _run(["--gpus", gpus, "--steps", "1", "--warmup", "0", "--no-cpu-baseline"])
        assert r.returncode != 0
        assert "no CPU fallback" in r.stderr
        assert '"metric"' not in r.stdout
