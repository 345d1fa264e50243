"""The sequential drop-in driver (apps/kth_seq.c): the reference's generator
(kth-problem-seq.c:23-28, seeded), the select block through VecKthSelectEx, and
the reference's output line "Solution found solution=%d \\ntime: %f\\n" (:37).

CPU: the binary fails loudly without a GPU.  GPU: its answer equals the true
order statistic of the regenerated input (oracle/ko_gen_shipped_seq, pinned to
the shipped program's own input stream in test_oracle_golden.py)."""
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import PKG

BIN = os.path.join(os.environ.get("KTH_BIN_DIR") or os.path.join(PKG, "bin"), "kth_seq")
OUT = re.compile(r"Solution found solution=(-?\d+) \ntime: ([0-9.]+)\n")


def _run(*args):
    return subprocess.run([BIN, *map(str, args)], capture_output=True, text=True, timeout=300,
                          stdin=subprocess.DEVNULL)


def test_seq_driver_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    r = _run(1000, 10, 1)
    assert r.returncode != 0 and not OUT.search(r.stdout)
    assert "no HIP device" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("n,k", [(1000, 250), ((1 << 20) + 3, 250), ((1 << 20) + 3, 0), ((1 << 22) + 1, 0)])
def test_seq_driver_output_line(oracle, n, k):
    seed = 4242
    args = [n, k, seed] if k else [n, 0, seed, "--median"]
    r = _run(*args)
    assert r.returncode == 0, r.stderr
    m = OUT.search(r.stdout)
    assert m, r.stdout
    a = np.empty(n, dtype=np.int32)
    oracle.ko_gen_shipped_seq(a.ctypes.data, n, seed)
    kk = k or n // 2
    assert int(m.group(1)) == int(np.partition(a, kk - 1)[kk - 1])
