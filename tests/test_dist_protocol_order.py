"""The per-rank protocol's call order on CPU (kselect.dist.DistSelector.steps,
run in lockstep over P CPU backends): the optional early result is queued
right after level 0's all-reduce and before level 1 looks at level 0's status,
the closing result comes last, and the answers stay exact.  The device side
of kth_dist_result_early (a no-op unless level 0 was the last) is covered by
the GPU lockstep tests of test_gpu_config3.py."""
import os
import sys

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

from conftest import PKG  # noqa: E402,F401 -- sets sys.path for kselect
from dist_cpu_backend import CpuBackend  # noqa: E402
from kselect.dist import DistSelector, lockstep  # noqa: E402


class RecordingBackend(CpuBackend):
    """The CPU restatement, recording the protocol calls it sees; with
    early=True it offers result_early (a recorded no-op, as on the device
    when a later level follows)."""

    def __init__(self, log, early):
        super().__init__()
        self.log = log
        if early:
            self.result_early = lambda out: self.log.append("result_early")

    def begin(self, *a):
        self.log.append("begin")
        return super().begin(*a)

    def level(self, shard, n_local, level):
        self.log.append(f"level{level}")
        return super().level(shard, n_local, level)

    def result(self, out):
        self.log.append("result")
        return super().result(out)


@pytest.mark.parametrize("early", [True, False])
@pytest.mark.parametrize("fam", ["uniform", "few", "wide"])
def test_early_result_order_and_answers(early, fam, monkeypatch):
    monkeypatch.setenv("KTH_DIST_EARLY", "1")
    rng = np.random.default_rng(7)
    P, n_local = 2, 1 << 16
    if fam == "uniform":
        a = rng.integers(-2 ** 30, 2 ** 30, P * n_local, dtype=np.int64)
    elif fam == "few":
        a = rng.integers(0, 4, P * n_local, dtype=np.int64)
    else:  # full int32 range: windows wider than 2^24 values take more levels
        a = rng.integers(-2 ** 31, 2 ** 31, P * n_local, dtype=np.int64)
    a = a.astype(np.int32)
    shards = [torch.from_numpy(a[i * n_local:(i + 1) * n_local].copy()) for i in range(P)]
    srt = np.sort(a)
    for k in (1, P * n_local // 2, P * n_local):
        logs = [[] for _ in range(P)]
        sels = [DistSelector(RecordingBackend(logs[i], early), world=P) for i in range(P)]
        outs = lockstep(sels, shards, [n_local] * P, k)
        assert all(int(o.reshape(-1)[0]) == int(srt[k - 1]) for o in outs), (fam, k)
        for log in logs:
            assert log[0] == "begin" and log[-1] == "result", log
            assert ("result_early" in log) == early, log
            if early:
                i = log.index("result_early")
                assert log[i - 1] == "level0" and log[i + 1] == "level1", log
            assert log.count("result") == 1


def test_early_result_switch(monkeypatch):
    """KTH_DIST_EARLY=0 leaves the early result out even when the backend has it."""
    monkeypatch.setenv("KTH_DIST_EARLY", "0")
    P, n_local = 2, 1 << 12
    a = np.arange(P * n_local, dtype=np.int32)[::-1].copy()
    shards = [torch.from_numpy(a[i * n_local:(i + 1) * n_local].copy()) for i in range(P)]
    logs = [[] for _ in range(P)]
    sels = [DistSelector(RecordingBackend(logs[i], True), world=P) for i in range(P)]
    outs = lockstep(sels, shards, [n_local] * P, 5)
    assert all(int(o.reshape(-1)[0]) == 4 for o in outs)
    assert all("result_early" not in log for log in logs)
