"""GPU tests of the sharded paths on the one-GPU box.

* kth_select_i32_sharded / kth_sharded_* (single process, RCCL communicators from
  ncclCommInitAll; include/kth.h) at ngpu = 1: golden reference fixtures and
  synthetic families against the oracle's order statistic.
* The gloo tests' CPU restatement of the per-rank steps (tests/dist_cpu_backend.py)
  against the device steps (kth_dist_* through kselect.dist.HipBackend) at world
  1: identical samples and identical stats slots after the scan and every level,
  so the multi-rank gloo runs exercise the arithmetic a GPU run performs.
"""
import numpy as np
import pytest

from conftest import load_input

pytestmark = pytest.mark.gpu

FAMS = ["uniform_full", "uniform_half", "few_distinct", "all_equal", "sorted_desc", "mod_1000"]


def _dev_keys(gpu, n, fam, param=7):
    import torch
    keys = torch.empty(n, dtype=torch.int32, device="cuda")
    gpu.fill(keys, n, fam, param=param)
    gpu.sync()
    return keys


@pytest.fixture(scope="module")
def sharded():
    import kselect
    s = kselect.ShardedSelector([0])
    yield s
    s.close()


def test_sharded_golden(sharded, golden):
    """Reference-generated fixtures (seq and mpirun CGM outputs): n <= 16384 --
    shards under 64 keys take the gather-to-device-0 path, the rest the protocol."""
    import torch
    for c in golden["cases"]:
        a = torch.from_numpy(load_input(c["input"])).cuda()
        got = sharded.select([a], c["k"])
        assert got == c["true"], c
        for p, v in c["cgm_ref"].items():
            if v != "livelock":
                assert got == v, (c, p)


@pytest.mark.parametrize("n", [(1 << 20) + 3, (1 << 24) + 5])
def test_sharded_families(gpu, sharded, n):
    import kselect
    for fam in FAMS:
        keys = _dev_keys(gpu, n, fam)
        srt = np.sort(keys.cpu().numpy())
        for k in (1, n // 3, n // 2, n):
            assert sharded.select([keys], k) == srt[k - 1], (fam, n, k)
            assert kselect.select_sharded([keys], k) == srt[k - 1], (fam, n, k)


def test_sharded_errors(gpu, sharded):
    import kselect
    import torch
    keys = torch.zeros(1000, dtype=torch.int32, device="cuda")
    for k in (0, 1001):
        with pytest.raises(kselect.KthError) as e:
            sharded.select([keys], k)
        assert e.value.code == kselect.KTH_EINVAL
    with pytest.raises(kselect.KthError) as e:  # host memory is not a shard
        kselect.select_sharded([np.zeros(1000, dtype=np.int32)], 5)
    assert e.value.code == kselect.KTH_EINVAL
    with pytest.raises(kselect.KthError) as e:  # one rank per device
        kselect.ShardedSelector([0, 0])
    assert e.value.code == kselect.KTH_EINVAL


@pytest.mark.parametrize("fam", FAMS)
def test_dist_backend_slots_match(gpu, fam):
    """HipBackend (device) and CpuBackend (the gloo tests' restatement) step by
    step on the same shard at world 1: same sample, same slots, same answer."""
    import torch
    from dist_cpu_backend import CpuBackend
    from kselect.dist import HipBackend
    n = (1 << 23) + 77
    keys = _dev_keys(gpu, n, fam)
    host = keys.cpu()
    hb, cb = HipBackend(0, gpu), CpuBackend()
    s = max(64, (hb.sample_size(n) // 1) & ~63)
    assert s == max(64, (cb.sample_size(n) // 1) & ~63)
    for k in (1, n // 2, n):
        sg, sc = hb.alloc_slots(), cb.alloc_slots()
        hb.begin(sg, n, k)
        cb.begin(sc, n, k)
        smp_g, smp_c = hb.alloc_sample(s), cb.alloc_sample(s)
        hb.sample(keys, n, smp_g, s)
        cb.sample(host, n, smp_c, s)
        torch.cuda.synchronize()
        assert torch.equal(smp_g.cpu(), smp_c), (fam, k, "sample")
        hb.window(smp_g, s)
        cb.window(smp_c, s)
        i, j = hb.scan(keys, n), cb.scan(host, n)
        torch.cuda.synchronize()
        assert i == j and torch.equal(sg[i].cpu(), sc[j]), (fam, k, "scan", sg[i][:5].tolist(), sc[j][:5].tolist())
        for level in range(3):
            i, j = hb.level(keys, n, level), cb.level(host, n, level)
            torch.cuda.synchronize()
            assert i == j and torch.equal(sg[i].cpu(), sc[j]), (fam, k, "level", level)
        og, oc = hb.alloc_out(), cb.alloc_out()
        hb.result(og)
        cb.result(oc)
        torch.cuda.synchronize()
        assert int(og.item()) == int(oc.item()) == int(np.sort(host.numpy())[k - 1]), (fam, k)
