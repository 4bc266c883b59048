"""Philox4x32-10 against the Random123 known-answer vectors (torch path) and the HIP device version."""
import pytest
import torch

from mat_dcml_amd.utils import philox as px

KAT = [
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 4, (0xFFFFFFFF, 0xFFFFFFFF), (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]


@pytest.mark.parametrize("ctr,key,expect", KAT)
def test_known_answers(ctr, key, expect):
    out = px.philox4x32(torch.tensor([ctr[0]]), ctr[1], ctr[2], ctr[3], key[0], key[1])
    assert tuple(int(o[0]) for o in out) == expect


def test_uniform_range_and_moments():
    u = px.philox4x32(torch.arange(200000), 7, 3, 1, 11, 13)[0]
    x = px.u01_open(u)
    assert float(x.min()) > 0 and float(x.max()) < 1
    assert abs(float(x.mean()) - 0.5) < 5e-3
    assert abs(float(x.var()) - 1 / 12) < 2e-3


@pytest.mark.gpu
def test_device_philox_matches_torch(gpu):
    from mat_dcml_amd.ops import kernels
    c0 = torch.arange(4096, dtype=torch.int64)
    ref = torch.stack(px.philox4x32(c0, 5, 9, 3, 123, 456), -1)
    dev = kernels.philox_fill(4096, 5, 9, 3, 123, 456, gpu).cpu()
    assert torch.equal(dev, ref)


def test_feistel_randperm_reference_is_a_permutation():
    """utils/philox.feistel_randperm (the reference of the HIP minibatch shuffle): a bijection of [0, n) for awkward
    n, key-dependent, far from the identity."""
    from mat_dcml_amd.utils.philox import feistel_randperm
    for n in (1, 2, 3, 5, 64, 1000, 12800):
        p = feistel_randperm(n, 7, 11)
        assert torch.equal(torch.sort(p).values, torch.arange(n)), n
    a, b = feistel_randperm(12800, 7, 11), feistel_randperm(12800, 8, 11)
    assert not torch.equal(a, b)
    assert (a == torch.arange(12800)).float().mean() < 0.01
