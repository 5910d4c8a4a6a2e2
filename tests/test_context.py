"""Context selection follows the data's device (no GPU needed): a decoder or
encoder given a tensor on cuda:1 uses device 1's context, and an explicit
context on another device than the tensor is an argument error -- the
multi-rank bench must never decode one rank's chunk on another rank's GPU."""
from types import SimpleNamespace

import pytest

import pa_amd
from pa_amd import read as R


class FakeCtx:
    def __init__(self, device):
        self.device = device


def fake_tensor(dev):
    return SimpleNamespace(is_cuda=True, device=SimpleNamespace(index=dev))


def test_default_context_follows_tensor_device(monkeypatch):
    made = {}
    monkeypatch.setattr(R, "_default_ctx", made)
    monkeypatch.setattr(R, "Context", FakeCtx)
    c1 = R.resolve_context(None, fake_tensor(1))
    c0 = R.resolve_context(None, fake_tensor(0))
    assert (c1.device, c0.device) == (1, 0)
    assert R.resolve_context(None, fake_tensor(1)) is c1  # one shared context per device
    assert R.resolve_context(c1, fake_tensor(1)) is c1


def test_context_device_mismatch_is_an_error():
    with pytest.raises(pa_amd.StrawboatError) as e:
        R.resolve_context(FakeCtx(0), fake_tensor(3))
    assert e.value.status == pa_amd._native.E_ARG
