"""Host logic of the batched sweep: the batch handle shrinks its
configuration count while the device refuses the buffers (ADVICE r02:
G was clamped only by the grid limit, so large n or B aborted the sweep)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mpc-mmd_amd")]

from optimizer import _native, sweep  # noqa: E402


class _Prob:
    _cfg = object()


def test_batch_handle_halves_until_created(monkeypatch):
    tried = []

    def fake_handle(cfg, max_configs=1):
        tried.append(max_configs)
        if max_configs > 5:
            raise _native.NativeError("libmpcmmd error -5: hipMalloc: out of memory")
        return ("handle", max_configs)

    monkeypatch.setattr(_native, "Handle", fake_handle)
    assert sweep.batch_handle(_Prob(), 32) == ("handle", 4)
    assert tried == [32, 16, 8, 4]


def test_batch_handle_gives_up_at_one(monkeypatch):
    def refuse(cfg, max_configs=1):
        raise _native.NativeError("libmpcmmd error -5: hipMalloc: out of memory")

    monkeypatch.setattr(_native, "Handle", refuse)
    try:
        sweep.batch_handle(_Prob(), 8)
    except _native.NativeError:
        return
    raise AssertionError("a refused single-configuration handle must raise")
