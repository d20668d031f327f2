"""Deferred split-K gradient sums (parallel/flat.py): the partial lookup and the non-deferred fallback, on CPU (the
reduce itself is a GPU kernel: tests/test_graph_gpu.py::test_deferred_split_sums_match_immediate_sums)."""
import pytest
import torch

from pytorch_rt1_for_distributed_training_amd.parallel import flat


@pytest.fixture(autouse=True)
def _clean():
    flat._PENDING.clear()
    flat._BASES.clear()
    yield
    flat._PENDING.clear()
    flat._BASES.clear()


def test_defer_partials_sums_when_not_deferred():
    part = torch.randn(5, 3, 4)
    torch.testing.assert_close(flat.defer_partials(part), part.sum(0))
    with flat.deferred_sums():          # CPU partials are never deferred
        torch.testing.assert_close(flat.defer_partials(part), part.sum(0))
    assert not flat._PENDING
    one = torch.randn(1, 3, 4)
    assert flat.defer_partials(one).data_ptr() == one.data_ptr()


def test_pending_lookup_finds_row_slices_of_a_first_split():
    parts = [torch.zeros(4, 6, 8), torch.zeros(2, 5, 8)]
    for p in parts:
        g = p[0]
        flat._PENDING[g.data_ptr()] = [p, g.numel() * 4, g.numel() * 4]
    g0 = parts[0][0]
    base, splits, stride = flat._pending_of(g0[2:4])
    assert (base, splits, stride) == (g0.data_ptr(), 4, 48)
    assert flat._pending_of(parts[1][0][1:3])[1:] == (2, 40)
    assert flat._pending_of(parts[0][1]) is None          # the second split itself is no gradient
    assert flat._pending_of(torch.zeros(6, 8)) is None
    with pytest.raises(RuntimeError, match="straddles"):
        flat._pending_of(parts[0].view(-1)[40:60])


def test_deferred_sums_context_nests():
    assert flat._DEFER[0] == 0
    with flat.deferred_sums():
        with flat.deferred_sums(enabled=False):
            assert flat._DEFER[0] == 1
        with flat.deferred_sums():
            assert flat._DEFER[0] == 2
    assert flat._DEFER[0] == 0
