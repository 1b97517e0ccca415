"""CPU: the invalidation rules of the two parameter-derived caches of round 5,
with the C-ABI calls stubbed (no GPU here; tests/test_eval_cache_gpu.py and
tests/test_bwd_colmax_gpu.py run them for real):

* gfd.fused.eval_weights -- a layer's packed weights (and BatchNorm affine) are
  rebuilt exactly when a source tensor is replaced, updated in place, given new
  storage, or the BatchNorm module / device changes;
* gfd.nn.x_colmax -- the per-column maxima of x, per tensor object and version.
"""
import torch

from gfd import _lib, fused, nn as gnn


class _Stub:
    """_lib.load() / _lib.call stand-in that counts calls by name."""

    def __init__(self):
        self.calls = []

    def gfd_gat_packed_size(self, F, H, C):
        return 64

    def call(self, name, *args):
        self.calls.append(name)
        return 0


def _patch(monkeypatch):
    stub = _Stub()
    monkeypatch.setattr(_lib, "load", lambda: stub)
    monkeypatch.setattr(_lib, "call", stub.call)
    monkeypatch.setattr(_lib, "stream_handle", lambda device=None: 0)
    monkeypatch.setattr(_lib, "x_dtype_code", lambda x: 0)
    return stub


def test_eval_weights_rebuilds_exactly_when_a_source_changes(monkeypatch):
    stub = _patch(monkeypatch)
    conv = gnn.GATConv(16, 64, heads=8, concat=False)
    bn = torch.nn.BatchNorm1d(64).eval()
    dev = torch.device("cpu")
    p1, a1 = fused.eval_weights(conv, bn, dev)
    p2, a2 = fused.eval_weights(conv, bn, dev)
    assert p2 is p1 and a2 is a1 and stub.calls.count("gfd_gat_pack_weights") == 1
    with torch.no_grad():
        conv.att_dst.add_(0.1)                                   # in-place update
    p3, _ = fused.eval_weights(conv, bn, dev)
    assert p3 is not p1 and stub.calls.count("gfd_gat_pack_weights") == 2
    bn.running_var.mul_(2.0)                                     # new statistics
    _, a4 = fused.eval_weights(conv, bn, dev)
    assert a4 is not a1 and stub.calls.count("gfd_gat_pack_weights") == 3
    conv.lin_src.weight = torch.nn.Parameter(conv.lin_src.weight.detach().clone())  # new object
    fused.eval_weights(conv, bn, dev)
    assert stub.calls.count("gfd_gat_pack_weights") == 4
    conv.att_src.data = conv.att_src.data.clone()                # same object, new storage
    fused.eval_weights(conv, bn, dev)
    assert stub.calls.count("gfd_gat_pack_weights") == 5
    fused.eval_weights(conv, torch.nn.BatchNorm1d(64).eval(), dev)   # another BatchNorm
    assert stub.calls.count("gfd_gat_pack_weights") == 6
    fused.eval_weights(conv, None, dev)                              # none
    fused.eval_weights(conv, None, dev)
    assert stub.calls.count("gfd_gat_pack_weights") == 7


def test_x_colmax_is_kept_per_tensor_object_and_version(monkeypatch):
    stub = _patch(monkeypatch)
    gnn._COLMAX.clear()
    x = torch.randn(10, 7)
    a = gnn.x_colmax(x)
    assert gnn.x_colmax(x) is a and stub.calls.count("gfd_x_colmax") == 1
    x.mul_(2.0)                                                      # new version
    b = gnn.x_colmax(x)
    assert b is not a and stub.calls.count("gfd_x_colmax") == 2
    y = x.clone()                                                    # another tensor
    assert gnn.x_colmax(y) is not b and stub.calls.count("gfd_x_colmax") == 3
    for _ in range(gnn._COLMAX_ENTRIES + 2):                         # bounded
        gnn.x_colmax(torch.randn(3, 7))
    assert len(gnn._COLMAX) <= gnn._COLMAX_ENTRIES
    gnn._COLMAX.clear()
