"""GPU: the backward's per-column maxima of |x| (gfd_x_colmax, ABI 6) and their
cache in gfd.nn (once per version of the x tensor: the first layer's input is
the same tensor every training step, train.py:115-143).

gfd_x_colmax against torch's column maxima (exact: a max of floats); the
backward through gfd_gat_bwd_ex with the cached maxima bit-identical to
gfd_gat_bwd computing them itself; an in-place change of x (new version) and a
new tensor at a recycled address both recompute."""
import pytest
import torch

from test_gatconv_gpu import _random_case

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _colmax_ref(x):
    return x.float().abs().amax(0).view(torch.int32)


@pytest.mark.parametrize("dtype,pitch", [(torch.float32, 166), (torch.float32, 176),
                                         (torch.bfloat16, 184), (torch.float32, 167)])
def test_x_colmax_matches_torch(dtype, pitch):
    from gfd import _lib
    g = torch.Generator().manual_seed(3)
    buf = torch.randn(5000, pitch, generator=g).to(dtype)
    buf[17, 5] = 1e7          # an outlier column
    buf[:, 100] = 0.0         # an all-zero column
    x = buf.to(DEV)[:, :166]
    cm = torch.empty(166, dtype=torch.int32, device=DEV)
    _lib.call("gfd_x_colmax", x.data_ptr(), _lib.x_dtype_code(x), x.size(0), 166, x.stride(0),
              cm.data_ptr(), _lib.stream_handle(x.device))
    assert torch.equal(cm.cpu(), _colmax_ref(x).cpu())


def _grads(x, graph, conv, gout):
    from gfd.nn import GATConvFunction
    ps = [conv.lin_src.weight.detach().to(DEV).requires_grad_(True),
          conv.att_src.detach().to(DEV).reshape(-1).requires_grad_(True),
          conv.att_dst.detach().to(DEV).reshape(-1).requires_grad_(True),
          conv.bias.detach().to(DEV).requires_grad_(True)]
    out = GATConvFunction.apply(x, ps[0], ps[1], ps[2], ps[3], graph, 0.2, 0.0, 0, True)
    out.backward(gout)
    torch.cuda.synchronize()
    return [p.grad.clone() for p in ps]


def test_cached_colmax_backward_is_bit_identical_and_tracks_versions():
    from gfd import graph as gg, nn as gnn, _lib
    x_cpu, ei, conv = _random_case(3000, 20000, 166, seed=5, kind="powerlaw")
    x = x_cpu.to(DEV)
    graph = gg.get_graph(ei.to(DEV), 3000)
    gout = torch.randn(3000, 64, generator=torch.Generator().manual_seed(1)).to(DEV)
    gnn._COLMAX.clear()
    a = _grads(x, graph, conv, gout)             # computes and caches x's maxima
    cm = gnn.x_colmax(x)
    assert torch.equal(cm, _colmax_ref(x))
    b = _grads(x, graph, conv, gout)             # served from the cache
    assert gnn.x_colmax(x) is cm
    for u, v in zip(a, b):
        assert torch.equal(u, v)
    # the same backward with the maxima computed inside (gfd_gat_bwd): bit-identical
    from gfd.nn import GATConvFunction
    orig = _lib.call

    def no_colmax(name, *args):
        if name == "gfd_gat_bwd_ex":
            args = list(args)
            args[-4] = None                      # x_colmax -> computed by the library
        return orig(name, *args)
    _lib.call = no_colmax
    try:
        c = _grads(x, graph, conv, gout)
    finally:
        _lib.call = orig
    for u, v in zip(a, c):
        assert torch.equal(u, v)
    # an in-place change of x is a new version: recomputed
    with torch.no_grad():
        x[7, 3] = 1e5
    cm2 = gnn.x_colmax(x)
    assert cm2 is not cm and torch.equal(cm2, _colmax_ref(x))
    # a different tensor (even at a recycled address) is never served x's entry
    y = x.clone()
    assert gnn.x_colmax(y) is not cm2
    gnn._COLMAX.clear()
