"""GPU parity of the fused source pass + grad_W' GEMM (k_src_gw; gfd_gat_bwd
with GFD_BWD_FUSED=1 when grad_x is not requested -- the first layer, as in the
reference's GAT and TGN models whose input features take no gradient).  Opt-in:
at C4 it is slower than the unfused dh' path.

Oracle: oracle/gatconv_ref.py (the PyG GATConv dataflow on the CPU), as in
test_gatconv_gpu.py; tolerance 1e-4 of each gradient's scale (per column where
the inputs are heavy-tailed).  The unfused dh' path (GFD_BWD_FUSED=0) is also
compared with the fused one on the same graph.
"""
import pytest
import torch

from _util import assert_close_scaled
from test_gatconv_gpu import _device_dropout_mask, _per_column_close, _random_case

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True, params=["1", "2"], ids=["w8", "w16"])
def _fused(monkeypatch, request):
    # read by libgfd on every backward call: 1 = 8-wave blocks, 2 = 16-wave blocks
    monkeypatch.setenv("GFD_BWD_FUSED", request.param)


def _param_grads(x, graph_or_ei, conv, g, p=0.0, seed=0):
    """Gradients of W, att_src, att_dst, bias with x taking none (the fused path)."""
    from gfd.nn import GATConvFunction
    from gfd import graph as gg
    graph = graph_or_ei if isinstance(graph_or_ei, gg.CSRGraph) else gg.get_graph(
        graph_or_ei.to(DEV), x.size(0))
    ps = [conv.lin_src.weight.detach().to(DEV).requires_grad_(True),
          conv.att_src.detach().to(DEV).reshape(-1).requires_grad_(True),
          conv.att_dst.detach().to(DEV).reshape(-1).requires_grad_(True),
          conv.bias.detach().to(DEV).requires_grad_(True)]
    out = GATConvFunction.apply(x.to(DEV), ps[0], ps[1], ps[2], ps[3], graph, 0.2, p, seed)
    (out * g.to(DEV)).sum().backward()
    torch.cuda.synchronize()
    return [q.grad for q in ps]


def _oracle_param_grads(x, ei, conv, g, mask=None):
    from oracle import gatconv_forward
    for t in (conv.lin_src.weight, conv.att_src, conv.att_dst, conv.bias):
        t.grad = None
    ref = gatconv_forward(x, ei, conv.lin_src.weight, conv.att_src, conv.att_dst, conv.bias,
                          alpha_mask=mask)
    (ref * g).sum().backward()
    return [conv.lin_src.weight.grad, conv.att_src.grad.reshape(-1),
            conv.att_dst.grad.reshape(-1), conv.bias.grad]


NAMES = ("grad_W", "grad_att_src", "grad_att_dst", "grad_bias")


@pytest.mark.parametrize("N,E,F,kind", [
    (1, 0, 166, "powerlaw"),        # one node, self loop only: a one-slab, one-tile pass
    (37, 100, 1, "powerlaw"),       # F = 1 (one n-tile, padded)
    (300, 2000, 17, "powerlaw"),
    (2000, 2300, 165, "elliptic"),  # checkpoint width, sparse (many 1-message sources)
    (2000, 8000, 166, "powerlaw"),  # BASELINE width
    (500, 3000, 192, "powerlaw"),   # the fused path's widest feature tile
    (20000, 160000, 166, "powerlaw"),  # many tiles per slab, sources split over waves
])
def test_fused_param_grads_vs_oracle(N, E, F, kind):
    x, ei, conv = _random_case(N, E, F, seed=N + F + 1, kind=kind)
    g = torch.randn(N, 64, generator=torch.Generator().manual_seed(N))
    ref = _oracle_param_grads(x, ei, conv, g)
    got = _param_grads(x, ei, conv, g)
    for name, a, b in zip(NAMES, got, ref):
        assert_close_scaled(a, b, what=f"fused {name} N={N} F={F}")


def test_fused_matches_unfused_and_is_deterministic(monkeypatch):
    """The fused pass against the dh' path on one graph (both against each
    other at 1e-4 of scale), and bit-identical across two fused calls."""
    from gfd import graph as gg
    x, ei, conv = _random_case(40000, 300000, 166, seed=23)
    g = torch.randn(40000, 64, generator=torch.Generator().manual_seed(9))
    graph = gg.get_graph(ei.to(DEV), 40000)
    a = _param_grads(x, graph, conv, g)
    b = _param_grads(x, graph, conv, g)
    for name, u, v in zip(NAMES, a, b):
        assert torch.equal(u, v), f"fused {name} differs between two identical calls"
    monkeypatch.setenv("GFD_BWD_FUSED", "0")
    c = _param_grads(x, graph, conv, g)
    for name, u, v in zip(NAMES, a, c):
        assert_close_scaled(u, v, what=f"fused vs unfused {name}")


@pytest.mark.parametrize("threshold,chunk", [(4, 3), (16, 16), (64, 512)])
def test_fused_source_hubs(threshold, chunk):
    """Source hubs (out-degree > threshold) take the chunked hub kernels; their
    rows reach the fused GEMM compact, by hub rank.  Low thresholds put many
    of every tile's sources there."""
    from gfd import graph as gg
    N = 3000
    x, ei, conv = _random_case(N, 30000, 166, seed=41)
    g = torch.randn(N, 64, generator=torch.Generator().manual_seed(4))
    graph = gg.csr_from_coo(ei.to(DEV), N)  # uncached: its CSC plan is replaced below
    csc = graph.csc()
    csc.plan = gg.hub_plan(csc.colptr, graph.num_messages, threshold=threshold, chunk=chunk)
    assert csc.plan.num_hubs > 0
    ref = _oracle_param_grads(x, ei, conv, g)
    got = _param_grads(x, graph, conv, g)
    for name, a, b in zip(NAMES, got, ref):
        assert_close_scaled(a, b, what=f"fused {name}, source hubs thr={threshold}")


def test_fused_dropout_vs_oracle_with_same_mask():
    """Attention dropout (keep factor in the y-row bound): the oracle runs with
    the device's mask."""
    N, p, seed = 5000, 0.2, 99
    x, ei, conv = _random_case(N, 40000, 166, seed=13)
    mask = _device_dropout_mask(ei, N, seed, p)
    g = torch.randn(N, 64, generator=torch.Generator().manual_seed(12))
    ref = _oracle_param_grads(x, ei, conv, g, mask=mask)
    got = _param_grads(x, ei, conv, g, p=p, seed=seed)
    for name, a, b in zip(NAMES, got, ref):
        assert_close_scaled(a, b, what=f"fused dropout {name}")


def test_fused_bf16_features():
    N = 3000
    x, ei, conv = _random_case(N, 24000, 166, seed=22)
    xb = x.to(torch.bfloat16)
    g = torch.randn(N, 64, generator=torch.Generator().manual_seed(6))
    ref = _oracle_param_grads(xb.float(), ei, conv, g)
    got = _param_grads(xb, ei, conv, g)
    for name, a, b in zip(NAMES, got, ref):
        assert_close_scaled(a, b, what=f"fused bf16 x {name}")


@pytest.mark.parametrize("big", [1e6, 1e9])
def test_fused_heavy_tailed_features(big):
    """An outlier x column (zero weight, as in test_backward_heavy_tailed_features):
    every grad_W column within 2e-4 of its own scale."""
    N = 3000
    x, ei, conv = _random_case(N, 24000, 166, seed=31)
    x[:40, 0] = big * torch.linspace(-1, 1, 40)
    with torch.no_grad():
        conv.lin_src.weight[:, 0] = 0.0
    g = torch.randn(N, 64, generator=torch.Generator().manual_seed(7))
    ref = _oracle_param_grads(x, ei, conv, g)
    got = _param_grads(x, ei, conv, g)
    _per_column_close(got[0], ref[0], 2e-4, f"fused grad_W, outlier column {big:g}")
    for name, a, b in zip(NAMES[1:], got[1:], ref[1:]):
        assert_close_scaled(a, b, what=f"fused {name}")


def test_fused_heavy_tailed_gradient_rows():
    """Upstream gradient rows from 1e-4 to 1e6 of the others: the y rows'
    launch-wide channel scales are bounds (keep x max out-degree x max |g|),
    each grad_W column still within 2e-4 of its own scale."""
    N = 4000
    x, ei, conv = _random_case(N, 32000, 166, seed=32)
    g = torch.randn(N, 64, generator=torch.Generator().manual_seed(8))
    g[5] *= 1e6
    g[77] *= 1e-4
    ref = _oracle_param_grads(x, ei, conv, g)
    got = _param_grads(x, ei, conv, g)
    _per_column_close(got[0], ref[0], 2e-4, "fused grad_W per column")
    for name, a, b in zip(NAMES[1:], got[1:], ref[1:]):
        assert_close_scaled(a, b, what=f"fused {name}")
