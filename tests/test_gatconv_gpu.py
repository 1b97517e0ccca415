"""GPU parity tests for the GATConv hot path (libgfd.so via the C ABI).

Oracle: oracle/gatconv_ref.py (PyG 2.x GATConv dataflow restated on the CPU),
pinned by tests/golden/*.npz which were produced by the reference's own model
code (tests/golden/make_golden.py).  Tolerance: 1e-4 (BASELINE.json north_star).
"""
import numpy as np
import pytest
import torch

from _util import FWD_ATOL, assert_close, assert_close_scaled, csr_cpu

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _gfd():
    import gfd.graph as graph
    import gfd.nn as gnn
    return gnn, graph


def _run_case(arr, name, backward=True):
    gnn, _ = _gfd()
    x = torch.from_numpy(arr[f"{name}.x"]).to(DEV).requires_grad_(backward)
    ei = torch.from_numpy(arr[f"{name}.edge_index"]).to(DEV)
    W = torch.from_numpy(arr[f"{name}.weight"]).to(DEV).requires_grad_(backward)
    a_s = torch.from_numpy(arr[f"{name}.att_src"]).to(DEV).requires_grad_(backward)
    a_d = torch.from_numpy(arr[f"{name}.att_dst"]).to(DEV).requires_grad_(backward)
    b = torch.from_numpy(arr[f"{name}.bias"]).to(DEV).requires_grad_(backward)
    out = gnn.gat_conv(x, ei, W, a_s, a_d, b)
    grads = None
    if backward:
        g = torch.from_numpy(arr[f"{name}.grad_out"]).to(DEV)
        (out * g).sum().backward()
        grads = {"x": x.grad, "weight": W.grad, "att_src": a_s.grad, "att_dst": a_d.grad,
                 "bias": b.grad}
    torch.cuda.synchronize()
    return out, grads


@pytest.mark.parametrize("case", ["base", "scale100"])
def test_edgecases_forward(golden, case):
    arr = golden("gatconv_edgecases.npz")
    out, _ = _run_case(arr, case, backward=False)
    assert_close(out, arr[f"{case}.out"], what=f"edgecases/{case} out")


@pytest.mark.parametrize("case", ["base", "scale100"])
def test_edgecases_backward(golden, case):
    arr = golden("gatconv_edgecases.npz")
    _, grads = _run_case(arr, case)
    for k, v in grads.items():
        assert_close_scaled(v.reshape(arr[f"{case}.grad_{k}"].shape), arr[f"{case}.grad_{k}"],
                            what=f"edgecases/{case} grad_{k}")


def test_powerlaw_f166_forward_backward(golden):
    arr = golden("gatconv_f166.npz")
    out, grads = _run_case(arr, "pl")
    assert_close(out, arr["pl.out"], what="f166 out")
    for k, v in grads.items():
        assert_close_scaled(v.reshape(arr[f"pl.grad_{k}"].shape), arr[f"pl.grad_{k}"],
                            what=f"f166 grad_{k}")


def _random_case(N, E, F, seed, kind="powerlaw"):
    from gfd import synth
    from oracle import GATConvRef
    if kind == "powerlaw":
        ei = torch.from_numpy(synth.power_law(N, E, seed=seed))
        x = torch.randn(N, F, generator=torch.Generator().manual_seed(seed))
    else:
        g = synth.elliptic_like(N, E, num_steps=7, num_features=F, seed=seed)
        ei, x = torch.from_numpy(g["edge_index"]), torch.from_numpy(g["x"])
    gen = torch.Generator().manual_seed(seed + 1)
    conv = GATConvRef(F, 64, heads=8, concat=False)
    conv.reset_parameters(gen)
    with torch.no_grad():
        conv.bias.copy_(torch.randn(64, generator=gen))
    return x, ei, conv


@pytest.mark.parametrize("N,E,F,kind", [
    (1, 0, 166, "powerlaw"),        # single node, no edges (self loop only)
    (37, 100, 1, "powerlaw"),       # F = 1
    (300, 2000, 17, "powerlaw"),
    (1000, 5000, 64, "powerlaw"),   # hidden-layer width
    (2000, 2300, 165, "elliptic"),  # checkpoint width
    (2000, 8000, 166, "powerlaw"),  # BASELINE width
    (500, 3000, 200, "powerlaw"),
    (333, 4000, 256, "powerlaw"),   # max width
    # k_stream's three register layouts (1, 2, 3 feature chunks) over many tiles per
    # block (N / 16 tiles on 256 blocks: the row/record pipeline runs several laps),
    # exact (F = 64, 128, 166) and padded (F = 100) K halves
    (20000, 160000, 64, "powerlaw"),
    (20000, 160000, 100, "powerlaw"),
    (20000, 160000, 128, "powerlaw"),
    (20000, 160000, 166, "powerlaw"),
])
def test_forward_vs_oracle(N, E, F, kind):
    gnn, _ = _gfd()
    x, ei, conv = _random_case(N, E, F, seed=N + F, kind=kind)
    with torch.no_grad():
        ref = conv(x, ei)
        out = gnn.gat_conv(x.to(DEV), ei.to(DEV), conv.lin_src.weight.to(DEV),
                           conv.att_src.to(DEV), conv.att_dst.to(DEV), conv.bias.to(DEV))
    assert_close(out, ref, what=f"N={N} E={E} F={F}")


def test_backward_vs_oracle_elliptic_like():
    gnn, _ = _gfd()
    x, ei, conv = _random_case(3000, 3500, 165, seed=9, kind="elliptic")
    g = torch.randn(3000, 64, generator=torch.Generator().manual_seed(3))
    xr = x.clone().requires_grad_(True)
    (conv(xr, ei) * g).sum().backward()
    xd = x.to(DEV).requires_grad_(True)
    W = conv.lin_src.weight.detach().to(DEV).requires_grad_(True)
    a_s = conv.att_src.detach().to(DEV).requires_grad_(True)
    a_d = conv.att_dst.detach().to(DEV).requires_grad_(True)
    b = conv.bias.detach().to(DEV).requires_grad_(True)
    (gnn.gat_conv(xd, ei.to(DEV), W, a_s, a_d, b) * g.to(DEV)).sum().backward()
    assert_close_scaled(xd.grad, xr.grad, what="grad_x")
    assert_close_scaled(W.grad, conv.lin_src.weight.grad, what="grad_W")
    assert_close_scaled(a_s.grad, conv.att_src.grad, what="grad_att_src")
    assert_close_scaled(a_d.grad, conv.att_dst.grad, what="grad_att_dst")
    assert_close_scaled(b.grad, conv.bias.grad, what="grad_bias")


def _grads(gnn, x, ei, conv, g):
    xd = x.to(DEV).requires_grad_(True)
    ps = [t.detach().to(DEV).requires_grad_(True)
          for t in (conv.lin_src.weight, conv.att_src, conv.att_dst, conv.bias)]
    (gnn.gat_conv(xd, ei.to(DEV), *ps) * g.to(DEV)).sum().backward()
    return [xd.grad] + [p.grad for p in ps]


def test_backward_is_deterministic():
    """No float atomics: grad_W (split-K over 40k nodes), grad_att and
    grad_bias (per-block partials) come out bit-identical run to run."""
    gnn, _ = _gfd()
    x, ei, conv = _random_case(40000, 300000, 166, seed=21)
    g = torch.randn(40000, 64, generator=torch.Generator().manual_seed(5))
    a = _grads(gnn, x, ei, conv, g)
    b = _grads(gnn, x, ei, conv, g)
    for name, u, v in zip(("x", "W", "att_src", "att_dst", "bias"), a, b):
        assert torch.equal(u, v), f"grad_{name} differs between two identical backward calls"


def test_backward_bf16_features():
    """bf16 x goes straight into the backward (rows converted on load): the
    gradients equal the fp32 oracle's on the bf16-rounded features."""
    gnn, _ = _gfd()
    x, ei, conv = _random_case(3000, 24000, 166, seed=22)
    xb = x.to(torch.bfloat16)
    g = torch.randn(3000, 64, generator=torch.Generator().manual_seed(6))
    xr = xb.float().requires_grad_(True)
    (conv(xr, ei) * g).sum().backward()
    gx, gW, gas, gad, gb = _grads(gnn, xb, ei, conv, g)
    assert gx.dtype == torch.bfloat16
    assert_close_scaled(gW, conv.lin_src.weight.grad, what="grad_W (bf16 x)")
    assert_close_scaled(gas, conv.att_src.grad, what="grad_att_src (bf16 x)")
    assert_close_scaled(gad, conv.att_dst.grad, what="grad_att_dst (bf16 x)")
    assert_close_scaled(gb, conv.bias.grad, what="grad_bias (bf16 x)")
    # grad_x is returned in x's dtype: compare at bf16 resolution
    assert torch.allclose(gx.float().cpu(), xr.grad.to(torch.bfloat16).float(),
                          rtol=2 ** -7, atol=1e-3 * xr.grad.abs().max().item())


def _per_column_close(got, ref, rtol, what, dim=0):
    """|got - ref| <= rtol * (max |ref| along dim) per column (dim=0) or per row
    (dim=1): a heavy-tailed column must not cost the other columns precision,
    which a whole-tensor scale would hide."""
    got = got.detach().cpu().double()
    ref = ref.detach().cpu().double()
    scale = ref.abs().amax(dim=dim, keepdim=True).clamp_min(1e-30)
    rel = ((got - ref).abs() / scale).amax()
    assert rel <= rtol, f"{what}: worst per-{'column' if dim == 0 else 'row'} error {rel:.3e} > {rtol}"


@pytest.mark.parametrize("big", [1e6, 1e9])
def test_backward_heavy_tailed_features(big):
    """An outlier feature column: the grad_W' GEMM scales each x
    and dh' column on its own, so the other columns keep fp32-faithful
    products (one scale from max |x| pushed them into fp16 subnormals at 1e9).
    The outlier feature has zero weight, so the attention (and dh') stay
    well-conditioned and the fp32 oracle is a fair reference; every grad_W
    column is checked against its own scale."""
    gnn, _ = _gfd()
    x, ei, conv = _random_case(3000, 24000, 166, seed=31)
    x[:40, 0] = big * torch.linspace(-1, 1, 40)
    with torch.no_grad():
        conv.lin_src.weight[:, 0] = 0.0
    g = torch.randn(3000, 64, generator=torch.Generator().manual_seed(7))
    xr = x.clone().requires_grad_(True)
    (conv(xr, ei) * g).sum().backward()
    gx, gW, gas, gad, gb = _grads(gnn, x, ei, conv, g)
    Wref = conv.lin_src.weight.grad  # [512, F]: columns = features
    _per_column_close(gW, Wref, 2e-4, f"grad_W, outlier column {big:g}")
    assert_close_scaled(gas, conv.att_src.grad, what="grad_att_src")
    assert_close_scaled(gad, conv.att_dst.grad, what="grad_att_dst")
    assert_close_scaled(gb, conv.bias.grad, what="grad_bias")


@pytest.mark.parametrize("layout", ["contiguous", "pitch168"])
def test_forward_logits_heavy_tailed_features(layout):
    """The logits pass on rows with an outlier feature (its weight zero, so it
    must not matter): the f16 split under one row scale would lose the row's
    other features; k_logits_lone detects such rows (nonzero features spanning
    more than 2^18) and runs their tile on fp32 MFMA.  Checked: the s | t
    logits (gfd_gat_logits_lone, exact to fp32 against the oracle's) and the
    self-loop-only rows' outputs, in the inference layout and the reference's
    contiguous [N, 166] layout."""
    from gfd import dist as gdist, graph as ggraph, _lib
    x, ei, conv = _random_case(3000, 9000, 166, seed=33)
    x[:40, 0] = 1e9 * torch.linspace(-1, 1, 40)
    with torch.no_grad():
        conv.lin_src.weight[:, 0] = 0.0
    N, F = x.shape
    W = conv.lin_src.weight.detach()
    h = (x.double() @ W.double().t()).view(N, 8, 64)
    st_ref = torch.cat([(h * conv.att_src.detach().double()).sum(-1),
                        (h * conv.att_dst.detach().double()).sum(-1)], 1)
    if layout == "contiguous":
        xd = x.to(DEV)
    else:
        xd = torch.nn.functional.pad(x, (0, 2)).to(DEV)[:, :F]
    g = ggraph.csr_from_coo(ei.to(DEV), N)
    packed = gdist.pack_weights(W.to(DEV), conv.att_src.detach().to(DEV),
                                conv.att_dst.detach().to(DEV))
    st = torch.empty((N, 16), device=DEV)
    out = torch.zeros((N, 64), device=DEV)
    xmax = torch.zeros(1, device=DEV)
    _lib.call("gfd_gat_logits_lone", xd.data_ptr(), _lib.x_dtype_code(xd), N, F, xd.stride(0),
              packed.data_ptr(), 8, 64, g.rowptr.data_ptr(), conv.bias.detach().to(DEV).data_ptr(),
              0.2, st.data_ptr(), xmax.data_ptr(), out.data_ptr(), None, _lib.stream_handle(DEV))
    torch.cuda.synchronize()
    err = (st.cpu().double() - st_ref).abs()
    bound = 1e-5 * st_ref.abs().amax(1, keepdim=True) + 1e-6
    assert bool((err <= bound).all()), f"logits: max err {err.max():.3e}"
    # the self-loop-only rows' outputs (Wbar x_i + bias) on the outlier rows too
    deg = (g.rowptr[1:] - g.rowptr[:-1]).cpu()
    lone = torch.nonzero(deg == 1).flatten()
    ref_out = conv(x, ei).detach()
    assert_close(out.cpu()[lone], ref_out[lone], what=f"lone rows' outputs ({layout})")


def test_backward_heavy_tailed_gradient_rows():
    """A destination whose upstream gradient is 10^6 times the others (hidden
    layer, F = 64: grad_x on the fp16 MFMA path): each dh' row is scaled on its
    own, so every row of grad_x keeps its precision."""
    gnn, _ = _gfd()
    x, ei, conv = _random_case(4000, 32000, 64, seed=32)
    g = torch.randn(4000, 64, generator=torch.Generator().manual_seed(8))
    g[5] *= 1e6
    g[77] *= 1e-4
    xr = x.clone().requires_grad_(True)
    (conv(xr, ei) * g).sum().backward()
    gx, gW, gas, gad, gb = _grads(gnn, x, ei, conv, g)
    nz = xr.grad.abs().amax(dim=1) > 0
    _per_column_close(gx[nz], xr.grad[nz], 2e-4, "grad_x per row", dim=1)
    _per_column_close(gW, conv.lin_src.weight.grad, 2e-4, "grad_W per column")


@pytest.mark.parametrize("threshold,chunk", [(1, 1), (4, 3), (16, 16), (1 << 30, 128)])
@pytest.mark.parametrize("classes", [False, True])
def test_hub_split_equivalence(threshold, chunk, classes):
    """Same outputs whatever the hub threshold/chunking (merge is exact math),
    through k_fused (plan without slot sources) and through the
    class-scheduled kernels (k_mid / k_stream / k_lone)."""
    gnn, graph = _gfd()
    x, ei, conv = _random_case(800, 6000, 166, seed=4)
    xd, eid = x.to(DEV), ei.to(DEV)
    g = graph.csr_from_coo(eid, 800)
    g._plan = graph.build_plan(g.rowptr, g.num_messages, threshold=threshold, chunk=chunk,
                               col=g.col if classes else None)
    with torch.no_grad():
        out = gnn.gat_conv(xd, g, conv.lin_src.weight.to(DEV), conv.att_src.to(DEV),
                           conv.att_dst.to(DEV), conv.bias.to(DEV))
        ref = conv(x, ei)
    assert_close(out, ref, what=f"hub thr={threshold} chunk={chunk}")


def test_csr_matches_pyg_self_loop_policy():
    _, graph = _gfd()
    rng = np.random.default_rng(0)
    N = 500
    ei = rng.integers(0, N, (2, 4000))
    ei[:, :50] = ei[0, :50]  # self loops in the input
    ei = torch.from_numpy(ei)
    g = graph.csr_from_coo(ei.to(DEV), N)
    rp, col = csr_cpu(ei, N)
    assert torch.equal(g.rowptr.cpu().long(), rp)
    assert torch.equal(g.col.cpu().long(), col)          # stable order, loops last
    csc = g.csc()
    # every message appears once in the CSC, grouped by source, CSR order inside
    eid = csc.eid.cpu().long()
    assert torch.equal(torch.sort(eid).values, torch.arange(g.num_messages))
    src_sorted = col[eid]
    assert bool((src_sorted[1:] >= src_sorted[:-1]).all())
    dst_of = torch.repeat_interleave(torch.arange(N), rp[1:] - rp[:-1])
    assert torch.equal(csc.dst.cpu().long(), dst_of[eid])


def test_index_out_of_range_raises():
    _, graph = _gfd()
    ei = torch.tensor([[0, 1, 5], [1, 2, 0]], device=DEV)
    with pytest.raises(IndexError):
        graph.csr_from_coo(ei, 5)


def test_deterministic_forward():
    gnn, _ = _gfd()
    x, ei, conv = _random_case(4000, 30000, 166, seed=2)
    args = (x.to(DEV), ei.to(DEV), conv.lin_src.weight.to(DEV), conv.att_src.to(DEV),
            conv.att_dst.to(DEV), conv.bias.to(DEV))
    with torch.no_grad():
        a = gnn.gat_conv(*args)
        b = gnn.gat_conv(*args)
    assert torch.equal(a, b)


def test_dropout_is_reproducible_and_unbiased():
    """Train-mode dropout on alpha: same seed -> same output; E[out] ~ eval output."""
    gnn, _ = _gfd()
    from gfd.nn import GATConvFunction
    x, ei, conv = _random_case(2000, 20000, 64, seed=5)
    xd = x.to(DEV)
    g = _gfd()[1].get_graph(ei.to(DEV), 2000)
    W, a_s, a_d, b = (conv.lin_src.weight.to(DEV), conv.att_src.to(DEV).reshape(-1),
                      conv.att_dst.to(DEV).reshape(-1), conv.bias.to(DEV))
    with torch.no_grad():
        o1 = GATConvFunction.apply(xd, W, a_s, a_d, b, g, 0.2, 0.2, 1234)
        o2 = GATConvFunction.apply(xd, W, a_s, a_d, b, g, 0.2, 0.2, 1234)
        o3 = GATConvFunction.apply(xd, W, a_s, a_d, b, g, 0.2, 0.2, 99)
        ev = GATConvFunction.apply(xd, W, a_s, a_d, b, g, 0.2, 0.0, 0)
        avg = sum(GATConvFunction.apply(xd, W, a_s, a_d, b, g, 0.2, 0.2, s) for s in range(64)) / 64
    assert torch.equal(o1, o2)
    assert not torch.equal(o1, o3)
    # unbiased: the mean over seeds approaches the eval output
    assert (avg - ev).abs().mean() < 0.25 * (o1 - ev).abs().mean()


def _device_dropout_mask(edge_index, num_nodes, seed, p):
    """Restate libgfd's counter-based mask (gfd_common.h dropout_keep) on the
    host, in the oracle's edge order (kept edges, then self loops)."""
    from oracle import remove_then_add_self_loops
    ei = remove_then_add_self_loops(edge_index, num_nodes)
    pos = torch.empty(ei.size(1), dtype=torch.long)
    pos[torch.argsort(ei[1], stable=True)] = torch.arange(ei.size(1))   # CSR position
    with np.errstate(over="ignore"):
        e = pos.numpy().astype(np.uint64)[:, None]
        h = np.arange(8, dtype=np.uint64)[None, :]
        z = np.uint64(seed) ^ (((e << np.uint64(3)) | h) * np.uint64(0x9E3779B97F4A7C15))
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    u = (z >> np.uint64(40)).astype(np.float32) * np.float32(1.0 / 16777216.0)
    keep = u >= np.float32(p)
    return torch.from_numpy(keep.astype(np.float32) / np.float32(1.0 - p))


def test_dropout_forward_backward_vs_oracle_with_same_mask():
    """Train-mode dropout on alpha (reference: GATConv dropout=0.2, gat.py:39):
    the device mask is regenerated in the backward; the oracle is run with the
    identical mask, forward and all gradients within 1e-4."""
    from gfd.nn import GATConvFunction
    from oracle import gatconv_forward
    _, graph = _gfd()
    N, p, seed = 600, 0.3, 77
    x, ei, conv = _random_case(N, 5000, 48, seed=8)
    mask = _device_dropout_mask(ei, N, seed, p)
    go = torch.randn(N, 64, generator=torch.Generator().manual_seed(2))
    xr = x.clone().requires_grad_(True)
    ref = gatconv_forward(xr, ei, conv.lin_src.weight, conv.att_src, conv.att_dst, conv.bias,
                          alpha_mask=mask)
    (ref * go).sum().backward()
    g = graph.get_graph(ei.to(DEV), N)
    xd = x.to(DEV).requires_grad_(True)
    W = conv.lin_src.weight.detach().to(DEV).requires_grad_(True)
    a_s = conv.att_src.detach().to(DEV).reshape(-1).requires_grad_(True)
    a_d = conv.att_dst.detach().to(DEV).reshape(-1).requires_grad_(True)
    b = conv.bias.detach().to(DEV).requires_grad_(True)
    out = GATConvFunction.apply(xd, W, a_s, a_d, b, g, 0.2, p, seed)
    (out * go.to(DEV)).sum().backward()
    assert_close(out, ref, what="dropout forward")
    assert_close_scaled(xd.grad, xr.grad, what="dropout grad_x")
    assert_close_scaled(W.grad, conv.lin_src.weight.grad, what="dropout grad_W")
    assert_close_scaled(a_s.grad, conv.att_src.grad.reshape(-1), what="dropout grad_att_src")
    assert_close_scaled(a_d.grad, conv.att_dst.grad.reshape(-1), what="dropout grad_att_dst")
    assert_close_scaled(b.grad, conv.bias.grad, what="dropout grad_bias")


def test_dropout_all_classes_at_20k_nodes():
    """The reference's training configuration (GATConv dropout=0.2, gat.py:39,
    config.py:35) through the class-scheduled kernels: hubs, general, light
    and the self-loop-only rows (which with dropout run in the light kernel:
    per-head masks), forward and backward against the oracle with the device's
    mask, on a 20k-node power-law graph where every class is populated."""
    from gfd.nn import GATConvFunction
    from oracle import gatconv_forward
    _, graph = _gfd()
    N, p, seed = 20000, 0.2, 4242
    x, ei, conv = _random_case(N, 100000, 166, seed=21)
    g = graph.get_graph(ei.to(DEV), N)
    plan = g.plan()
    light_b, lone_b = plan.classes()
    assert plan.num_hubs > 0 and 0 < light_b < lone_b < N          # every class present
    mask = _device_dropout_mask(ei, N, seed, p)
    go = torch.randn(N, 64, generator=torch.Generator().manual_seed(3))
    xr = x.clone().requires_grad_(True)
    ref = gatconv_forward(xr, ei, conv.lin_src.weight, conv.att_src, conv.att_dst, conv.bias,
                          alpha_mask=mask)
    (ref * go).sum().backward()
    xd = x.to(DEV).requires_grad_(True)
    W = conv.lin_src.weight.detach().to(DEV).requires_grad_(True)
    a_s = conv.att_src.detach().to(DEV).reshape(-1).requires_grad_(True)
    a_d = conv.att_dst.detach().to(DEV).reshape(-1).requires_grad_(True)
    b = conv.bias.detach().to(DEV).requires_grad_(True)
    out = GATConvFunction.apply(xd, W, a_s, a_d, b, g, 0.2, p, seed)
    (out * go.to(DEV)).sum().backward()
    assert_close(out, ref, what="dropout forward, all classes")
    assert_close_scaled(xd.grad, xr.grad, what="dropout grad_x")
    assert_close_scaled(W.grad, conv.lin_src.weight.grad, what="dropout grad_W")
    assert_close_scaled(a_s.grad, conv.att_src.grad.reshape(-1), what="dropout grad_att_src")
    assert_close_scaled(a_d.grad, conv.att_dst.grad.reshape(-1), what="dropout grad_att_dst")
    assert_close_scaled(b.grad, conv.bias.grad, what="dropout grad_bias")


@pytest.mark.slow
def test_full_size_sampled_parity_and_invariants():
    """C4-shaped graph (2M nodes / 10M edges here to bound test time): exact
    oracle on a sample of destinations (incl. the biggest hubs) + invariants."""
    gnn, graph = _gfd()
    from gfd import synth
    from oracle import GATConvRef, gatconv_forward_at
    N, E, F = 2_000_000, 10_000_000, 166
    ei = synth.power_law_device(N, E, seed=1, device=DEV)
    x = torch.randn(N, F, device=DEV, generator=torch.Generator(device=DEV).manual_seed(0))
    conv = GATConvRef(F, 64, heads=8, concat=False)
    conv.reset_parameters(torch.Generator().manual_seed(0))
    with torch.no_grad():
        conv.bias.normal_()
    g = graph.get_graph(ei, N)
    assert g.plan().num_hubs > 0
    with torch.no_grad():
        out = gnn.gat_conv(x, g, conv.lin_src.weight.to(DEV), conv.att_src.to(DEV),
                           conv.att_dst.to(DEV), conv.bias.to(DEV))
    assert torch.isfinite(out).all()
    deg = (g.rowptr[1:] - g.rowptr[:-1]).cpu()
    top = torch.topk(deg, 8).indices
    rnd = torch.randint(0, N, (256,), generator=torch.Generator().manual_seed(1))
    dsts = torch.unique(torch.cat([top, rnd]))
    ref = gatconv_forward_at(x.cpu(), g.rowptr.cpu().long(), g.col.cpu().long(), dsts,
                             conv.lin_src.weight, conv.att_src, conv.att_dst, conv.bias)
    assert_close(out[dsts.to(DEV)], ref, what="sampled full-size")
    # self-loop-only destinations: output is exactly mean_h W_h x_i + b
    lone = torch.nonzero(deg == 1).flatten()[:64]
    Wbar = conv.lin_src.weight.view(8, 64, F).mean(0)
    ref_lone = x.cpu()[lone] @ Wbar.t() + conv.bias
    assert_close(out[lone.to(DEV)], ref_lone.detach(), what="self-loop-only rows")


def _checked_lib():
    import os
    from gfd import _lib
    path = os.path.join(os.path.dirname(_lib.LIB_PATH), "libgfd_checked.so")
    assert os.path.exists(path), "libgfd_checked.so missing: __graft_entry__.build() ships it"
    return _lib.open_variant(path)


@pytest.mark.parametrize("corrupt", ["col", "rowptr", "slot_desc", "csc_dst"])
def test_checked_build_rejects_bad_indices(corrupt):
    """The checked build validates every index array before any gather kernel
    runs: one corrupted entry (a source >= N, a rowptr past the end, a slot
    descriptor of another row, a CSC destination >= N) makes the forward /
    backward return GFD_ERR_INDEX instead of faulting inside a gather, and the
    output buffer is not touched."""
    from gfd import _lib
    chk = _checked_lib()
    _, graph = _gfd()
    N, F = 3000, 64
    x, ei, conv = _random_case(N, 20000, F, seed=32)
    g = graph.get_graph(ei.to(DEV), N)
    plan, csc = g.plan(), g.csc()
    rowptr, col = g.rowptr.clone(), g.col.clone()
    desc = plan.slot_desc.clone() if plan.slot_desc is not None else None
    cdst = csc.dst.clone()
    if corrupt == "col":
        col[len(col) // 2] = N
    elif corrupt == "rowptr":
        rowptr[N // 2] = rowptr[-1] + 7
    elif corrupt == "slot_desc":
        desc.view(-1, 4)[N // 3, 1] += 1           # e_begin no longer its row's start
    else:
        cdst[5] = N + 3
    plan.cstruct()
    pc = _lib.GfdPlan.from_buffer_copy(plan._c)
    if corrupt == "slot_desc":
        pc.slot_desc = desc.data_ptr()
    cp = _lib.ct.byref(pc)
    xd = x.to(DEV).contiguous()
    W = conv.lin_src.weight.detach().to(DEV).contiguous()
    a_s = conv.att_src.detach().to(DEV).reshape(-1).contiguous()
    a_d = conv.att_dst.detach().to(DEV).reshape(-1).contiguous()
    b = conv.bias.detach().to(DEV)
    stream = _lib.stream_handle(DEV)
    out = torch.full((N, 64), 7.0, device=DEV)
    st = torch.zeros(N, 16, device=DEV)
    ws = torch.empty(chk.gfd_gat_fwd_workspace_size(N, N, F, 8, 64, plan.num_hubs, plan.num_chunks),
                     dtype=torch.uint8, device=DEV)
    if corrupt != "csc_dst":
        rc = chk.gfd_gat_fwd(xd.data_ptr(), 0, N, F, F, rowptr.data_ptr(), col.data_ptr(),
                             W.data_ptr(), a_s.data_ptr(), a_d.data_ptr(), b.data_ptr(), 8, 64, 0.2,
                             0.0, 0, cp, out.data_ptr(), st.data_ptr(), None, ws.data_ptr(),
                             ws.numel(), stream)
        torch.cuda.synchronize()
        assert rc == 2, f"checked forward returned {rc} for a corrupted {corrupt}"
        assert torch.all(out == 7.0), "no kernel may write the output after a failed check"
        return
    # backward over a valid forward, the CSC corrupted
    stats = torch.empty(N, 16, device=DEV)
    assert chk.gfd_gat_fwd(xd.data_ptr(), 0, N, F, F, rowptr.data_ptr(), col.data_ptr(),
                           W.data_ptr(), a_s.data_ptr(), a_d.data_ptr(), b.data_ptr(), 8, 64, 0.2,
                           0.0, 0, cp, out.data_ptr(), st.data_ptr(), stats.data_ptr(),
                           ws.data_ptr(), ws.numel(), stream) == 0
    go = torch.randn(N, 64, device=DEV)
    gw = torch.full_like(W, 7.0)
    ga, gd = torch.empty_like(a_s), torch.empty_like(a_d)
    gb = torch.empty(64, device=DEV)
    bws = torch.empty(chk.gfd_gat_bwd_workspace_size(N, g.num_messages, F, 8, 64, plan.num_hubs,
                                                     plan.num_chunks, csc.plan.num_chunks),
                      dtype=torch.uint8, device=DEV)
    rc = chk.gfd_gat_bwd(xd.data_ptr(), 0, N, F, F, rowptr.data_ptr(), col.data_ptr(), cp,
                         csc.colptr.data_ptr(), cdst.data_ptr(), csc.eid.data_ptr(),
                         csc.plan.cstruct(), g.num_messages, W.data_ptr(), a_s.data_ptr(),
                         a_d.data_ptr(), 8, 64, 0.2, 0.0, 0, st.data_ptr(), stats.data_ptr(),
                         go.data_ptr(), None, gw.data_ptr(), ga.data_ptr(), gd.data_ptr(),
                         gb.data_ptr(), bws.data_ptr(), bws.numel(), stream)
    torch.cuda.synchronize()
    assert rc == 2, f"checked backward returned {rc} for a corrupted csc_dst"
    assert torch.all(gw == 7.0)


def test_checked_build_accepts_valid_graphs():
    """The bounds-checked diagnostic build (-DGFD_CHECKED, libgfd_checked.so:
    every index array validated on the device before the kernels run) gives
    the product library's forward and backward on a valid graph with hubs and
    every class (no false positives).  build() ships the variant."""
    from gfd import _lib
    chk = _checked_lib()
    prod = _lib.load()
    _, graph = _gfd()
    N, F = 6000, 166
    x, ei, conv = _random_case(N, 48000, F, seed=31)
    g = graph.get_graph(ei.to(DEV), N)
    plan, csc = g.plan(), g.csc()
    xd = x.to(DEV).contiguous()
    W = conv.lin_src.weight.detach().to(DEV).contiguous()
    a_s = conv.att_src.detach().to(DEV).reshape(-1).contiguous()
    a_d = conv.att_dst.detach().to(DEV).reshape(-1).contiguous()
    b = conv.bias.detach().to(DEV)
    go = torch.randn(N, 64, device=DEV)
    stream = _lib.stream_handle(DEV)
    res = []
    for lib in (prod, chk):
        out = torch.empty(N, 64, device=DEV)
        st = torch.empty(N, 16, device=DEV)
        stats = torch.empty(N, 16, device=DEV)
        ws = torch.empty(lib.gfd_gat_fwd_workspace_size(N, N, F, 8, 64, plan.num_hubs, plan.num_chunks),
                         dtype=torch.uint8, device=DEV)
        assert lib.gfd_gat_fwd(xd.data_ptr(), 0, N, F, F, g.rowptr.data_ptr(), g.col.data_ptr(),
                               W.data_ptr(), a_s.data_ptr(), a_d.data_ptr(), b.data_ptr(), 8, 64,
                               0.2, 0.0, 0, plan.cstruct(), out.data_ptr(), st.data_ptr(),
                               stats.data_ptr(), ws.data_ptr(), ws.numel(), stream) == 0
        gw = torch.empty_like(W)
        ga, gd = torch.empty_like(a_s), torch.empty_like(a_d)
        gb = torch.empty(64, device=DEV)
        bws = torch.empty(lib.gfd_gat_bwd_workspace_size(N, g.num_messages, F, 8, 64, plan.num_hubs,
                                                         plan.num_chunks, csc.plan.num_chunks),
                          dtype=torch.uint8, device=DEV)
        assert lib.gfd_gat_bwd(xd.data_ptr(), 0, N, F, F, g.rowptr.data_ptr(), g.col.data_ptr(),
                               plan.cstruct(), csc.colptr.data_ptr(), csc.dst.data_ptr(),
                               csc.eid.data_ptr(), csc.plan.cstruct(), g.num_messages, W.data_ptr(),
                               a_s.data_ptr(), a_d.data_ptr(), 8, 64, 0.2, 0.0, 0, st.data_ptr(),
                               stats.data_ptr(), go.data_ptr(), None, gw.data_ptr(), ga.data_ptr(),
                               gd.data_ptr(), gb.data_ptr(), bws.data_ptr(), bws.numel(),
                               stream) == 0
        torch.cuda.synchronize()
        res.append((out, gw, ga, gd, gb))
    for u, v in zip(*res):
        assert torch.equal(u, v)
