"""Destination-sharded forward through the HIP library.

One GPU here, so the ranks are run one after the other in this process: each
"rank" computes its node block's logits and its destination shard with
gfd.dist's stage functions, the blocks are concatenated as the all-gathers
would, and the result must match the single-call forward and the oracle.  A
world_size-1 RCCL group then runs gat_conv_sharded end to end (collectives
included).
"""
import os
import socket

import pytest
import torch

from _util import assert_close
from oracle import gatconv_ref as ref

pytestmark = pytest.mark.gpu
H, C = 8, 64


def _problem(N, E, F, seed, dev):
    from gfd import synth
    g = torch.Generator().manual_seed(seed)
    ei = torch.from_numpy(synth.power_law(N, E, gamma=2.1, seed=seed))
    x = torch.randn(N, F, generator=g)
    W = ref.glorot_(torch.empty(H * C, F), g)
    a_s = ref.glorot_(torch.empty(1, H, C), g)
    a_d = ref.glorot_(torch.empty(1, H, C), g)
    b = torch.randn(C, generator=g) * 0.1
    return ei, x, W, a_s, a_d, b


@pytest.mark.parametrize("world,use_xmax", [(2, False), (3, False), (8, False), (2, True),
                                            (3, True)])
def test_virtual_ranks_match_oracle(world, use_xmax):
    from gfd import dist as gdist, graph as ggraph
    dev = torch.device("cuda", 0)
    N, E, F = 20000, 160000, 166
    ei, x, W, a_s, a_d, b = _problem(N, E, F, 11, dev)
    g = ggraph.csr_from_coo(ei.to(dev), N)
    xd, Wd, asd, add, bd = (t.to(dev) for t in (x, W, a_s, a_d, b))
    packed = gdist.pack_weights(Wd, asd, add)
    specs = [gdist.ShardSpec(g.rowptr, r, world) for r in range(world)]
    # use_xmax: the ranks' atomic max|x| accumulated into one tensor (= the
    # all-reduced value), tile stage with one Z-row scale
    xmax = torch.zeros(1, device=dev) if use_xmax else None
    st = torch.cat([gdist.shard_logits(xd, packed, s, xmax) for s in specs])
    if use_xmax:
        assert float(xmax) == float(xd.abs().max())
    out = torch.cat([gdist.shard_aggregate(xd, g, st, packed, bd, s, 0.2, xmax) for s in specs])
    torch.cuda.synchronize()
    expect = ref.gatconv_forward(x, ei, W, a_s, a_d, b, heads=H)
    assert_close(out, expect, what=f"{world} virtual ranks vs oracle")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_rccl_world1_end_to_end():
    import torch.distributed as dist
    from gfd import dist as gdist, graph as ggraph
    dev = torch.device("cuda", 0)
    N, E, F = 5000, 40000, 166
    ei, x, W, a_s, a_d, b = _problem(N, E, F, 12, dev)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        g = ggraph.csr_from_coo(ei.to(dev), N)
        # padded row pitch, as bench.py lays x out (168 floats for F = 166)
        xbuf = torch.zeros((N, 168), device=dev)
        xbuf[:, :F] = x.to(dev)
        spec = gdist.ShardSpec(g.rowptr, 0, 1)
        out = gdist.gat_conv_sharded(xbuf[:, :F], g, W.to(dev), a_s.to(dev), a_d.to(dev),
                                     b.to(dev), spec)
        torch.cuda.synchronize()
    finally:
        dist.destroy_process_group()
    assert_close(out, ref.gatconv_forward(x, ei, W, a_s, a_d, b, heads=H), what="RCCL world 1")


@pytest.mark.parametrize("balance", ["nodes", "messages"])
def test_exchange_tables_are_read_and_written_in_place(balance):
    """The hidden-layer exchange layout (gfd.dist.gather_hidden): a layer's
    input h and the next layer's s read as strided views of one [rows, 72]
    table, t from the own block's logits (stride 16), residual rows from the
    same view, and the aggregation writing its output rows straight into the
    rank's block of the next table (output row stride 72).  Every rank's rows
    must equal the contiguous-tensor call bit for bit, and the table's other
    columns must be left alone."""
    from gfd import dist as gdist, graph as ggraph
    from gfd.fused import bn_affine
    dev = torch.device("cuda", 0)
    N, E, F, world = 6000, 48000, 64, 3
    ei, x, W, a_s, a_d, b = _problem(N, E, F, 13, dev)
    g = ggraph.csr_from_coo(ei.to(dev), N)
    W, a_s, a_d, b = W.to(dev), a_s.to(dev), a_d.to(dev), b.to(dev)
    packed = gdist.pack_weights(W, a_s, a_d)
    bn = torch.nn.BatchNorm1d(64).to(dev).eval()
    with torch.no_grad():
        bn.running_mean.normal_()
        bn.running_var.uniform_(0.5, 2.0)
    aff = bn_affine(bn, dev)
    h = x.to(dev)
    st = gdist.logits_rows(h, packed, 0, N)
    specs = [gdist.ShardSpec(g.rowptr, r, world, balance) for r in range(world)]
    table = gdist.exchange_table(gdist.HID, specs[0], dev)
    table.fill_(float("nan"))
    table[:N, :64] = h
    table[:N, 64:] = st[:, :8]
    nxt = gdist.exchange_table(gdist.HID, specs[0], dev)
    nxt.fill_(7.0)
    for sp in specs:
        lo, hi = sp.dst_lo, sp.dst_hi
        want = gdist.shard_aggregate_ep(h, g, st, packed, b, sp, 0.2, None, aff, True, h[lo:hi])
        hv = table[:N, :64]
        tab = gdist.LogitsTable(table[:N, 64:], st[lo:hi, 8:])
        got = gdist.shard_aggregate_ep(hv, g, tab, packed, b, sp, 0.2, None, aff, True, hv[lo:hi],
                                       out=gdist.own_block(nxt, sp)[:, :64])
        torch.cuda.synchronize()
        assert got.data_ptr() == nxt[lo:].data_ptr()
        assert torch.equal(got, want), f"rank {sp.rank}: strided tables differ"
    assert torch.all(nxt[:N, 64:] == 7.0), "the s columns of the next table were written"


@pytest.mark.parametrize("cols,stride", [(8, 8), (8, 72), (72, 72), (5, 7)])
def test_rows_copy_gather_scatter(cols, stride):
    """gfd_rows_copy (the halo exchange's pack and scatter): gathered rows equal
    torch indexing bit for bit, scattered rows land at their node rows and no
    other row is written (16-B path: cols and strides multiples of 4; 4-B path
    otherwise); strided column views as the hidden-layer table uses."""
    from gfd import dist as gdist
    g = torch.Generator(device="cuda").manual_seed(5)
    n_rows, n = 10000, 3000
    base = torch.randn((n_rows, stride), generator=g, device="cuda")
    table = base[:, stride - cols:] if stride > cols else base
    idx = torch.randperm(n_rows, generator=g, device="cuda")[:n].to(torch.int32)
    buf = torch.empty((n, cols), device="cuda")
    gdist.rows_copy(table, idx, buf, None)
    torch.cuda.synchronize()
    assert torch.equal(buf, table[idx.long()])
    dst_base = torch.full((n_rows, stride), float("nan"), device="cuda")
    dst = dst_base[:, stride - cols:] if stride > cols else dst_base
    gdist.rows_copy(buf, None, dst, idx)
    torch.cuda.synchronize()
    assert torch.equal(dst[idx.long()], table[idx.long()])
    untouched = torch.ones(n_rows, dtype=torch.bool, device="cuda")
    untouched[idx.long()] = False
    assert torch.isnan(dst_base[untouched]).all()
    if stride > cols:
        assert torch.isnan(dst_base[:, :stride - cols]).all()


@pytest.mark.parametrize("world,balance", [(2, "messages"), (4, "cost"), (8, "nodes")])
def test_sharded_train_step_virtual_ranks(world, balance):
    """The sharded training step (gfd.dist "Sharded training") through the HIP
    kernels: each virtual rank runs gat_conv_local forward + backward on its
    LocalGraph (own destinations + halo sources), the ranks' partial parameter
    gradients are summed (what all_reduce_grads does over RCCL), and the sum
    must equal the whole-graph gradients; the outputs equal the whole-graph
    forward's rows.  Each rank's local graph is smaller than the whole graph."""
    from gfd import dist as gdist, graph as ggraph
    from gfd.nn import gat_conv
    dev = torch.device("cuda", 0)
    N, E, F = 20000, 160000, 166
    ei, x, W, a_s, a_d, b = _problem(N, E, F, 21, dev)
    graph = ggraph.csr_from_coo(ei.to(dev), N)
    xd = x.to(dev)
    gout = torch.randn(N, C, generator=torch.Generator().manual_seed(3)).to(dev)

    def leaf():
        return [t.to(dev).clone().requires_grad_(True) for t in (W, a_s, a_d, b)]

    full = leaf()
    out_full = gat_conv(xd, graph, *full, training=True)
    (out_full * gout).sum().backward()
    sh = leaf()
    spec = gdist.ShardSpec(graph.rowptr, 0, world, balance)
    outs = []
    for r in range(world):
        lo, hi = spec.dst_bounds[r], spec.dst_bounds[r + 1]
        lg = gdist.local_graph(graph, lo, hi)
        assert lg.graph.num_nodes < N and lg.n_dst == hi - lo
        o = gdist.gat_conv_local(xd, lg, *sh, training=True)
        (o * gout[lo:hi]).sum().backward()      # grads accumulate: the all-reduce's sum
        outs.append(o.detach())
    torch.cuda.synchronize()
    assert_close(torch.cat(outs), out_full.detach(), what=f"sharded outputs, world {world}")
    for name, a, bb in zip(("W", "att_src", "att_dst", "bias"), sh, full):
        err = (a.grad - bb.grad).abs().max().item()
        scale = bb.grad.abs().max().item()
        assert err <= 1e-4 * scale + 1e-6, f"{name}: {err:.3e} vs scale {scale:.3e} (world {world})"


@pytest.mark.parametrize("F,balance", [(64, "cost"), (166, "nodes")])
def test_halo_tables_never_touch_non_halo_rows(F, balance):
    """The halo exchange leaves every row outside a shard's own block and its
    halo unwritten: fill those rows of the exchange tables with
    NaN -- the [rows, 8] s table and, for a hidden layer, the [rows, 72]
    h | s table -- and the shard's aggregation through the HIP kernels
    (light slots' padding, clamped slots, hub chunks) must equal the
    full-table result bit for bit: no kernel reads a non-halo row."""
    from gfd import dist as gdist, graph as ggraph
    from gfd.fused import bn_affine
    dev = torch.device("cuda", 0)
    N, E, world = 8000, 64000, 3
    ei, x, W, a_s, a_d, b = _problem(N, E, F, 17, dev)
    g = ggraph.csr_from_coo(ei.to(dev), N)
    W, a_s, a_d, b = W.to(dev), a_s.to(dev), a_d.to(dev), b.to(dev)
    packed = gdist.pack_weights(W, a_s, a_d)
    aff = bn_affine(None, dev)
    h = x.to(dev)
    st = gdist.logits_rows(h, packed, 0, N)
    xmax = h.abs().max().reshape(1)
    for r in range(world):
        sp = gdist.ShardSpec(g.rowptr, r, world, balance)
        lo, hi = sp.dst_lo, sp.dst_hi
        need, _ = gdist.halo_needs(gdist.shard_columns(g, sp), sp)
        keep = torch.zeros(N, dtype=torch.bool, device=dev)
        keep[lo:hi] = True
        keep[need.long()] = True
        want = gdist.shard_aggregate_ep(h, g, st, packed, b, sp, 0.2, xmax, aff, True, None)
        # layer 0: x resident, the s table filled only on own + halo rows
        s_tab = torch.full((N, 8), float("nan"), device=dev)
        s_tab[keep] = st[keep, :8]
        got = gdist.shard_aggregate_ep(h, g, gdist.LogitsTable(s_tab, st[lo:hi, 8:]), packed, b,
                                       sp, 0.2, xmax, aff, True, None)
        torch.cuda.synchronize()
        assert torch.equal(got, want), f"rank {r}: the s table's non-halo rows were read"
        if F == 64:   # hidden layer: h and s from one [rows, 72] table
            tab = torch.full((N, gdist.HID), float("nan"), device=dev)
            tab[keep, :64] = h[keep]
            tab[keep, 64:] = st[keep, :8]
            hv = tab[:, :64]
            got = gdist.shard_aggregate_ep(hv, g, gdist.LogitsTable(tab[:, 64:], st[lo:hi, 8:]),
                                           packed, b, sp, 0.2, xmax, aff, True, None)
            torch.cuda.synchronize()
            assert torch.equal(got, want), f"rank {r}: the h table's non-halo rows were read"
