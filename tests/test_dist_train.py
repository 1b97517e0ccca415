"""Sharded training step of a GATConv layer on CPU with gloo (train.py:115-143
on the destination-sharded variant; gfd.dist "Sharded training").

Each rank builds the LocalGraph of its destination shard (own destinations,
then the halo sources with only their self loop), runs the layer forward and
backward on it (oracle arithmetic in place of the HIP kernels, which need a
GPU; tests/test_dist_gpu.py runs the kernels), and the partial parameter
gradients are all-reduced: the result must equal the single-process
gradients of the whole graph."""
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from _util import assert_close_scaled, csr_cpu
from test_dist_cpu import _problem, _store_path, N, F, H, C
from gfd import dist as gdist
from gfd.graph import CSRGraph
from oracle import gatconv_ref as ref


def _graph_cpu(ei):
    rowptr, col = csr_cpu(ei, N)
    return CSRGraph(N, rowptr.to(torch.int32), col.to(torch.int32), int(rowptr[-1]), ei.size(1))


def _local_coo(lg):
    """The LocalGraph's messages as a COO edge list without self loops (the
    oracle re-adds one per node, as the local CSR holds)."""
    rp, col = lg.graph.rowptr.long(), lg.graph.col.long()
    n = lg.graph.num_nodes
    dst = torch.repeat_interleave(torch.arange(n), rp[1:] - rp[:-1])
    keep = col != dst
    return torch.stack([col[keep], dst[keep]])


def _grad_out():
    return torch.randn(N, C, generator=torch.Generator().manual_seed(9))


def _train_rank(rank, world, path, balance, q):
    dist.init_process_group("gloo", init_method=f"file://{path}", rank=rank, world_size=world)
    try:
        ei, x, W, a_s, a_d, b = _problem()
        g = _graph_cpu(ei)
        spec = gdist.ShardSpec(g.rowptr.long(), rank, world, balance)
        lg = gdist.local_graph(g, spec.dst_lo, spec.dst_hi)
        params = [t.clone().requires_grad_(True) for t in (W, a_s, a_d, b)]
        x_loc = lg.rows(x)
        out = ref.gatconv_forward(x_loc, _local_coo(lg), *params, heads=H)[:lg.n_dst]
        (out * _grad_out()[spec.dst_lo:spec.dst_hi]).sum().backward()
        gdist.all_reduce_grads(params)
        if rank == 0:
            q.put(([p.grad.numpy() for p in params], lg.graph.num_nodes, lg.n_dst))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,balance", [(2, "messages"), (3, "cost"), (2, "nodes")])
def test_sharded_train_step_matches_single_process(world, balance):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    path = _store_path()
    procs = [ctx.Process(target=_train_rank, args=(r, world, path, balance, q))
             for r in range(world)]
    for p in procs:
        p.start()
    grads, n_loc, n_dst = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ei, x, W, a_s, a_d, b = _problem()
    params = [t.clone().requires_grad_(True) for t in (W, a_s, a_d, b)]
    out = ref.gatconv_forward(x, ei, *params, heads=H)
    (out * _grad_out()).sum().backward()
    for name, got, p in zip(("W", "att_src", "att_dst", "bias"), grads, params):
        assert_close_scaled(torch.from_numpy(got), p.grad, rtol=2e-5,
                            what=f"sharded {name} grad, world {world} ({balance})")
    assert n_dst < N and n_loc < N + 1   # rank 0's local rows: own block + halo, not all N


def test_local_graph_structure():
    ei, x, *_ = _problem()
    g = _graph_cpu(ei)
    rowptr = g.rowptr.long()
    deg = rowptr[1:] - rowptr[:-1]
    for lo, hi in ((0, 200), (150, 420), (480, N)):
        lg = gdist.local_graph(g, lo, hi)
        nodes = lg.nodes
        assert torch.equal(nodes[:hi - lo], torch.arange(lo, hi))
        assert nodes.unique().numel() == nodes.numel()
        lrp = lg.graph.rowptr.long()
        ldeg = lrp[1:] - lrp[:-1]
        # own rows keep every message in order (global ids through the node map)
        assert torch.equal(ldeg[:hi - lo], deg[lo:hi])
        own = lg.graph.col[:int(lrp[hi - lo])].long()
        assert torch.equal(nodes[own], g.col[int(rowptr[lo]):int(rowptr[hi])].long())
        # halo rows: their own self loop only, and exactly the sources read
        assert bool((ldeg[hi - lo:] == 1).all())
        halo_col = lg.graph.col[int(lrp[hi - lo]):].long()
        assert torch.equal(halo_col, torch.arange(hi - lo, nodes.numel()))
        src = g.col[int(rowptr[lo]):int(rowptr[hi])].long()
        want = torch.unique(src[(src < lo) | (src >= hi)])
        assert torch.equal(nodes[hi - lo:], want)
        assert lg.graph.num_messages == int(lrp[-1])
        # constant x: gathered once per version
        a = lg.rows(x)
        assert lg.rows(x) is a and torch.equal(a, x[nodes])


# ---------------------------------------------------------------------------
# The whole model (gat.py:60-96, train.py:115-143): three GATConv layers with
# BatchNorm, ReLU and the residual, sharded by destination.  Hidden layers
# receive their halo rows through gdist.halo_rows (and send the halo rows'
# gradients back to the owners), BatchNorm takes all ranks' rows
# (gdist.sharded_batch_norm), and the loss is each rank's share of the
# labelled-node mean.  fp64 throughout, so the comparison is tight.

LAYERS = 3


def _model_problem():
    ei, x, *_ = _problem()
    g = torch.Generator().manual_seed(11)
    y = (torch.rand(N, generator=g) < 0.2).double()
    mask = torch.rand(N, generator=g) < 0.6
    torch.manual_seed(3)
    from gfd.models import GAT
    model = GAT(F, C, 1, num_layers=LAYERS, dropout=0.0).double().train()
    with torch.no_grad():   # non-trivial BN affine parameters
        for bn in model.batch_norms:
            bn.weight.uniform_(0.5, 1.5)
            bn.bias.uniform_(-0.2, 0.2)
    return ei, x.double(), y, mask, model


def _oracle_conv(conv, x_local, lg, training):
    return ref.gatconv_forward(x_local, _local_coo(lg), conv.lin_src.weight, conv.att_src,
                               conv.att_dst, conv.bias, heads=H)[:lg.n_dst]


def _reference_step(ei, x, y, mask, model):
    import torch.nn.functional as Fn
    h = x
    for li, conv in enumerate(model.gat_layers):
        z = ref.gatconv_forward(h, ei, conv.lin_src.weight, conv.att_src, conv.att_dst,
                                conv.bias, heads=H)
        z = Fn.relu(model.batch_norms[li](z))
        h = h + z if h.size(-1) == z.size(-1) else z
    logits = model.out(h).squeeze(-1)
    loss = Fn.binary_cross_entropy_with_logits(logits[mask], y[mask])
    loss.backward()
    return loss.item()


def _model_rank(rank, world, path, balance, q):
    import torch.nn.functional as Fn
    dist.init_process_group("gloo", init_method=f"file://{path}", rank=rank, world_size=world)
    try:
        ei, x, y, mask, model = _model_problem()
        g = _graph_cpu(ei)
        spec = gdist.ShardSpec(g.rowptr.long(), rank, world, balance)
        lo, hi = spec.dst_lo, spec.dst_hi
        lg = gdist.local_graph(g, lo, hi)
        rp = g.rowptr.long()
        plan = gdist.HaloPlan.create(g.col[int(rp[lo]):int(rp[hi])], spec)
        logits = gdist.gat_forward_sharded_train(model, x, lg, plan, N,
                                                 conv_fn=_oracle_conv).squeeze(-1)
        m = mask[lo:hi]
        part = Fn.binary_cross_entropy_with_logits(logits[m], y[lo:hi][m], reduction="sum")
        loss = part / int(mask.sum())
        loss.backward()
        gdist.all_reduce_grads(list(model.parameters()))
        tot = loss.detach().clone()
        dist.all_reduce(tot)
        # eval mode after the step: BatchNorm on the (all-rank) running statistics
        model.eval()
        with torch.no_grad():
            ev = gdist.gat_forward_sharded_train(model, x, lg, plan, N, conv_fn=_oracle_conv)
        full = gdist.all_gather_v_rows(ev.contiguous(), spec.dst_bounds)
        if rank == 0:
            q.put(({k: p.grad.numpy() for k, p in model.named_parameters()},
                   {k: b.numpy() for k, b in model.named_buffers()}, tot.item(),
                   plan.recv_rows.numel(), full.numpy()))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,balance", [(2, "messages"), (3, "cost")])
def test_sharded_model_train_step_matches_single_process(world, balance):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    path = _store_path()
    procs = [ctx.Process(target=_model_rank, args=(r, world, path, balance, q))
             for r in range(world)]
    for p in procs:
        p.start()
    grads, bufs, loss, n_halo, eval_logits = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ei, x, y, mask, model = _model_problem()
    want_loss = _reference_step(ei, x, y, mask, model)
    assert abs(loss - want_loss) <= 1e-12 * max(1.0, abs(want_loss))
    assert n_halo > 0   # the hidden layers really exchanged rows
    for k, p in model.named_parameters():
        # atol: a GATConv bias feeding a train-mode BatchNorm has a zero gradient
        assert_close_scaled(torch.from_numpy(grads[k]), p.grad, rtol=1e-10, atol=1e-13,
                            what=f"sharded model grad {k}, world {world} ({balance})")
    for k, b in model.named_buffers():
        if b.dtype.is_floating_point:
            assert_close_scaled(torch.from_numpy(bufs[k]), b, rtol=1e-10,
                                what=f"BN buffer {k}, world {world}")
        else:
            assert int(bufs[k]) == int(b)
    # the eval forward of the updated buffers, sharded vs whole graph
    model.eval()
    with torch.no_grad():
        h = x
        for li, conv in enumerate(model.gat_layers):
            z = ref.gatconv_forward(h, ei, conv.lin_src.weight, conv.att_src, conv.att_dst,
                                    conv.bias, heads=H)
            z = torch.relu(model.batch_norms[li](z))
            h = h + z if h.size(-1) == z.size(-1) else z
        want = model.out(h)
    assert_close_scaled(torch.from_numpy(eval_logits), want, rtol=1e-10,
                        what=f"sharded eval logits, world {world}")


# ---------------------------------------------------------------------------
# all_reduce_grads with ranks that disagree about which gradients
# exist, and sharded_batch_norm without an affine transform.

def _advice_rank(rank, world, path, q):
    dist.init_process_group("gloo", init_method=f"file://{path}", rank=rank, world_size=world)
    try:
        # rank 1 never touched the second parameter (its grad is None there)
        ps = [torch.zeros(3, requires_grad=True), torch.zeros(2, requires_grad=True),
              torch.zeros(4, requires_grad=True)]
        ps[0].grad = torch.full((3,), float(rank + 1))
        if rank == 0:
            ps[1].grad = torch.tensor([5.0, 7.0])
        ps[2].grad = torch.arange(4.0) * (rank + 1)
        gdist.all_reduce_grads(ps)
        # BatchNorm1d(affine=False) on this rank's rows of a 2-rank batch
        gen = torch.Generator().manual_seed(3)
        y_all = torch.randn(10, 4, generator=gen, dtype=torch.float64)
        rows = y_all[:6] if rank == 0 else y_all[6:]
        y = rows.clone().requires_grad_(True)
        bn = torch.nn.BatchNorm1d(4, affine=False).double()
        out = gdist.sharded_batch_norm(y, bn, 10)
        g_all = torch.randn(10, 4, generator=gen, dtype=torch.float64)
        (out * (g_all[:6] if rank == 0 else g_all[6:])).sum().backward()
        q.put((rank, [p.grad.clone() for p in ps], out.detach(), y.grad.clone(),
               bn.running_mean.clone(), bn.running_var.clone()))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_all_reduce_grads_missing_grads_and_bn_without_affine():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    path = _store_path()
    procs = [ctx.Process(target=_advice_rank, args=(r, 2, path, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r[0], r[1:]) for r in (q.get(timeout=180), q.get(timeout=180)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank in (0, 1):
        grads = res[rank][0]
        assert torch.equal(grads[0], torch.full((3,), 3.0))
        assert torch.equal(grads[1], torch.tensor([5.0, 7.0]))   # rank 1's None counted as 0
        assert torch.equal(grads[2], torch.arange(4.0) * 3)
    gen = torch.Generator().manual_seed(3)
    y_all = torch.randn(10, 4, generator=gen, dtype=torch.float64).requires_grad_(True)
    bn = torch.nn.BatchNorm1d(4, affine=False).double()
    ref_out = bn(y_all)
    g_all = torch.randn(10, 4, generator=gen, dtype=torch.float64)
    (ref_out * g_all).sum().backward()
    out = torch.cat([res[0][1], res[1][1]])
    gy = torch.cat([res[0][2], res[1][2]])
    assert torch.allclose(out, ref_out.detach(), atol=1e-12)
    assert torch.allclose(gy, y_all.grad, atol=1e-12)
    for rank in (0, 1):
        assert torch.allclose(res[rank][3], bn.running_mean, atol=1e-12)
        assert torch.allclose(res[rank][4], bn.running_var, atol=1e-12)
