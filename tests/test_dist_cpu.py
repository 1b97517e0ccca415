"""Destination-sharded data flow on CPU with gloo, world_size 2.

Each rank computes the attention logits of its node block, the blocks are
all-gathered, each rank computes its destination shard (oracle arithmetic in
place of the HIP kernels) and the uneven output shards are all-gathered: the
result must equal the single-process forward.  This is the exchange pattern
bench.py and gfd.dist.gat_conv_sharded run over RCCL on the GPUs.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from _util import assert_close, csr_cpu
from gfd import dist as gdist
from oracle import gatconv_ref as ref

N, E, F, H, C = 600, 4000, 23, 8, 64


def _problem():
    g = torch.Generator().manual_seed(5)
    # power-law-ish destinations so shards are uneven in node count
    w = torch.arange(1, N + 1, dtype=torch.float64) ** -0.8
    dst = torch.multinomial(w, E, replacement=True, generator=g)
    src = torch.randint(0, N, (E,), generator=g)
    ei = torch.stack([src, dst])
    x = torch.randn(N, F, generator=g)
    W = ref.glorot_(torch.empty(H * C, F), g)
    a_s = ref.glorot_(torch.empty(1, H, C), g)
    a_d = ref.glorot_(torch.empty(1, H, C), g)
    b = torch.randn(C, generator=g) * 0.1
    return ei, x, W, a_s, a_d, b


def _logits(x, W, a_s, a_d):
    h = (x @ W.t()).view(-1, H, C)
    return torch.cat([(h * a_s).sum(-1), (h * a_d).sum(-1)], 1)


def _store_path():
    import tempfile
    fd, path = tempfile.mkstemp(prefix="gfd_gloo_")
    os.close(fd)
    os.unlink(path)  # the FileStore creates it
    return path


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, q):
    # file rendezvous: no TCP port to race for (a freed ephemeral port can be
    # taken again before rank 0 binds it)
    dist.init_process_group("gloo", init_method=f"file://{port}", rank=rank, world_size=world)
    try:
        ei, x, W, a_s, a_d, b = _problem()
        rowptr, col = csr_cpu(ei, N)
        spec = gdist.ShardSpec(rowptr, rank, world)
        st_local = _logits(x[spec.node_lo:spec.node_hi], W, a_s, a_d)
        st = gdist.all_gather_rows(st_local, N, world)
        # the product exchange: s of every node gathered, [s | t] of the own destinations
        st_x = gdist.exchange_logits(x, None, spec,
                                     logits_fn=lambda lo, hi: _logits(x[lo:hi], W, a_s, a_d)).st(spec)
        out_local = ref.gatconv_forward_at(x, rowptr, col, torch.arange(spec.dst_lo, spec.dst_hi),
                                           W, a_s, a_d, b)
        out = gdist.all_gather_v_rows(out_local, spec.dst_bounds)
        if rank == 0:
            # by value: a tensor would travel as a shared-memory handle that its
            # sender's exit can invalidate before the parent unpickles it
            q.put((st.numpy(), out.numpy(), spec.dst_bounds, st_x.numpy(),
                   (spec.dst_lo, spec.dst_hi)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_forward_matches_single_process(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _store_path()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    st, out, bounds, st_x, (d_lo, d_hi) = q.get(timeout=120)
    st, out, st_x = torch.from_numpy(st), torch.from_numpy(out), torch.from_numpy(st_x)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ei, x, W, a_s, a_d, b = _problem()
    full_st = _logits(x, W, a_s, a_d)
    assert_close(st, full_st, what="gathered logits")
    assert_close(st_x[:, :H], full_st[:, :H], what="exchanged source logits")
    assert_close(st_x[d_lo:d_hi], full_st[d_lo:d_hi], what="own destinations' [s | t]")
    full = ref.gatconv_forward(x, ei, W, a_s, a_d, b, heads=H)
    assert_close(out, full, what=f"sharded forward, world {world}")
    # the shards really are uneven in destinations but balanced in messages
    rowptr, _ = csr_cpu(ei, N)
    msgs = [int(rowptr[bounds[r + 1]] - rowptr[bounds[r]]) for r in range(world)]
    assert max(msgs) - min(msgs) <= int((rowptr[1:] - rowptr[:-1]).max())
    assert len({bounds[r + 1] - bounds[r] for r in range(world)}) > 1


def test_edge_balanced_bounds_properties():
    ei, *_ = _problem()
    rowptr, _ = csr_cpu(ei, N)
    for parts in (1, 2, 5, 8, N + 3):
        b = gdist.edge_balanced_bounds(rowptr, parts)
        assert b[0] == 0 and b[-1] == N
        assert len(b) == (parts + 1 if parts > 1 else 2)
        assert all(b[k] <= b[k + 1] for k in range(len(b) - 1))
    empty = torch.zeros(1, dtype=torch.long)
    assert gdist.edge_balanced_bounds(empty, 4) == [0, 0]


def test_node_bounds_cover():
    for n, p in ((10, 3), (7, 8), (0, 2), (1024, 8)):
        b = gdist.node_bounds(n, p)
        assert b[0] == 0 and b[-1] == n and len(b) == p + 1
        assert all(b[k] <= b[k + 1] for k in range(p))


def _halo_main(rank, world, path, balance, q):
    dist.init_process_group("gloo", init_method=f"file://{path}", rank=rank, world_size=world)
    try:
        ei, x, W, a_s, a_d, b = _problem()
        rowptr, col = csr_cpu(ei, N)
        spec = gdist.ShardSpec(rowptr, rank, world, balance)
        shard_col = col[int(rowptr[spec.dst_lo]):int(rowptr[spec.dst_hi])]
        plan = gdist.HaloPlan.create(shard_col, spec)
        full = _logits(x, W, a_s, a_d)[:, :H].contiguous()
        # a node-row table with only the own rows set (the fused logits pass's
        # output); the halo exchange fills in exactly the rows the shard reads
        table = torch.full((N, H), float("nan"))
        table[spec.dst_lo:spec.dst_hi] = full[spec.dst_lo:spec.dst_hi]
        plan.exchange(table)
        need = torch.unique(shard_col.long())
        ok_rows = bool(torch.equal(table[need], full[need]))
        # the same exchange in two row-range phases (bench's overlapped form)
        table2 = torch.full((N, H), float("nan"))
        table2[spec.dst_lo:spec.dst_hi] = full[spec.dst_lo:spec.dst_hi]
        for part in plan.split(spec, 2):
            part.exchange_async(table2)()
        ok_rows = ok_rows and bool(torch.equal(table2[need], full[need]))
        untouched = torch.ones(N, dtype=torch.bool)
        untouched[need] = False
        untouched[spec.dst_lo:spec.dst_hi] = False
        stale = bool(torch.isnan(table[untouched]).all())
        # the shard's aggregation over the halo-filled table matches the oracle
        out_local = ref.gatconv_forward_at(x, rowptr, col, torch.arange(spec.dst_lo, spec.dst_hi),
                                           W, a_s, a_d, b)
        q.put((rank, ok_rows, stale, plan.recv_counts, plan.send_counts,
               int(plan.recv_rows.numel()), out_local.numpy(), (spec.dst_lo, spec.dst_hi)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,balance", [(2, "nodes"), (3, "messages"), (4, "nodes"),
                                           (3, "cost")])
def test_halo_exchange_delivers_exactly_the_rows_a_shard_reads(world, balance):
    """gfd.dist.HaloPlan over gloo: the plan's all-to-alls of counts and ids,
    then one exchange of the source-logit rows -- every row a shard's messages
    read arrives bit-exact, no other row is written, rank q's sends to r are
    r's requests from q, and the rows received are a fraction of the others'."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    path = _store_path()
    procs = [ctx.Process(target=_halo_main, args=(r, world, path, balance, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok_rows, stale, rc, sc, nrecv, _, (lo, hi) in res:
        assert ok_rows, f"rank {rank}: halo rows"
        assert stale, f"rank {rank}: wrote rows outside its halo"
        assert rc[rank] == 0 and sc[rank] == 0 and sum(rc) == nrecv
        for peer in range(world):
            assert res[peer][4][rank] == rc[peer], "sends to r = r's requests"
        assert nrecv < N - (hi - lo)
    ei, x, W, a_s, a_d, b = _problem()
    full = ref.gatconv_forward(x, ei, W, a_s, a_d, b, heads=H)
    for rank, *_, out_local, (lo, hi) in res:
        assert_close(torch.from_numpy(out_local), full[lo:hi], what=f"halo shard {rank} of {world}")


def test_cost_balanced_bounds_equalise_the_modelled_time():
    """balance="cost": contiguous, monotone ranges covering every destination,
    each within one destination's cost of the mean modelled time -- and a
    graph with a few heavy hubs is split unevenly in nodes to do it."""
    from gfd import synth
    N = 50_000
    ei = torch.from_numpy(synth.power_law(N, 250_000, seed=3))
    rowptr, _ = csr_cpu(ei, N)
    cost = gdist.destination_costs(rowptr)
    for world in (2, 3, 8):
        b = gdist.ShardSpec(rowptr, 0, world, "cost").dst_bounds
        assert b[0] == 0 and b[-1] == N and all(b[k] <= b[k + 1] for k in range(world))
        parts = [float(cost[b[r]:b[r + 1]].sum()) for r in range(world)]
        mean = sum(parts) / world
        assert max(abs(p - mean) for p in parts) <= float(cost.max()) + 1e-9
    sizes = {b[r + 1] - b[r] for r in range(8)}
    assert len(sizes) > 1
