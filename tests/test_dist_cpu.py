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
            q.put((st, out, spec.dst_bounds, st_x, (spec.dst_lo, spec.dst_hi)))
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
