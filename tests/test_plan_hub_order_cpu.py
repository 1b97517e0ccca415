"""CPU: gfd.graph._hubs_by_size -- the hubs of a plan renumbered by descending
message count (the chunk launch order of k_hub_partial), on a node-order hub
split built here the way gfd_plan_hubs builds it (k_hub_flags / k_hub_write in
csrc/gfd_graph.hip).  The GPU tests run the renumbered plans through every
kernel that reads them (forward hubs, backward hub chunks, sharded plans)."""
import torch

from gfd.graph import _hubs_by_size


def _node_order_hubs(deg, thr, chunk):
    rowptr = torch.zeros(len(deg) + 1, dtype=torch.int32)
    rowptr[1:] = torch.cumsum(torch.tensor(deg, dtype=torch.int32), 0)
    hub_rank = torch.full((len(deg),), -1, dtype=torch.int32)
    chunks, ptr, dst = [], [0], []
    for i, d in enumerate(deg):
        if d <= thr:
            continue
        h = len(dst)
        hub_rank[i] = h
        dst.append(i)
        b, e = int(rowptr[i]), int(rowptr[i + 1])
        for p in range(b, e, chunk):
            chunks += [h, p, min(p + chunk, e), i]
        ptr.append(len(chunks) // 4)
    return (rowptr, hub_rank, torch.tensor(chunks, dtype=torch.int32),
            torch.tensor(ptr, dtype=torch.int32), torch.tensor(dst, dtype=torch.int32),
            len(dst), len(chunks) // 4)


def test_hubs_renumbered_by_descending_size_keep_every_chunk():
    g = torch.Generator().manual_seed(3)
    deg = (torch.rand(400, generator=g) ** 6 * 2000).long().clamp(min=1).tolist()
    deg[7] = deg[11] = 700          # equal sizes keep node order (stable)
    rowptr, rank0, ck0, ptr0, dst0, nh, nc = _node_order_hubs(deg, 128, 384)
    assert nh > 5
    rank, ck, ptr, dst, nh2, nc2 = _hubs_by_size(rowptr, rank0, ck0, ptr0, dst0, nh, nc)
    assert (nh2, nc2) == (nh, nc)
    size = (rowptr[dst.long() + 1] - rowptr[dst.long()]).tolist()
    assert size == sorted(size, reverse=True)
    assert dst.tolist().index(7) < dst.tolist().index(11)
    ck = ck.view(-1, 4)
    old = ck0.view(-1, 4)
    assert sorted(map(tuple, ck[:, 1:].tolist())) == sorted(map(tuple, old[:, 1:].tolist()))
    for k in range(nh):
        i = int(dst[k])
        assert int(rank[i]) == k
        rows = ck[int(ptr[k]):int(ptr[k + 1])]
        assert (rows[:, 0] == k).all() and (rows[:, 3] == i).all()
        # the hub's chunks in their original order (its merged row bit-identical)
        h0 = int(rank0[i])
        assert rows[:, 1:].tolist() == old[int(ptr0[h0]):int(ptr0[h0 + 1]), 1:].tolist()
    assert int(ptr[-1]) == nc
    non = [i for i in range(len(deg)) if deg[i] <= 128]
    assert (rank[non] == -1).all()


def test_single_hub_and_no_hub_plans_pass_through():
    rowptr, rank0, ck0, ptr0, dst0, nh, nc = _node_order_hubs([3, 500, 2], 128, 384)
    out = _hubs_by_size(rowptr, rank0, ck0, ptr0, dst0, nh, nc)
    assert out[0] is rank0 and out[1] is ck0
    rowptr, rank0, ck0, ptr0, dst0, nh, nc = _node_order_hubs([3, 5, 2], 128, 384)
    assert _hubs_by_size(rowptr, rank0, ck0, ptr0, dst0, nh, nc)[4] == 0
