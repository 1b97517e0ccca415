"""The graph cache of the drop-in path (gfd.graph.get_graph) in the reference's
training loop shape: a new device copy of the same edge_index every epoch
(``batch.to(device)``, /root/reference/src/train.py:105).  With speculation
on, the steady-state lookup does not synchronise the host (VERDICT r4 weak
#8), and a copy with different edges at a reused address is detected."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True)
def speculation():
    from gfd import graph as gg
    prev = gg.set_speculation(True)
    yield
    gg.set_speculation(prev)
    gg.clear_cache()


def _edges(n, e, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.randint(0, n, (2, e), generator=g)


def test_reference_loop_lookups_are_sync_free_in_steady_state():
    from gfd import graph as gg
    gg.clear_cache()
    host = _edges(5000, 20000, 0)
    graphs, spec = [], []
    batch = None
    for _ in range(12):                     # the reference's epoch loop
        before = gg.STATS["speculated"]
        batch = host.to(DEV)                # new tensor every epoch; the old one dies here
        graphs.append(gg.get_graph(batch, 5000))
        spec.append(gg.STATS["speculated"] - before)
    torch.cuda.synchronize()
    gg.sync_pending_checks()               # every speculated hit verified on the device
    assert all(g is graphs[0] for g in graphs)
    # the allocator cycles a few addresses; once each has held the edges
    # SPECULATE_AFTER times (each checked by the synchronous fingerprint), every
    # later epoch is a sync-free lookup
    assert spec[-4:] == [1, 1, 1, 1], spec


def test_changed_edges_at_a_reused_address_raise():
    from gfd import graph as gg
    gg.clear_cache()
    host = _edges(3000, 9000, 1)
    a = host.to(DEV)
    g1 = gg.get_graph(a, 3000)
    ptr = a.data_ptr()
    for _ in range(gg.SPECULATE_AFTER):     # the same edges verified at this address
        del a
        a = host.to(DEV)
        if a.data_ptr() != ptr:
            pytest.skip("the allocator did not reuse the block")
        assert gg.get_graph(a, 3000) is g1
    del a
    b = _edges(3000, 9000, 2).to(DEV)       # same shape, different edges
    if b.data_ptr() != ptr:
        pytest.skip("the allocator did not reuse the block")
    g2 = gg.get_graph(b, 3000)              # speculated (no sync) ...
    assert g2 is g1
    torch.cuda.synchronize()
    with pytest.raises(gg.GraphChangedError):
        gg.sync_pending_checks()            # ... and caught by the device-side check
    # the object entry the speculated hit made is gone too: the
    # same tensor, looked up again, is fingerprinted and gets its own graph
    gb = gg.get_graph(b, 3000)
    assert gb is not g1
    assert torch.equal(gb.col, gg.csr_from_coo(b, 3000).col)
    # the address entry is gone: the next lookup takes the fingerprint path
    c = b.clone()
    del b
    g3 = gg.get_graph(c, 3000)
    assert g3 is not g1
    assert torch.equal(g3.rowptr, gg.csr_from_coo(c, 3000).rowptr)
    gg.clear_cache()


def test_different_graphs_at_one_address_never_speculate():
    """Different same-shaped graphs allocated one after another (e.g. test
    cases) land on one address but never twice with the same edges."""
    from gfd import graph as gg
    gg.clear_cache()
    before = gg.STATS["speculated"]
    for seed in range(5):
        e = _edges(2500, 8000, 10 + seed).to(DEV)
        gr = gg.get_graph(e, 2500)
        assert torch.equal(gr.col, gg.csr_from_coo(e, 2500).col)
        del e, gr
    assert gg.STATS["speculated"] == before
    gg.sync_pending_checks()
    gg.clear_cache()


def test_speculation_off_always_fingerprints():
    from gfd import graph as gg
    gg.set_speculation(False)
    gg.clear_cache()
    host = _edges(4000, 12000, 7)
    before = dict(gg.STATS)
    batch = None
    for _ in range(6):
        batch = host.to(DEV)
        gg.get_graph(batch, 4000)
    d = {k: gg.STATS[k] - before[k] for k in gg.STATS}
    assert d["speculated"] == 0 and d["fingerprint"] == 6, d


def test_no_content_cache_edge_lists_never_speculate():
    from gfd import graph as gg
    gg.clear_cache()
    a = _edges(2000, 6000, 3).to(DEV)
    gg.get_graph(a, 2000)
    ptr = a.data_ptr()
    del a
    b = gg.no_content_cache(_edges(2000, 6000, 3).to(DEV))
    before = gg.STATS["speculated"]
    gg.get_graph(b, 2000)
    assert gg.STATS["speculated"] == before or b.data_ptr() != ptr
    gg.clear_cache()
