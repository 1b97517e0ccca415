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
