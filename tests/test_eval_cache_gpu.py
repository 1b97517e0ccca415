"""GPU: inference with cached packed weights (gfd.fused.eval_weights, the
gfd_gat_fwd_ep_packed entry of ABI 6).  The drop-in module's no_grad forward
and the fused model layers pack a layer's weights once and reuse them while no
source tensor changes: results bit-identical to the per-call packing path, and
an in-place update, a replaced parameter or new BatchNorm statistics rebuild
the cache."""
import pytest
import torch

from test_gatconv_gpu import _random_case

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _per_call(conv, x, graph):
    """The autograd path (gfd_gat_fwd packs inside every call)."""
    from gfd.nn import GATConvFunction
    return GATConvFunction.apply(x, conv.lin_src.weight, conv.att_src.reshape(-1),
                                 conv.att_dst.reshape(-1), conv.bias, graph,
                                 conv.negative_slope, 0.0, 0, False)


def test_module_no_grad_forward_uses_cached_pack_and_tracks_parameters():
    from gfd import graph as gg
    from gfd.nn import GATConv
    x_cpu, ei, ref = _random_case(4000, 30000, 166, seed=8, kind="powerlaw")
    conv = GATConv(166, 64, heads=8, concat=False).to(DEV).eval()
    conv.load_state_dict({k: v.to(DEV) for k, v in ref.state_dict().items()}, strict=False)
    x = x_cpu.to(DEV)
    graph = gg.get_graph(ei.to(DEV), 4000)
    with torch.no_grad():
        a = conv(x, graph)
        packed = conv.__dict__["_gfd_eval"][1]
        b = conv(x, graph)
        assert conv.__dict__["_gfd_eval"][1] is packed          # reused
        want = _per_call(conv, x, graph)
        assert torch.equal(a, want) and torch.equal(b, want)
        conv.lin_src.weight.mul_(1.01)                          # in place: new version
        c = conv(x, graph)
        assert conv.__dict__["_gfd_eval"][1] is not packed
        assert torch.equal(c, _per_call(conv, x, graph)) and not torch.equal(c, a)
        conv.att_src = torch.nn.Parameter(conv.att_src.detach() * 0.5)   # a new object
        d = conv(x, graph)
        assert torch.equal(d, _per_call(conv, x, graph)) and not torch.equal(d, c)


def test_fused_layers_rebuild_on_new_batchnorm_statistics():
    from gfd import graph as gg
    from gfd.models import GAT
    x_cpu, ei, _ = _random_case(3000, 20000, 165, seed=9, kind="elliptic")
    m = GAT(165, 64, 1, num_layers=3, dropout=0.0).to(DEV).eval()
    x, graph = x_cpu.to(DEV), gg.get_graph(ei.to(DEV), 3000)
    with torch.no_grad():
        a = m(x, graph)
        b = m(x, graph)
        assert torch.equal(a, b)
        m.batch_norms[1].running_mean.add_(0.3)                 # new statistics (in place)
        c = m(x, graph)
    assert not torch.equal(a, c)
    m2 = GAT(165, 64, 1, num_layers=3, dropout=0.0).to(DEV).eval()
    m2.load_state_dict(m.state_dict())
    with torch.no_grad():
        assert torch.equal(m2(x, graph), c)                     # fresh caches agree


def test_module_parameters_on_the_wrong_device_or_dtype_raise():
    """the packed-weights inference path checks the layer's own
    tensors (device, dtype) before their pointers reach a kernel."""
    from gfd import graph as gg
    from gfd.nn import GATConv
    x_cpu, ei, _ = _random_case(600, 3000, 166, seed=3, kind="powerlaw")
    x = x_cpu.to(DEV)
    graph = gg.get_graph(ei.to(DEV), 600)
    conv = GATConv(166, 64, heads=8, concat=False).eval()        # left on the CPU
    with torch.no_grad():
        with pytest.raises(RuntimeError, match="HIP device"):
            conv(x, graph)
        conv = conv.to(DEV).double()                               # wrong dtype
        with pytest.raises(TypeError, match="float32"):
            conv(x, graph)
        conv = conv.float()
        conv.bias.data = conv.bias.data.cpu()                     # one tensor left behind
        with pytest.raises(RuntimeError, match="bias"):
            conv(x, graph)
