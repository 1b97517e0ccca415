"""Diagnostic: world-1 sharded model step vs the single-process GPU model,
per layer: conv outputs (forward) and their gradients."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "gnn-fraud-detection_amd"))
import torch
import torch.distributed as dist
import torch.nn.functional as Fn
import test_dist_model_train_gpu as T
from test_dist_cpu import _store_path
from gfd import dist as gdist, graph as ggraph


def run_sharded(model, x, y, mask, ei, dev):
    N = x.size(0)
    g = ggraph.csr_from_coo(ei.to(dev), N)
    spec = gdist.ShardSpec(g.rowptr.long(), 0, 1, "cost")
    lg = gdist.local_graph(g, 0, N)
    plan = gdist.HaloPlan.create(g.col, spec)
    zs = []

    def conv_fn(conv, xl, lgr, training):
        z = gdist.gat_conv_on_local(conv, xl, lgr, training)
        z.retain_grad()
        zs.append(z)
        return z
    logits = gdist.gat_forward_sharded_train(model, x, lg, plan, N, conv_fn=conv_fn).squeeze(-1)
    m = mask.to(dev)
    loss = Fn.binary_cross_entropy_with_logits(logits[m], y.to(dev)[m], reduction="sum") / int(mask.sum())
    loss.backward()
    return logits.detach(), zs


PLAIN_O = []


def run_plain(model, x, y, mask, ei, dev):
    """the sharded loop with torch BatchNorm (no collectives)"""
    from gfd.models import _head
    N = x.size(0)
    g = ggraph.csr_from_coo(ei.to(dev), N)
    lg = gdist.local_graph(g, 0, N)
    zs = []
    h = None
    for li, conv in enumerate(model.gat_layers):
        xl = lg.rows(x) if li == 0 else h
        z = gdist.gat_conv_on_local(conv, xl, lg, True)
        z.retain_grad()
        zs.append(z)
        ob = model.batch_norms[li](z)
        ob.retain_grad()
        PLAIN_O.append(ob)
        yy = Fn.relu(ob)
        h = xl + yy if xl.size(-1) == yy.size(-1) else yy
    logits = _head(model.out, h).squeeze(-1)
    m = mask.to(dev)
    loss = Fn.binary_cross_entropy_with_logits(logits[m], y.to(dev)[m])
    loss.backward()
    return logits.detach(), zs


def run_single(model, x, y, mask, ei, dev):
    zs = []

    def hook(mod, inp, out):
        out.retain_grad()
        zs.append(out)
    hs = [c.register_forward_hook(hook) for c in model.gat_layers]
    logits = model(x, ei.to(dev)).squeeze(-1)
    m = mask.to(dev)
    loss = Fn.binary_cross_entropy_with_logits(logits[m], y.to(dev)[m])
    loss.backward()
    for h in hs:
        h.remove()
    return logits.detach(), zs


def main():
    dev = torch.device("cuda", 0)
    dist.init_process_group("gloo", init_method=f"file://{_store_path()}", rank=0, world_size=1)
    ei, x, y, mask, model = T._problem()
    ma = model.to(dev)
    la, za = run_sharded(ma, x.to(dev), y, mask, ei, dev)
    ei, x, y, mask, model = T._problem()
    mb = model.to(dev)
    lb, zb = run_single(mb, x.to(dev), y, mask, ei, dev)
    print("logits max diff", (la - lb).abs().max().item())
    # layer-2 BN in isolation inside the sharded run: recompute dy from the
    # retained BN-output gradient and the retained input
    ei, x, y, mask, model = T._problem()
    md = model.to(dev)
    got = {}
    orig = gdist.sharded_batch_norm

    def bn_spy(yy, bn, n_total, group=None):
        o = orig(yy, bn, n_total, group)
        o.retain_grad()
        got.setdefault("o", []).append(o)
        got.setdefault("y", []).append(yy)
        return o
    gdist.sharded_batch_norm = bn_spy
    ld, zd = run_sharded(md, x.to(dev), y, mask, ei, dev)
    gdist.sharded_batch_norm = orig
    for i in range(3):
        o, yy = got["o"][i], got["y"][i]
        yl = yy.detach().clone().requires_grad_()
        bn2 = torch.nn.BatchNorm1d(64).to(dev)
        bn2.load_state_dict({k: v for k, v in md.batch_norms[i].state_dict().items()})
        bn2.running_mean.zero_(); bn2.running_var.fill_(1)
        (bn2(yl) * o.grad).sum().backward()
        print(f"layer {i}: recomputed dy vs z.grad {(yl.grad - zd[i].grad).abs().max().item():.3e} "
              f"scale {yl.grad.abs().max().item():.3e}; o.grad scale {o.grad.abs().max().item():.3e}")
    ei, x, y, mask, model = T._problem()
    mc = model.to(dev)
    lc, zc = run_plain(mc, x.to(dev), y, mask, ei, dev)
    for i, (a, b) in enumerate(zip(zc, zb)):
        print(f"plain layer {i}: z diff {(a - b).abs().max().item():.3e} "
              f"grad diff {(a.grad - b.grad).abs().max().item():.3e} (scale {b.grad.abs().max().item():.3e})")
    for i in range(3):
        a, b = got["o"][i], PLAIN_O[i]
        flips = int(((a > 0) != (b > 0)).sum())
        print(f"BN out layer {i}: diff {(a - b).abs().max().item():.3e} relu flips {flips} "
              f"grad diff {(a.grad - b.grad).abs().max().item():.3e} (scale {b.grad.abs().max().item():.3e}) "
              f"min|o| {b.abs().min().item():.3e}")
    for i, (a, b) in enumerate(zip(za, zc)):
        print(f"sharded vs plain layer {i}: grad diff {(a.grad - b.grad).abs().max().item():.3e}")
    for i, (a, b) in enumerate(zip(za, zb)):
        print(f"layer {i}: z diff {(a - b).abs().max().item():.3e} (scale {b.abs().max().item():.3e}) "
              f"grad diff {(a.grad - b.grad).abs().max().item():.3e} (scale {b.grad.abs().max().item():.3e})")
    for (k, p), (_, q) in zip(ma.named_parameters(), mb.named_parameters()):
        s = q.grad.abs().max().item()
        print(f"{k:36s} {((p.grad - q.grad).abs().max().item()) / max(s, 1e-30):.2e}")
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
