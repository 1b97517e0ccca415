"""Per-rank time of the destination-sharded TRAINING step of a GATConv layer
(train.py:115-143 on the sharded variant; gfd.dist "Sharded training"),
measured one rank at a time on ONE GPU (show the per-rank
backward shrinking with the rank count; the driver's 8-GPU run is the real
measurement, and it times bench.py's forward).

For each world W in --worlds and each rank r of it: the rank's LocalGraph of
the C4 graph (own destinations + the halo sources its messages read, the halo
rows with only their self loop; gfd.dist.local_graph), x gathered into the
local order once (gfd.dist.LocalGraph.rows, outside the timing, as a constant
layer input is), then the rank's layer forward in training mode (softmax
statistics kept) and its backward (grad W, att, bias; no grad_x: layer 0) on
those rows -- gfd_gat_fwd / gfd_gat_bwd through gfd.nn.gat_conv.  HIP events,
median over --steps.  The one all-reduce of the 0.35 MB of parameter
gradients and the halo exchange are not in these numbers (no peers here).
Prints one JSON line: per world, per rank (rows, messages, fwd / bwd ms) and
the max over ranks, beside the whole graph's fwd / bwd.

    python scripts/virtual_ranks_train.py [--worlds 1,2,4,8] [--balance nodes]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "gnn-fraud-detection_amd"))

import torch  # noqa: E402

import bench  # noqa: E402


def _median(xs):
    xs = sorted(xs)
    return xs[len(xs) // 2]


def time_fwd_bwd(x_loc, graph, n_dst, params, steps, warmup):
    from gfd.nn import gat_conv
    W, a_s, a_d, b = params
    dev = x_loc.device
    grad = torch.randn((n_dst, 64), device=dev, generator=torch.Generator(device=dev).manual_seed(4))
    graph.csc()
    graph.plan()
    fw, bw = [], []
    for i in range(warmup + steps):
        for p in params:
            p.grad = None
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        e0.record()
        out = gat_conv(x_loc, graph, W, a_s, a_d, b, dropout=0.0, training=True)
        e1.record()
        out[:n_dst].backward(grad)
        e2.record()
        torch.cuda.synchronize()
        if i >= warmup:
            fw.append(e0.elapsed_time(e1))
            bw.append(e1.elapsed_time(e2))
    return _median(fw), _median(bw)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--worlds", default="1,2,4,8")
    p.add_argument("--balance", choices=["nodes", "messages", "cost"], default="nodes")
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--nodes", type=int, default=10_000_000)
    p.add_argument("--edges", type=int, default=50_000_000)
    a = p.parse_args()
    from gfd import dist as gdist
    dev = torch.device("cuda", 0)
    s = bench.setup(dev, a.nodes, a.edges, 166)
    g = s["graph"]
    params = [s[k].clone().requires_grad_(True) for k in ("W", "a_s", "a_d", "bias")]
    res = {"workload": f"C4 GATConv layer 0 training step (fwd with softmax stats + bwd: grad W, "
                       f"att, bias), N={g.num_nodes} E={g.num_input_edges}, per rank of a "
                       f"destination-sharded world ({a.balance}-balanced), one rank at a time on "
                       f"one GPU; collectives not included",
           "device": torch.cuda.get_device_name(dev), "worlds": {}}
    for world in [int(w) for w in a.worlds.split(",")]:
        ranks = []
        for r in range(world):
            if world == 1:
                x_loc, graph, n_dst = s["x"], g, g.num_nodes
                rows, msgs = g.num_nodes, g.num_messages
            else:
                spec = gdist.ShardSpec(g.rowptr, r, world, a.balance)
                lg = gdist.local_graph(g, spec.dst_lo, spec.dst_hi)
                x_loc, graph, n_dst = lg.rows(s["x"]), lg.graph, lg.n_dst
                rows, msgs = graph.num_nodes, graph.num_messages
            fwd_ms, bwd_ms = time_fwd_bwd(x_loc, graph, n_dst, params, a.steps, a.warmup)
            ranks.append({"rank": r, "own_rows": n_dst, "local_rows": rows, "messages": msgs,
                          "fwd_ms": round(fwd_ms, 3), "bwd_ms": round(bwd_ms, 3),
                          "step_ms": round(fwd_ms + bwd_ms, 3)})
            print(f"world {world} rank {r}: {ranks[-1]}", file=sys.stderr, flush=True)
            del x_loc, graph
            torch.cuda.empty_cache()
        slow = max(ranks, key=lambda q: q["step_ms"])
        res["worlds"][str(world)] = {"ranks": ranks, "max_step_ms": slow["step_ms"],
                                     "max_fwd_ms": max(q["fwd_ms"] for q in ranks),
                                     "max_bwd_ms": max(q["bwd_ms"] for q in ranks)}
    w1 = res["worlds"].get("1")
    if w1:
        for w, d in res["worlds"].items():
            d["speedup_vs_1"] = round(w1["max_step_ms"] / d["max_step_ms"], 2)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
