#!/usr/bin/env python3
"""bench.py -- GATConv layer-0 forward throughput on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[3]): synthetic Chung-Lu
power-law graph, N = 10M nodes, E = 50M input edges (gamma 2.1, seed 1),
x ~ N(0,1) fp32 [N, 166], glorot weights (seed 0), GATConv(166 -> 64, heads=8,
concat=False) forward with self loops, eval mode.  One step = one full layer
forward: weight packing + per-node logits + hub chunks + fused
softmax-aggregate-project tiles, inputs already resident in HBM.

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...   (destination-sharded)

value = input edges of the whole graph per second (all ranks together); the
timed region is bracketed by barrier + synchronize, max over ranks.
Rank 0 prints ONE JSON line with ``roofline`` (dominant kernel: the tile stage,
``k_stream`` for F <= 168, timed live with HIP events on the launch stream) and
``cpu_baseline`` (the oracle's PyG-dataflow restatement on a bounded sample,
host cores of the same box, N=1 only).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "gnn-fraud-detection_amd"))

import torch  # noqa: E402

METRIC = "edges/sec GAT forward (166-feat, 8 heads); achieved HBM GB/s vs peak"
HBM_PEAK_GBPS = 8000.0        # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
BF16_PEAK_TFLOPS = 2500.0     # dense bf16 MFMA
H, C = 8, 64


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--nodes", type=int, default=10_000_000)
    p.add_argument("--edges", type=int, default=50_000_000)
    p.add_argument("--features", type=int, default=166)
    p.add_argument("--gamma", type=float, default=2.1)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-nodes", type=int, default=1_000_000)
    p.add_argument("--cpu-edges", type=int, default=5_000_000)
    p.add_argument("--pmc", default=os.path.join(REPO, "profiles", "pmc_summary.json"))
    return p.parse_args()


def glorot(shape, gen, device):
    a = math.sqrt(6.0 / (shape[-2] + shape[-1]))
    return (torch.rand(shape, generator=gen) * 2 * a - a).to(device)


def cpu_baseline(args):
    """Oracle (PyG CPU dataflow) on a bounded sample of the same generator."""
    import numpy as np
    from gfd import synth
    from oracle import gatconv_forward_chunked
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)
    torch.set_num_threads(threads)
    n, e, F = args.cpu_nodes, args.cpu_edges, args.features
    ei = torch.from_numpy(synth.power_law(n, e, gamma=args.gamma, seed=1))
    x = torch.from_numpy(np.random.default_rng(0).standard_normal((n, F), dtype=np.float32))
    gen = torch.Generator().manual_seed(0)
    W = glorot((H * C, F), gen, "cpu")
    a_s = glorot((1, H, C), gen, "cpu")
    a_d = glorot((1, H, C), gen, "cpu")
    b = torch.zeros(C)
    keep = ei[0] != ei[1]
    src = torch.cat([ei[0][keep], torch.arange(n)])
    dst = torch.cat([ei[1][keep], torch.arange(n)])
    order = torch.argsort(dst, stable=True)
    rowptr = torch.zeros(n + 1, dtype=torch.long)
    rowptr[1:] = torch.cumsum(torch.bincount(dst, minlength=n), 0)
    col = src[order]
    times = []
    with torch.no_grad():
        for _ in range(3):  # 1 warm-up + 2 timed (~10-15 s of CPU work on 16 cores)
            t0 = time.perf_counter()
            gatconv_forward_chunked(x, rowptr, col, W, a_s, a_d, b, heads=H, chunk_edges=4_000_000)
            times.append(time.perf_counter() - t0)
    t = sum(times[1:]) / len(times[1:])
    return {"value": e / t, "unit": "edges/s", "cores": threads, "kind": "port",
            "seconds": round(t, 3),
            "sample": f"C4 generator at N={n}, E={e} (gamma {args.gamma}, seed 1), F={F}, "
                      "layer-0 forward, eval, oracle/gatconv_ref.py PyG CPU dataflow "
                      "(Linear -> index_select -> scatter_reduce(amax) -> exp -> index_add), "
                      "dst chunks of 4M messages; 1 warm-up + mean of 2 timed runs"}


def tile_kernel_name(F):
    """The tile-stage kernel gfd_gat_aggregate launches (GFD_TILE_KERNEL, F)."""
    tk = int(os.environ.get("GFD_TILE_KERNEL", "0"))
    if tk == 0 and (F + 7) // 8 * 8 <= 168:
        return "k_stream (weight-stationary tile stage)"
    return {2: "k_persist", 3: "k_tile32", 4: "k_pair"}.get(tk, "k_fused") + " (tile stage)"


def load_pmc(path, workload_key):
    try:
        with open(path) as f:
            d = json.load(f)
        ent = d.get(workload_key)
        if ent:
            return ent
    except (OSError, ValueError):
        pass
    return None


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local if world > 1 else 0)
    torch.cuda.set_device(dev)

    from gfd import _lib, dist as gdist, graph as ggraph, synth
    lib = _lib.load()
    N, E, F = args.nodes, args.edges, args.features
    t_setup = time.perf_counter()
    ei = synth.power_law_device(N, E, gamma=args.gamma, seed=1, device=dev)
    g = ggraph.csr_from_coo(ei, N)
    del ei
    torch.cuda.empty_cache()
    gx = torch.Generator(device=dev).manual_seed(0)
    LDX = (F + 3) // 4 * 4  # row pitch 168 for F = 166 (16-B aligned rows)
    xbuf = torch.randn((N, LDX), generator=gx, device=dev, dtype=torch.float32)
    x = xbuf[:, :F]
    gen = torch.Generator().manual_seed(0)
    W = glorot((H * C, F), gen, dev).contiguous()
    a_s = glorot((1, H, C), gen, dev).contiguous()
    a_d = glorot((1, H, C), gen, dev).contiguous()
    bias = torch.zeros(C, device=dev)

    spec = gdist.ShardSpec(g.rowptr, rank, world)   # dst shard + logits node block
    lo, hi = spec.dst_lo, spec.dst_hi
    shard = g.shard(lo, hi)
    plan = shard.plan
    n_dst = hi - lo
    m_local = int(shard.rowptr[-1].item()) - int(shard.rowptr[0].item())
    st_lo, st_hi = spec.node_lo, spec.node_hi

    packed = torch.empty(lib.gfd_gat_packed_size(F, H, C), dtype=torch.uint8, device=dev)
    st = torch.empty((N, 2 * H), dtype=torch.float32, device=dev)
    st_local = torch.empty((max(st_hi - st_lo, 1), 2 * H), dtype=torch.float32, device=dev)
    out = torch.empty((max(n_dst, 1), C), dtype=torch.float32, device=dev)
    ws = torch.empty(lib.gfd_gat_fwd_workspace_size(N, n_dst, F, H, C, plan.num_hubs,
                                                    plan.num_chunks), dtype=torch.uint8, device=dev)
    stream = _lib.stream_handle(dev)
    cplan = plan.cstruct()

    xmax = torch.zeros(1, dtype=torch.float32, device=dev)   # max |x| (one Z-row scale)

    def pack_and_logits():
        _lib.call("gfd_gat_pack_weights", W.data_ptr(), a_s.data_ptr(), a_d.data_ptr(), F, H, C,
                  packed.data_ptr(), stream)
        xmax.zero_()
        if world == 1:
            _lib.call("gfd_gat_logits_ex", x.data_ptr(), N, F, LDX, packed.data_ptr(), H, C,
                      st.data_ptr(), xmax.data_ptr(), stream)
        else:
            rows = st_hi - st_lo
            if rows > 0:
                _lib.call("gfd_gat_logits_ex", x[st_lo:].data_ptr(), rows, F, LDX,
                          packed.data_ptr(), H, C, st_local.data_ptr(), xmax.data_ptr(), stream)
            st.copy_(gdist.all_gather_rows(st_local[:rows], N, world))
            dist.all_reduce(xmax, op=dist.ReduceOp.MAX)

    def aggregate(stage):
        _lib.call("gfd_gat_aggregate_ex", x.data_ptr(), N, F, LDX, shard.rowptr.data_ptr(),
                  g.col.data_ptr(), n_dst, lo, st.data_ptr(), xmax.data_ptr(), packed.data_ptr(),
                  bias.data_ptr(), H, C, 0.2, 0.0, 0, cplan, stage, out.data_ptr(), None,
                  ws.data_ptr(), ws.numel(), stream)

    def step(evs=None):
        if evs:
            evs[0].record()
        pack_and_logits()
        if evs:
            evs[1].record()
        aggregate(1)
        if evs:
            evs[2].record()
        aggregate(2)
        if evs:
            evs[3].record()

    log(f"[bench] rank {rank}/{world}: N={N} E={E} messages={g.num_messages} shard=[{lo},{hi}) "
        f"local msgs={m_local} hubs={plan.num_hubs} chunks={plan.num_chunks} "
        f"setup {time.perf_counter() - t_setup:.1f}s")
    for _ in range(args.warmup):
        step()
    # events record on torch's current stream == the stream every gfd launch uses
    events = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(args.steps)]
    torch.cuda.synchronize()
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(events[k])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if os.environ.get("GFD_PROF_DUMP") and hasattr(lib, "gfd_debug_prof"):
        import ctypes
        buf = (ctypes.c_ulonglong * 32)()
        lib.gfd_debug_prof(buf)
        names = {0: "mfma", 1: "barrier1", 2: "reduce", 8: "wait-rows", 9: "agg-compute",
                 3: "agg-epilogue0", 4: "agg-epilogue1", 19: "pair-light", 18: "drain", 16: "issue0", 17: "issue1",
                 5: "records", 6: "barrier2"}
        tot = sum(buf[i] for i in names)
        log("[bench] k_stream phase cycles (summed over waves): " + ", ".join(
            f"{n} {buf[i] / max(tot, 1) * 100:.1f}%" for i, n in names.items()) +
            f"; per tile-wave {tot / max(buf[7], 1):.0f} cyc")
        log("[bench] k_stream slot cycles by degree: " + ", ".join(
            f"{n}: {buf[i + 1]} slots x {buf[i] / max(buf[i + 1], 1):.0f} cyc"
            for i, n in ((10, "deg<=4"), (12, "deg 5-8"), (14, "deg>8"))))
    pre_ms = [e[0].elapsed_time(e[1]) for e in events]
    hub_ms = [e[1].elapsed_time(e[2]) for e in events]
    tile_ms = [e[2].elapsed_time(e[3]) for e in events]
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())

    # ---- numbers ----
    ms_step = elapsed * 1e3 / args.steps
    value = E * args.steps / elapsed
    s = 4  # bytes per feature element (fp32)
    M = g.num_messages
    B_layer = M * (s * F + 4) + N * (4 + 4 * C) + 4 * F * H * C
    flop_layer = 2 * N * F * H * C + M * H * (2 * C + 8)
    t_roof = max(B_layer / (HBM_PEAK_GBPS * 1e9), flop_layer / (BF16_PEAK_TFLOPS * 1e12))
    # dominant kernel = the tile stage on this rank (k_stream for F <= 168, else k_fused):
    # the light messages + all its rows
    hub_msgs = plan.hub_messages()
    light_msgs = m_local - hub_msgs
    B_tile = light_msgs * (s * F + 4) + n_dst * (4 + 4 * C) + 4 * F * H * C
    t_tile = sorted(tile_ms)[len(tile_ms) // 2] * 1e-3
    achieved = B_tile / t_tile / 1e9
    workload = (f"C4 power-law N={N} E={E} F={F} gamma={args.gamma}: GATConv layer-0 forward "
                f"(H=8, C=64, concat=False, self loops)")
    pmc = load_pmc(args.pmc, f"tile:N={N}:E={E}:F={F}:world={world}")
    traffic = pmc.get("hbm_bytes_per_launch") if pmc else None

    res = {
        "metric": METRIC, "value": value, "unit": "edges/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms_step,
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic (Chung-Lu power-law graph on device, seed 1; x ~ N(0,1) seed 0; "
                "glorot weights seed 0)",
        "config": {"workload": workload, "nodes": N, "input_edges": E, "messages": M,
                   "features": F, "heads": H, "channels": C,
                   "parallelism": f"dst-shard x{world}" if world > 1 else "single GPU",
                   "hubs": plan.num_hubs, "hub_chunks": plan.num_chunks},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBPS, "traffic": traffic,
                     "kernel": tile_kernel_name(F), "algorithmic_bytes": B_tile,
                     "kernel_ms": t_tile * 1e3},
        "layer": {"algorithmic_bytes": B_layer, "flop": flop_layer,
                  "hbm_gbps": B_layer / (ms_step * 1e-3) / 1e9,
                  "t_roof_ms": t_roof * 1e3, "roofline_frac": t_roof / (ms_step * 1e-3),
                  "stage_ms": {"pack+logits": sorted(pre_ms)[len(pre_ms) // 2],
                               "hubs": sorted(hub_ms)[len(hub_ms) // 2],
                               "tiles": sorted(tile_ms)[len(tile_ms) // 2]}},
        "cpu_baseline": None,
    }
    if world == 1 and rank == 0 and not args.no_cpu_baseline:
        del x, xbuf, out, ws, st, g
        torch.cuda.empty_cache()
        log("[bench] timing CPU baseline (oracle, bounded sample) ...")
        res["cpu_baseline"] = cpu_baseline(args)
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
