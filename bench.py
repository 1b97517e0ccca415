#!/usr/bin/env python3
"""bench.py -- GATConv layer-0 forward throughput on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[3]): synthetic Chung-Lu
power-law graph, N = 10M nodes, E = 50M input edges (gamma 2.1, seed 1),
x ~ N(0,1) fp32 [N, 166] at row pitch 168, glorot weights (seed 0),
GATConv(166 -> 64, heads=8, concat=False) forward with self loops, eval mode.
One step = one full layer forward: weight packing + per-node logits + hub
chunks + the class-scheduled tile stage (general / light / lone kernels),
inputs already resident in HBM.

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...   (destination-sharded)
    python bench.py --config c5        (bf16 features, 50M / 500M, one line)

value = input edges of the whole graph per second (all ranks together); the
timed region is bracketed by barrier + synchronize, max over ranks.  Rank 0
prints ONE JSON line with ``roofline`` (the dominant kernel of the step, timed
live with HIP events on the launch stream), ``kernels`` (every stage),
``cpu_baseline`` (the oracle's PyG-dataflow restatement on a bounded sample of
the same C4 graph, host cores of the same box, N = 1 only) and ``legs`` (the
config-5 bf16 forward at N = 1).
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
BF16_PEAK_TFLOPS = 2500.0     # dense bf16/f16 MFMA (the projection runs on f16 MFMA)
H, C = 8, 64
STAGE_HUBS, STAGE_MID, STAGE_LIGHT, STAGE_LONE = 1, 4, 8, 16


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=None,
                   help="ranks (one per GPU); > 1 without torchrun launches them itself")
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--config", choices=["c4", "c5"], default="c4")
    p.add_argument("--nodes", type=int, default=None)
    p.add_argument("--edges", type=int, default=None)
    p.add_argument("--features", type=int, default=166)
    p.add_argument("--gamma", type=float, default=2.1)
    p.add_argument("--row-align", type=int, default=None,
                   help="byte alignment of x rows (16: fp32 pitch 176 with the s slot; 128: "
                        "whole cache lines).  Default: 16 for C4, 128 for C5 (bf16 rows: "
                        "measured -1.6 ms at C5, +0.1 ms at C4)")
    p.add_argument("--balance", choices=["nodes", "messages", "cost"], default="cost",
                   help="N > 1 destination shards: ranges balanced by the modelled "
                        "per-destination stage time (default; C4 x8 rank by rank: slowest "
                        "rank 2.03 ms against 2.06 for equal node blocks), equal node blocks "
                        "(C4's ids are randomly permuted: messages within 2.6 %% at 8 ranks) "
                        "or message-balanced ranges")
    p.add_argument("--overlap", action="store_true",
                   help="run the light class on a second stream beside hubs -> general")
    p.add_argument("--exchange", choices=["halo", "halo1", "allgather"], default="halo",
                   help="N > 1 source-logits exchange: each rank receives only the rows its "
                        "messages read (RCCL all-to-all; ~22 %% of the other ranks' nodes at "
                        "C4 x8), in two phases whose first runs under the second half of the "
                        "logits pass (halo) or in one after it (halo1); or every node's "
                        "(allgather)")
    p.add_argument("--rehearse", action="store_true",
                   help="N > 1 ranks on however many GPUs are visible (rank -> GPU rank %% "
                        "count), gloo host-staged exchange: exercises the launcher and the "
                        "per-rank path on a 1-GPU box; NOT a scaling measurement")
    p.add_argument("--no-s-in-row", action="store_true",
                   help="keep the source logits in their own [N, 16] table instead of an "
                        "8-float slot in every x row")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-legs", action="store_true")
    p.add_argument("--legs", default="c4bwd,dropin,sample,c5,c1,c2,c3,temporal,ingest",
                   help="comma list of legs run after the headline line (N = 1)")
    p.add_argument("--legs-only", action="store_true",
                   help="skip the C4 headline timing (development)")
    p.add_argument("--cpu-messages", type=int, default=3_000_000,
                   help="messages in the CPU-baseline sample of the C4 graph")
    p.add_argument("--cpu-runs", type=int, default=5)
    p.add_argument("--pmc", default=os.path.join(REPO, "profiles", "pmc_summary.json"))
    return p.parse_args(argv)


def glorot(shape, gen, device):
    a = math.sqrt(6.0 / (shape[-2] + shape[-1]))
    return (torch.rand(shape, generator=gen) * 2 * a - a).to(device)


def setup(dev, nodes, edges, F=166, gamma=2.1, dtype=torch.float32, rank=0, world=1,
          row_align=16, balance="nodes", s_in_row=True):
    """The bench workload, built on the device exactly as timed: Chung-Lu
    graph (seed 1) -> CSR, x ~ N(0,1) (seed 0) at a 16-B row pitch, glorot W
    (seed 0), zero bias, this rank's destination shard and its cached plan.
    ``s_in_row``: every x row carries an 8-float slot for its node's source
    logits s_j after the features (16-B aligned), written by the logits pass
    and read by the gather kernels through gfd_gat_aggregate_split's (s,
    s_stride) -- so a message's s_j comes from the line its x row's gather
    fetches anyway instead of a line of its own (fp32 F = 166: pitch 176, the
    slot at 168; bf16: pitch 184, the slot at 168).  The features x = xbuf[:, :F]
    are unchanged.  Also used by tests/test_bench_parity_gpu.py."""
    from gfd import dist as gdist, graph as ggraph, synth
    ei = synth.power_law_device(nodes, edges, gamma=gamma, seed=1, device=dev)
    g = ggraph.csr_from_coo(ei, nodes)
    del ei
    torch.cuda.empty_cache()
    gx = torch.Generator(device=dev).manual_seed(0)
    esz = torch.tensor([], dtype=dtype).element_size()
    # rows aligned to row_align bytes: 16 -> pitch 168 for F = 166; 128 -> whole
    # 128-B lines per row (pitch 192: fp32 6 lines, bf16 3 lines per gathered row)
    s_off = (F * esz + 15) // 16 * 16                      # byte offset of the s slot
    row_bytes = s_off + 4 * H if s_in_row else F * esz
    ldx = (row_bytes + row_align - 1) // row_align * row_align // esz
    xbuf = torch.randn((nodes, ldx), generator=gx, device=dev, dtype=torch.float32).to(dtype)
    x = xbuf[:, :F]
    gen = torch.Generator().manual_seed(0)
    W = glorot((H * C, F), gen, dev).contiguous()
    a_s = glorot((1, H, C), gen, dev).contiguous()
    a_d = glorot((1, H, C), gen, dev).contiguous()
    bias = torch.zeros(C, device=dev)
    spec = gdist.ShardSpec(g.rowptr, rank, world, balance)   # the rank's destinations
    shard = g.shard(spec.dst_lo, spec.dst_hi)
    return {"graph": g, "x": x, "xbuf": xbuf, "ldx": ldx, "W": W, "a_s": a_s, "a_d": a_d,
            "bias": bias, "spec": spec, "shard": shard, "dtype": dtype, "F": F,
            # the s slot as a float pointer offset and float row stride (or None)
            "s_row": (s_off // 4, ldx * esz // 4) if s_in_row else None}


class Layer:
    """One GATConv layer-0 forward through the C ABI, split into timed stages."""

    def __init__(self, s, dev, world, exchange="halo"):
        from gfd import _lib
        self.s, self.dev, self.world = s, dev, world
        self.lib = _lib.load()
        self._lib = _lib
        g, x, F, spec = s["graph"], s["x"], s["F"], s["spec"]
        self.N = g.num_nodes
        self.xdt = _lib.x_dtype_code(x)
        self.n_dst = spec.dst_hi - spec.dst_lo
        self.plan = s["shard"].plan
        self.packed = torch.empty(self.lib.gfd_gat_packed_size(F, H, C), dtype=torch.uint8,
                                  device=dev)
        # whole graph: one [N, 16] logits table.  A shard (N > 1, or the tests'
        # virtual shards): the split layout of gfd_gat_aggregate_split -- s of
        # every node in s_all [N, 8] (rank r's rows at its destination block,
        # so the all-gather-v of the source logits writes straight into the
        # table the kernels read: no scatter between collective and kernels),
        # t of the own destinations in t_loc [n_dst, 8]
        self.st = torch.empty((self.N, 2 * H), dtype=torch.float32, device=dev)
        b = spec.dst_bounds
        # equal blocks (node balance): rank r's rows r*per .. are its nodes, the
        # table padded to world*per rows; uneven blocks: views at their rows
        self.equal = all(b[r] == r * spec.per for r in range(world))
        rows = world * spec.per if self.equal else self.N
        self.s_all = torch.empty((max(rows, self.N), H), dtype=torch.float32, device=dev)
        self.t_loc = torch.empty((max(self.n_dst, 1), H), dtype=torch.float32, device=dev)
        self.s_blocks = ([self.s_all[r * spec.per:(r + 1) * spec.per] for r in range(world)]
                         if self.equal else [self.s_all[b[r]:b[r + 1]] for r in range(world)])
        self.out = torch.empty((max(self.n_dst, 1), C), dtype=torch.float32, device=dev)
        self.ws = torch.empty(self.lib.gfd_gat_fwd_workspace_size(
            self.N, self.n_dst, F, H, C, self.plan.num_hubs, self.plan.num_chunks),
            dtype=torch.uint8, device=dev)
        self.xmax = torch.zeros(1, dtype=torch.float32, device=dev)
        # max |x| over ALL rows (the tile stage's one Z-row scale) is a property
        # of the input, like the CSR and the plan: computed by the first step's
        # logits passes and all-reduced once per x version, then kept
        # (it was all-reduced every step)
        self._xmax_key = None
        self.stream = _lib.stream_handle(dev)
        self.overlap = False   # --overlap (set by measure): light on a second stream
        self.side = torch.cuda.Stream(device=dev)
        self._ready = torch.cuda.Event()
        self.cplan = self.plan.cstruct()
        # the lone destinations' outputs come out of the logits pass
        # (gfd_gat_logits_lone over the rank's destinations) and the tile stage
        # skips that class -- whole graph or shard, at every world size
        self.whole = spec.dst_lo == 0 and spec.dst_hi == self.N and world == 1
        self.stages = self.STAGES_FUSED if world == 1 else self.STAGES_SHARDED
        # whole graph with an s slot in every x row: s written into the rows by
        # the logits pass, t into t_loc, both read through the split ABI
        self.in_row = self.whole and s.get("s_row") is not None
        if self.in_row:
            off, self.lds = s["s_row"]
            self.s_ptr = s["xbuf"].data_ptr() + 4 * off
        # N > 1, halo exchange: the other ranks' rows this shard's messages read
        # (plan built once here, by two all-to-alls of counts and row ids)
        self.halo = None
        self.halo_parts = None   # "halo": the two row-range phases of the exchange
        self.pending = []
        if world > 1 and exchange in ("halo", "halo1"):
            from gfd import dist as gdist
            lo, hi = int(g.rowptr[spec.dst_lo].item()), int(g.rowptr[spec.dst_hi].item())
            self.halo = gdist.HaloPlan.create(g.col[lo:hi], spec)
            if exchange == "halo":
                self.halo_parts = self.halo.split(spec, 2)

    def logits_table(self):
        """[N, 16] s | t of the last step (tests): from the row slots or st."""
        if not self.in_row:
            return self.st
        off, lds = self.s["s_row"]
        rows = self.s["xbuf"].view(torch.float32).view(self.N, lds)   # bf16 rows: as bytes
        return torch.cat([rows[:, off:off + H], self.t_loc[:self.N]], 1)

    def pack_and_logits(self):
        s, _lib, F = self.s, self._lib, self.s["F"]
        _lib.call("gfd_gat_pack_weights", s["W"].data_ptr(), s["a_s"].data_ptr(),
                  s["a_d"].data_ptr(), F, H, C, self.packed.data_ptr(), self.stream)
        if not self.xmax_current():
            self.xmax.zero_()   # (kept: the passes' atomic max of the same rows changes nothing)
        x, spec = s["x"], s["spec"]
        if self.in_row:
            _lib.call("gfd_gat_logits_lone_split", x.data_ptr(), self.xdt, self.N, F, s["ldx"],
                      self.packed.data_ptr(), H, C, s["shard"].rowptr.data_ptr(),
                      s["bias"].data_ptr(), 0.2, self.s_ptr, self.lds, self.t_loc.data_ptr(), H,
                      self.xmax.data_ptr(), self.out.data_ptr(), C, None, self.stream)
            return
        if self.whole:
            _lib.call("gfd_gat_logits_lone", x.data_ptr(), self.xdt, self.N, F, s["ldx"],
                      self.packed.data_ptr(), H, C, s["shard"].rowptr.data_ptr(),
                      s["bias"].data_ptr(), 0.2, self.st.data_ptr(), self.xmax.data_ptr(),
                      self.out.data_ptr(), None, self.stream)
            return
        # a shard: s | t and the lone outputs of the own destinations in one
        # pass, s straight into the rank's block of s_all.  The tests' virtual
        # shards on one GPU (world 1) take the other rows' s from a logits pass
        # over every row (the all-gather's stand-in, untimed by bench)
        n = self.n_dst
        if self.world == 1:
            _lib.call("gfd_gat_logits_ex", x.data_ptr(), self.xdt, self.N, F, s["ldx"],
                      self.packed.data_ptr(), H, C, self.st.data_ptr(), self.xmax.data_ptr(),
                      self.stream)
            self.s_all.copy_(self.st[:, :H])

        def logits(a, b):   # own destinations a..b (local rows)
            if b > a:
                lo = spec.dst_lo + a
                _lib.call("gfd_gat_logits_lone_split", x[lo:].data_ptr(), self.xdt, b - a, F,
                          s["ldx"], self.packed.data_ptr(), H, C,
                          s["shard"].rowptr[a:].data_ptr(), s["bias"].data_ptr(), 0.2,
                          self.s_all[lo:].data_ptr(), H, self.t_loc[a:].data_ptr(), H,
                          self.xmax.data_ptr(), self.out[a:].data_ptr(), C, None, self.stream)
        if self.halo_parts is not None:
            # phase k of the halo exchange leaves as soon as its rows' logits are
            # written; phase 0's collective runs under the second half's pass
            self.pending = []
            cut = [n * k // len(self.halo_parts) for k in range(len(self.halo_parts) + 1)]
            for k, part in enumerate(self.halo_parts):
                logits(cut[k], cut[k + 1])
                self.pending.append(part.exchange_async(self.s_all))
            return
        logits(0, n)

    def xmax_current(self) -> bool:
        x = self.s["x"]
        return self._xmax_key == (x.data_ptr(), x._version)

    def exchange(self):
        # ONE all-gather-v of the [N, 8] source logits (RCCL; uneven blocks land
        # at their node rows) and, once per x version, the max |x| reduction the
        # tile stage's row scale needs
        import torch.distributed as dist
        r = self.s["spec"].rank
        reduce_xmax = not self.xmax_current()
        self._xmax_key = (self.s["x"].data_ptr(), self.s["x"]._version)
        if self.halo is not None:
            # the rows this shard reads, straight into s_all (gfd_rows_copy pack,
            # RCCL all-to-all, gfd_rows_copy scatter; gloo: host-staged); the
            # phased form was issued by pack_and_logits and is completed here
            if self.halo_parts is not None:
                for finish in self.pending:
                    finish()
                self.pending = []
            else:
                self.halo.exchange(self.s_all)
            if not reduce_xmax:
                return
            if dist.get_backend() == "gloo":
                xm = self.xmax.cpu()
                dist.all_reduce(xm, op=dist.ReduceOp.MAX)
                self.xmax.copy_(xm)
            else:
                dist.all_reduce(self.xmax, op=dist.ReduceOp.MAX)
            return
        if dist.get_backend() == "gloo":   # --rehearse: the same exchange, host-staged
            # (equal blocks: one in-place all-gather; uneven blocks, e.g. the
            # default cost balance: gather_blocks' padded gloo path -- ADVICE r4)
            from gfd import dist as gdist
            cpu = self.s_all.cpu()
            gdist.gather_blocks(cpu, self.s["spec"])
            self.s_all.copy_(cpu)
            if reduce_xmax:
                xm = self.xmax.cpu()
                dist.all_reduce(xm, op=dist.ReduceOp.MAX)
                self.xmax.copy_(xm)
            return
        if self.equal:
            # s_all IS the gathered layout: in place, one RCCL all-gather
            dist.all_gather_into_tensor(self.s_all[:len(self.s_blocks) * self.s_blocks[0].shape[0]],
                                        self.s_blocks[r])
        else:  # uneven blocks (RCCL grouped broadcasts into the row views)
            dist.all_gather(self.s_blocks, self.s_blocks[r])
        if reduce_xmax:
            dist.all_reduce(self.xmax, op=dist.ReduceOp.MAX)

    def aggregate(self, stages, stream=None):
        s = self.s
        st_h = self.stream if stream is None else stream
        if self.in_row:
            self._lib.call("gfd_gat_aggregate_split", s["x"].data_ptr(), self.xdt, self.N, s["F"],
                           s["ldx"], s["shard"].rowptr.data_ptr(), s["graph"].col.data_ptr(),
                           self.n_dst, 0, self.s_ptr, self.lds, self.t_loc.data_ptr(), H,
                           self.xmax.data_ptr(), self.packed.data_ptr(), s["bias"].data_ptr(), H,
                           C, 0.2, 0.0, 0, self.cplan, stages, None, self.out.data_ptr(), C, None,
                           self.ws.data_ptr(), self.ws.numel(), st_h)
            return
        if self.whole:
            self._lib.call("gfd_gat_aggregate_ex", s["x"].data_ptr(), self.xdt, self.N, s["F"],
                           s["ldx"], s["shard"].rowptr.data_ptr(), s["graph"].col.data_ptr(),
                           self.n_dst, 0, self.st.data_ptr(), self.xmax.data_ptr(),
                           self.packed.data_ptr(), s["bias"].data_ptr(), H, C, 0.2, 0.0, 0,
                           self.cplan, stages, self.out.data_ptr(), None, self.ws.data_ptr(),
                           self.ws.numel(), st_h)
            return
        self._lib.call("gfd_gat_aggregate_split", s["x"].data_ptr(), self.xdt, self.N, s["F"],
                       s["ldx"], s["shard"].rowptr.data_ptr(), s["graph"].col.data_ptr(),
                       self.n_dst, s["spec"].dst_lo, self.s_all.data_ptr(), H,
                       self.t_loc.data_ptr(), H, self.xmax.data_ptr(), self.packed.data_ptr(),
                       s["bias"].data_ptr(), H, C, 0.2, 0.0, 0, self.cplan, stages, None,
                       self.out.data_ptr(), C, None, self.ws.data_ptr(), self.ws.numel(),
                       self.stream)

    STAGES_FUSED = (("pack+logits+lone", None), ("hubs", STAGE_HUBS), ("general", STAGE_MID),
                    ("light", STAGE_LIGHT))
    STAGES_SHARDED = (("pack+logits+lone", None), ("exchange", "x"), ("hubs", STAGE_HUBS),
                      ("general", STAGE_MID), ("light", STAGE_LIGHT))

    def step(self, evs=None):
        """One layer forward.  ``evs`` (timing): a dict filled with one
        (start, end) event pair per stage name, recorded on the stream the
        stage's launches go to."""
        # events record on torch's current stream == the stream every gfd launch
        # uses (and the one RCCL's collectives are ordered against)
        main = torch.cuda.current_stream(self.dev)

        def run(name, stg, stream=None):
            ev = None
            if evs is not None:
                ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                ev[0].record(stream or main)
            if stg is None:
                self.pack_and_logits()
            elif stg == "x":
                self.exchange()
            else:
                self.aggregate(stg, None if stream is None else stream.cuda_stream)
            if ev is not None:
                ev[1].record(stream or main)
                evs[name] = ev

        if not self.overlap:
            for name, stg in self.stages:
                run(name, stg)
            return
        # --overlap: the light class on a second stream once the logits (and
        # the exchange) are in, beside hubs -> general on the main stream (the
        # three tile launches are independent but for general reading the hub
        # rows' merged z), so light's blocks take the CUs general's tail frees.
        # Each stage's span is timed on its own stream; the step ends when both
        # streams are done.
        for name, stg in self.stages:
            if stg is None or stg == "x":
                run(name, stg)
        self._ready.record(main)
        self.side.wait_event(self._ready)
        with torch.cuda.stream(self.side):
            run("light", STAGE_LIGHT, self.side)
        for name, stg in self.stages:
            if stg in (STAGE_HUBS, STAGE_MID):
                run(name, stg)
        main.wait_stream(self.side)


def time_layer(layer, steps, warmup, world):
    for _ in range(warmup):
        layer.step()
    events = [{} for _ in range(steps)]
    torch.cuda.synchronize()
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        layer.step(events[k])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    med = lambda v: sorted(v)[len(v) // 2]  # noqa: E731
    stage_ms = {name: med([e[name][0].elapsed_time(e[name][1]) for e in events])
                for name, _ in layer.stages}
    mine = elapsed
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=layer.dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    return elapsed, stage_ms, mine


def stage_bytes(s, plan, esz, halo=None):
    """Algorithmic bytes per stage (SURVEY.md §8d terms: a message gathers one
    x row + one int32 column index; a destination writes its fp32 out row and
    reads its rowptr entry; the weights once per kernel)."""
    g, F = s["graph"], s["F"]
    rp = s["shard"].rowptr
    deg = (rp[1:] - rp[:-1]).long()
    light_b, lone_b = plan.classes(s["dtype"])   # (bf16 x: one message more is light)
    order = plan.row_order.long() if plan.row_order is not None else None
    sdeg = deg[order] if order is not None else deg
    hubs_mask = torch.zeros_like(sdeg, dtype=torch.bool)
    if plan.num_hubs > 0:
        hr = plan.hub_rank[:deg.numel()]
        hubs_mask = (hr[order] if order is not None else hr) >= 0
    t = 16
    lb = (light_b + t - 1) // t * t   # the general launch owns the rest of its last tile
    idx = torch.arange(sdeg.numel(), device=sdeg.device)
    gen = idx < lb
    light = (idx >= lb) & (idx < lone_b)
    lone = idx >= lone_b
    row_b = F * esz + 4
    W_b = 4 * F * H * C
    hub_msgs = int(sdeg[hubs_mask].sum().item())
    out_b = 4 + 4 * C
    n_rows = s["spec"].dst_hi - s["spec"].dst_lo   # rows the rank's logits pass streams
    res = {
        "pack+logits": n_rows * (F * esz + 64) + W_b,
        "pack+logits+lone": n_rows * (F * esz + 64 + 4) + W_b + int(lone.sum().item()) * out_b,
        # the exchanged source logits land in HBM once: 32 B per node (all-gather)
        # or per halo row received
        "exchange": (halo.bytes_received(H) if halo is not None else s["graph"].num_nodes * H * 4),
        "hubs": hub_msgs * row_b + plan.num_chunks * 4 * (16 + 8 * ((F + 7) // 8 * 8)),
        "general": int(sdeg[gen & ~hubs_mask].sum().item()) * row_b +
                   int(gen.sum().item()) * out_b + W_b,
        "light": int(sdeg[light].sum().item()) * row_b + int(light.sum().item()) * out_b + W_b,
        "lone": int(lone.sum().item()) * (F * esz + out_b) + W_b // H,
    }
    counts = {"general_dst": int(gen.sum().item()), "light_dst": int(light.sum().item()),
              "lone_dst": int(lone.sum().item()), "hub_messages": hub_msgs}
    return res, counts


def load_pmc(path, key):
    try:
        with open(path) as f:
            return json.load(f).get(key)
    except (OSError, ValueError):
        return None


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(s, args):
    """The oracle's PyG CPU dataflow (Linear -> index_select ->
    scatter_reduce(amax) -> exp -> index_add -> message -> index_add) on a
    bounded sample of the SAME C4 graph: the first destinations of a random
    permutation covering ``--cpu-messages`` messages.  x is copied to host
    memory once (resident, like the device copy in HBM); the timed region
    gathers the rows the sample touches out of the full host x (the
    dataflow's index_select, cache behaviour included), projects them and runs
    the softmax / message / scatter.  1 warm-up, then min and median of
    ``--cpu-runs`` timed runs."""
    from oracle import gatconv_forward_sampled
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)
    torch.set_num_threads(threads)
    g = s["graph"]
    rp = g.rowptr.long()
    deg = rp[1:] - rp[:-1]
    perm = torch.randperm(g.num_nodes, generator=torch.Generator(device=rp.device).manual_seed(7),
                          device=rp.device)
    csum = torch.cumsum(deg[perm], 0)
    k = int(torch.searchsorted(csum, torch.tensor([args.cpu_messages], device=rp.device)).item())
    dsts = perm[:max(k, 1)].sort().values
    msgs = int(deg[dsts].sum().item())
    idx = gatconv_forward_sampled.prepare_indices(g.rowptr, g.col, dsts)
    x_host = s["x"].cpu()
    W, a_s, a_d, b = (s["W"].cpu(), s["a_s"].cpu(), s["a_d"].cpu(), s["bias"].cpu())
    times = []
    with torch.no_grad():
        for _ in range(1 + args.cpu_runs):
            t0 = time.perf_counter()
            gatconv_forward_sampled.run_from(x_host, idx, W, a_s, a_d, b)
            times.append(time.perf_counter() - t0)
    tt = sorted(times[1:])
    med, mn = tt[len(tt) // 2], tt[0]
    in_edges = msgs - dsts.numel()   # input edges of the sample (each dst has one self loop)
    # the whole C4 graph, projected from the sample (the dataflow's work is
    # per message: gather, projection of the gathered rows, message tensor,
    # scatter); BASELINE.md §4's dst-sorted chunked full run would take about
    # this long per run, which does not fit beside the other legs' time limit
    full_s = med * g.num_messages / msgs
    return {"value": in_edges / med, "unit": "edges/s", "cores": threads, "kind": "port",
            "projected_full_graph_s": round(full_s, 1),
            "projected_full_graph_note": f"median x messages ({g.num_messages}) / sampled "
                                         f"messages ({msgs}): linear in messages",
            "min_s": round(mn, 3), "median_s": round(med, 3), "runs": args.cpu_runs,
            "cpu_model": cpu_model(), "value_best": in_edges / mn,
            "sample": f"{dsts.numel()} random destinations of the C4 graph itself "
                      f"({msgs} messages, {in_edges} input edges, {idx['rows']} gathered rows "
                      "out of the full host x); oracle/gatconv_ref.py PyG CPU dataflow restricted "
                      "to the sampled destinations (row gather + projection of the rows they "
                      "read, message tensor, scatter softmax, index_add); fp32, eval; 1 warm-up, "
                      f"min and median of {args.cpu_runs}"}


def measure(args, dev, rank, world, config):
    F = args.features
    if config == "c5":
        N, E, dtype = args.nodes or 50_000_000, args.edges or 500_000_000, torch.bfloat16
    else:
        N, E, dtype = args.nodes or 10_000_000, args.edges or 50_000_000, torch.float32
    t_setup = time.perf_counter()
    row_align = args.row_align or (128 if config == "c5" else 16)
    s = setup(dev, N, E, F, args.gamma, dtype, rank, world, row_align=row_align,
              balance=args.balance, s_in_row=not args.no_s_in_row)
    layer = Layer(s, dev, world, getattr(args, "exchange", "halo"))
    layer.overlap = bool(getattr(args, "overlap", False))
    plan = layer.plan
    esz = s["xbuf"].element_size()
    log(f"[bench] {config} rank {rank}/{world}: N={N} E={E} messages={s['graph'].num_messages} "
        f"shard=[{s['spec'].dst_lo},{s['spec'].dst_hi}) hubs={plan.num_hubs} "
        f"chunks={plan.num_chunks} classes={plan.classes(dtype)} "
        f"setup {time.perf_counter() - t_setup:.1f}s")
    if getattr(args, "legs_only", False) and config == "c4":
        return {"legs_only": True}, s, layer
    elapsed, stage_ms, rank_elapsed = time_layer(layer, args.steps, args.warmup, world)
    ms_step = elapsed * 1e3 / args.steps
    value = E * args.steps / elapsed
    M = s["graph"].num_messages
    B_layer = M * (esz * F + 4) + N * (4 + 4 * C) + 4 * F * H * C
    flop_layer = 2 * N * F * H * C + M * H * (2 * C + 8)
    # per GPU: the layer's bytes and flops split over the ranks (dst sharding)
    t_roof = max(B_layer / (HBM_PEAK_GBPS * 1e9), flop_layer / (BF16_PEAK_TFLOPS * 1e12)) / world
    sb, counts = stage_bytes(s, plan, esz, layer.halo)
    kernels = {}
    for name, ms in stage_ms.items():
        gbps = sb[name] / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
        kernels[name] = {"ms": ms, "algorithmic_bytes": sb[name], "gbps": gbps,
                         "frac": gbps / HBM_PEAK_GBPS}
    dom = max((k for k in kernels if k != "exchange"), key=lambda k: kernels[k]["ms"])
    kname = {"pack+logits": "k_logits_s (+ pack)",
             "pack+logits+lone": "k_logits_lone (+ pack): logits + self-loop-only rows",
             "exchange": ("RCCL all-to-all of the halo rows of the [N, 8] source logits "
                          "(gfd_rows_copy pack / scatter) + max|x| all-reduce" +
                          (" -- two row-range phases, the first issued under the second "
                           "half of the logits pass (its wait and scatter timed here)"
                           if layer.halo_parts is not None else "")
                          if layer.halo is not None else
                          "RCCL all-gather-v of the [N, 8] source logits + max|x| all-reduce"),
             "hubs": "k_hub_partial + k_hub_fin",
             "general": "k_stream<general> (hub rows, 7+ messages)",
             "light": "k_stream<light> (2-6 messages: the 4-6-message tiles, then the "
                      "short tiles of at most 3 -- two launches)",
             "lone": "k_lone (self-loop-only rows)"}
    pmc = load_pmc(args.pmc, f"{config}:{dom}:N={N}:E={E}:F={F}:world={world}")
    workload = (f"{config.upper()} power-law N={N} E={E} F={F} gamma={args.gamma} "
                f"x {str(dtype).replace('torch.', '')}: GATConv layer-0 forward "
                f"(H=8, C=64, concat=False, self loops)")
    res = {
        "metric": METRIC, "value": value, "unit": "edges/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms_step,
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
        "dtype": "bf16" if dtype == torch.bfloat16 else "f32",
        "data": "synthetic (Chung-Lu power-law graph on device, seed 1; x ~ N(0,1) seed 0; "
                "glorot weights seed 0)",
        "config": {"workload": workload, "nodes": N, "input_edges": E, "messages": M,
                   "features": F, "heads": H, "channels": C, "row_pitch": s["ldx"],
                   "parallelism": (f"dst-shard x{world} ({args.balance}-balanced)" if world > 1
                                   else "single GPU"),
                   "hubs": plan.num_hubs, "hub_chunks": plan.num_chunks, **counts},
        "roofline": {"bound": "hbm", "achieved": kernels[dom]["gbps"], "peak": HBM_PEAK_GBPS,
                     "unit": "GB/s", "frac": kernels[dom]["frac"],
                     "traffic": pmc.get("hbm_bytes_per_launch") if pmc else None,
                     # provenance of traffic: the git tree its PMC passes ran on
                     "traffic_source": ({"tree": pmc.get("tree"), "source": pmc.get("source")}
                                        if pmc else None),
                     "kernel": kname[dom], "algorithmic_bytes": sb[dom],
                     "kernel_ms": kernels[dom]["ms"]},
        "kernels": kernels,
        "layer": {"algorithmic_bytes": B_layer, "flop": flop_layer,
                  "hbm_gbps": B_layer / (ms_step * 1e-3) / 1e9,
                  "hbm_gbps_per_gpu": B_layer / world / (ms_step * 1e-3) / 1e9,
                  "t_roof_ms": t_roof * 1e3, "roofline_frac": t_roof / (ms_step * 1e-3)},
        "cpu_baseline": None,
    }
    if world > 1:
        # every rank's own clock and stages (rank 0 prints them): the line's
        # ms_per_step is the max over ranks
        import torch.distributed as dist
        mine = {"rank": rank, "elapsed_s": rank_elapsed, "stage_ms": stage_ms,
                "exchange": args.exchange,
                "halo_rows": (int(layer.halo.recv_rows.numel()) if layer.halo is not None
                              else None),
                "dst": [s["spec"].dst_lo, s["spec"].dst_hi],
                "messages": int(s["shard"].rowptr[-1].item() - s["shard"].rowptr[0].item()),
                "device": torch.cuda.get_device_name(dev)}
        allr = [None] * world
        dist.all_gather_object(allr, mine)
        res["distributed"] = {"backend": dist.get_backend(), "world_size": dist.get_world_size(),
                              "ranks": allr}
    return res, s, layer


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def rank_command(args, argv, port: int):
    """The command that runs ``--gpus N`` as N ranks: torch.distributed.run
    with one process per GPU on this node, rendezvous on 127.0.0.1."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
            f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1",
            f"--master-port={port}", os.path.abspath(__file__), *argv]


def launch_ranks(args, argv, device_count=None, run=None) -> int:
    """``python bench.py --gpus N`` (N > 1) outside a launcher: start the N
    ranks as a CHILD torch.distributed.run and return its exit status.  This
    process never touches the GPU (device_count() only counts devices on this
    image; no HIP context is created) and never re-execs itself.  Fewer than N
    visible devices is an error (exit 2), not a silently smaller run."""
    import subprocess
    n = args.gpus
    have = torch.cuda.device_count() if device_count is None else device_count
    if have < n and not args.rehearse:
        log(f"[bench] --gpus {n}: only {have} device(s) visible; refusing to time fewer ranks")
        return 2
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # dmabuf IPC (RCCL peer buffers)
    cmd = rank_command(args, argv, free_port())
    log(f"[bench] launching {n} ranks: {' '.join(cmd)}")
    return (run or subprocess.call)(cmd, env=env)


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and (args.gpus or 1) > 1:
        sys.exit(launch_ranks(args, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus is None:
        args.gpus = world
    if world != args.gpus:
        log(f"[bench] WORLD_SIZE={world} but --gpus {args.gpus}: refusing a mismatched run")
        sys.exit(2)
    gpu = local % max(torch.cuda.device_count(), 1) if args.rehearse else local
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(gpu)
        if args.rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
    dev = torch.device("cuda", gpu if world > 1 else 0)
    torch.cuda.set_device(dev)
    res, s, layer = measure(args, dev, rank, world, args.config)
    if args.rehearse:
        res["rehearsal"] = ("ranks share the visible GPU(s) with a gloo host-staged exchange: "
                            "a functional run of the N-rank path, not a scaling measurement")
    if world == 1 and rank == 0 and args.config == "c4":
        import bench_legs
        want = [w for w in args.legs.split(",") if w] if not args.no_legs else []
        legs = {}
        if not args.no_cpu_baseline and not args.legs_only:
            log("[bench] timing CPU baseline (oracle, bounded sample of the C4 graph) ...")
            res["cpu_baseline"] = cpu_baseline(s, args)
        if "c4bwd" in want:
            log("[bench] leg C4 forward + backward ...")
            leg = bench_legs.c4_layer_fwd_bwd(s, dev)
            pmc_b = load_pmc(args.pmc, f"c4:backward:N={s['graph'].num_nodes}:world=1")
            if pmc_b:  # the backward kernels' HBM bytes (scripts/pmc_bwd_summary.py)
                leg["roofline"]["traffic"] = pmc_b.get("hbm_bytes_per_pass")
                leg["roofline"]["traffic_source"] = {"tree": pmc_b.get("tree"),
                                                     "source": pmc_b.get("source")}
            legs["c4_layer_fwd_bwd"] = leg
            log("[bench] leg C4 forward + backward, attention dropout 0.2 ...")
            legs["c4_layer_fwd_bwd_dropout"] = bench_legs.c4_layer_fwd_bwd(s, dev, dropout=0.2)
        if "dropin" in want:
            log("[bench] leg drop-in module (gfd.nn.GATConv on the COO edge_index) ...")
            legs["c4_dropin_module"] = bench_legs.dropin_module(s, dev, res.get("ms_per_step"))
        if "sample" in want:
            log("[bench] leg neighbour sampling on the C4 graph ...")
            legs["neighbor_sampling"] = bench_legs.neighbor_sampling(s, dev)
        del s, layer
        torch.cuda.empty_cache()
        if "c5" in want:
            log("[bench] leg C5: bf16 features, 50M nodes / 500M edges ...")
            c5, s5, l5 = measure(args, dev, 0, 1, "c5")
            del s5, l5
            torch.cuda.empty_cache()
            legs["c5_bf16_forward"] = {k: c5[k] for k in ("metric", "value", "unit", "ms_per_step",
                                                          "dtype", "config", "roofline",
                                                          "kernels", "layer")}
        for name, fn in (("c1", "c1_gat2_forward"), ("c2", "c2_gat3_train_step"),
                         ("c3", "c3_tgn_49_steps"), ("temporal", "temporal_snapshots"),
                         ("ingest", "ingest_id_map")):
            if name in want:
                log(f"[bench] leg {fn} ...")
                legs[fn] = getattr(bench_legs, fn)(dev)
                torch.cuda.empty_cache()
        if legs:
            res["legs"] = legs
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
