"""Graph ingest to the device.

* ``ingest_elliptic(data_dir, device)`` -- EllipticBitcoinDataset.process
  (/root/reference/src/data/dataset.py:75-129): the three CSVs are parsed on
  the host (pandas' C parser, as the reference reads them, including its
  header=0 behaviour that turns the first transaction into the header,
  SURVEY.md Appendix B item 1), then the id -> index dict (:92), the edge
  filter and remap (:95-101) and the label assignment (:106-113) run on the
  GPU (gfd_id_map_build / gfd_edges_from_ids / gfd_id_map_lookup) instead of
  DataFrame.iterrows() loops.
* ``save_graph`` / ``load_graph`` -- a binary graph directory (raw .npy per
  tensor: x, edge_index, y, time_steps) that ``load_graph`` memory-maps and
  streams to the GPU in pinned chunks, replacing the reference's
  torch.save/torch.load of the processed dataset and its per-epoch
  ``batch.to(device)`` (train.py:105).
* ``partition_bounds`` -- edge-balanced destination ranges for the sharded
  layer (gfd.dist), from the device CSR.
"""
from __future__ import annotations

import os
from typing import Dict, Optional

import numpy as np
import torch

from . import _lib
from .graph import _ws

CLASS_MAPPING = {"unknown": -1, "1": 1, "2": 0}    # config.py:24-28
FILES = ("elliptic_txs_features.csv", "elliptic_txs_edgelist.csv", "elliptic_txs_classes.csv")


def read_elliptic_csv(data_dir: str) -> Dict[str, np.ndarray]:
    """The three CSVs as the reference reads them (dataset.py:81-89)."""
    import pandas as pd
    feats = pd.read_csv(os.path.join(data_dir, FILES[0]))           # header=0 (Appendix B1)
    edges = pd.read_csv(os.path.join(data_dir, FILES[1]))
    classes = pd.read_csv(os.path.join(data_dir, FILES[2]), dtype={"class": str})
    return {"ids": feats.iloc[:, 0].to_numpy(np.int64),
            "time_steps": feats.iloc[:, 1].to_numpy(np.int64),
            "x": np.ascontiguousarray(feats.iloc[:, 2:].to_numpy(np.float32)),
            "src_ids": edges["txId1"].to_numpy(np.int64),
            "dst_ids": edges["txId2"].to_numpy(np.int64),
            "class_ids": classes["txId"].to_numpy(np.int64),
            "class_labels": np.array([CLASS_MAPPING.get(str(c), -1) for c in classes["class"]],
                                     np.int64)}


def _upload(a: np.ndarray, device, chunk_bytes: int = 64 << 20) -> torch.Tensor:
    """Host array (possibly memory-mapped) -> device tensor through pinned
    staging chunks (non-blocking copies overlap the next chunk's staging)."""
    out = torch.empty(a.shape, dtype=torch.from_numpy(a[:0].copy()).dtype, device=device)
    if a.size == 0:
        return out
    flat_src = a.reshape(-1)
    flat_dst = out.view(-1)
    per = max(1, chunk_bytes // a.itemsize)
    bufs = [torch.empty(per, dtype=out.dtype).pin_memory() for _ in range(2)]
    events = [None, None]
    # the copies run on the destination device's current stream; every event
    # is recorded there too (not on the current device's), so a pinned buffer
    # is refilled only after the DMA out of it has finished
    with torch.cuda.device(out.device):
        stream = torch.cuda.current_stream(out.device)
        for k, s in enumerate(range(0, flat_src.size, per)):
            n = min(per, flat_src.size - s)
            b = k & 1
            if events[b] is not None:
                events[b].synchronize()          # the copy out of this buffer is done
            bufs[b][:n].numpy()[...] = flat_src[s:s + n]
            flat_dst[s:s + n].copy_(bufs[b][:n], non_blocking=True)
            events[b] = torch.cuda.Event()
            events[b].record(stream)
        stream.synchronize()
    return out


def ingest_elliptic(data_dir: str, device="cuda") -> Dict[str, torch.Tensor]:
    """dataset.py:75-129 with the index work on the GPU: x [N, F] fp32,
    edge_index [2, E'] int64, y [N] int64 (-1 unknown, 1 illicit, 0 licit),
    time_steps [N] int64."""
    h = read_elliptic_csv(data_dir)
    return ingest_arrays(h, device)


def ingest_arrays(h: Dict[str, np.ndarray], device="cuda") -> Dict[str, torch.Tensor]:
    lib = _lib.load()
    dev = torch.device(device)
    stream = _lib.stream_handle(dev)
    ids = _upload(h["ids"], dev)
    N = ids.numel()
    sorted_ids = torch.empty(N, dtype=torch.int64, device=dev)
    sorted_idx = torch.empty(N, dtype=torch.int32, device=dev)
    ws = _ws(lib.gfd_id_map_workspace_size(N), dev)
    _lib.call("gfd_id_map_build", ids.data_ptr(), N, sorted_ids.data_ptr(), sorted_idx.data_ptr(),
              ws.data_ptr(), ws.numel(), stream)
    src, dst = _upload(h["src_ids"], dev), _upload(h["dst_ids"], dev)
    E = src.numel()
    ei = torch.empty((2, max(E, 1)), dtype=torch.int64, device=dev)
    kept = torch.zeros(1, dtype=torch.int64, device=dev)
    ws = _ws(lib.gfd_edges_from_ids_workspace_size(E), dev)
    _lib.call("gfd_edges_from_ids", sorted_ids.data_ptr(), sorted_idx.data_ptr(), N,
              src.data_ptr(), dst.data_ptr(), E, ei.data_ptr(), kept.data_ptr(), ws.data_ptr(),
              ws.numel(), stream)
    k = int(kept.item())
    if k == 0:
        raise ValueError("No valid edges found after mapping node IDs to indices.")  # dataset.py:103
    edge_index = ei.view(-1)[:2 * E].view(2, E)[:, :k].contiguous()
    # labels: class rows in file order, the last row of a node wins (dataset.py:108-113)
    cid = _upload(h["class_ids"], dev)
    lab = _upload(h["class_labels"], dev)
    pos = torch.empty(cid.numel(), dtype=torch.int32, device=dev)
    _lib.call("gfd_id_map_lookup", sorted_ids.data_ptr(), sorted_idx.data_ptr(), N,
              cid.data_ptr(), cid.numel(), pos.data_ptr(), stream)
    ok = (pos >= 0) & (lab >= 0)
    rows = torch.arange(cid.numel(), device=dev)
    last = torch.full((N,), -1, dtype=torch.int64, device=dev)
    last.scatter_reduce_(0, pos[ok].long(), rows[ok], reduce="amax")
    y = torch.full((N,), -1, dtype=torch.int64, device=dev)
    has = last >= 0
    y[has] = lab[last[has]]
    return {"x": _upload(h["x"], dev), "edge_index": edge_index, "y": y,
            "time_steps": _upload(h["time_steps"], dev)}


def save_graph(path: str, **tensors: torch.Tensor) -> None:
    """One raw .npy per tensor under ``path`` (memory-mappable)."""
    os.makedirs(path, exist_ok=True)
    for name, t in tensors.items():
        np.save(os.path.join(path, name + ".npy"), t.detach().cpu().numpy())


def load_graph(path: str, device="cuda") -> Dict[str, torch.Tensor]:
    """Memory-map every .npy under ``path`` (no pickles: allow_pickle=False)
    and stream it to ``device`` through pinned chunks."""
    out = {}
    for f in sorted(os.listdir(path)):
        if f.endswith(".npy"):
            a = np.load(os.path.join(path, f), mmap_mode="r", allow_pickle=False)
            out[f[:-4]] = (_upload(a, device) if torch.device(device).type == "cuda"
                           else torch.from_numpy(np.array(a)))
    return out


def partition_bounds(graph, parts: int):
    """Edge-balanced destination ranges (gfd.dist.edge_balanced_bounds) of a CSRGraph."""
    from .dist import edge_balanced_bounds
    return edge_balanced_bounds(graph.rowptr, parts)
