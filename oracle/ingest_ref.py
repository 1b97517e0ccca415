"""CPU restatement of EllipticBitcoinDataset.process -- TEST INFRASTRUCTURE ONLY
(the checker for gfd.ingest).  Follows /root/reference/src/data/dataset.py:
  :81-83  pd.read_csv of the three files (header=0: the features file has no
          header, so its first transaction becomes the header row);
  :86-88  ids = column 0 (as str), time steps = column 1, features = 2:;
  :92     node_id_to_idx = {id: position} (a repeated id keeps its last position);
  :95-101 edges kept when both ids are known, original order, remapped;
  :106-113 y = -1, then per class row in order: '1' -> 1, '2' -> 0.
Small inputs only (the per-row loops are the reference's)."""
from __future__ import annotations

import os

import numpy as np


def process_ref(data_dir: str):
    import pandas as pd
    feats = pd.read_csv(os.path.join(data_dir, "elliptic_txs_features.csv"))
    edges = pd.read_csv(os.path.join(data_dir, "elliptic_txs_edgelist.csv"))
    classes = pd.read_csv(os.path.join(data_dir, "elliptic_txs_classes.csv"))
    node_ids = feats.iloc[:, 0].astype(str).values
    time_steps = feats.iloc[:, 1].values
    x = feats.iloc[:, 2:].values.astype(np.float32)
    idx = {nid: i for i, nid in enumerate(node_ids)}
    ei = []
    for _, row in edges.iterrows():
        s, d = str(int(row["txId1"])), str(int(row["txId2"]))
        if s in idx and d in idx:
            ei.append([idx[s], idx[d]])
    y = np.full(len(node_ids), -1, np.int64)
    for _, row in classes.iterrows():
        nid, label = str(int(row["txId"])), row["class"]
        if nid in idx and str(label) in ("1", "2"):
            y[idx[nid]] = 1 if str(label) == "1" else 0
    return {"x": x, "edge_index": np.array(ei, np.int64).T, "y": y,
            "time_steps": np.asarray(time_steps, np.int64)}
