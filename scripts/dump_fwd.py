"""Dump one GATConv forward (out, st, stats) of the C2 fixture's layer 0 for
the library named by GFD_LIB_PATH, into gpurun_out/<tag>.npz (A/B of kernel
variants: compare two dumps with numpy on the host)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "gnn-fraud-detection_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from conftest import load_golden  # noqa: E402
from gfd import _lib  # noqa: E402
from gfd.graph import _ws, get_graph  # noqa: E402

tag = sys.argv[1]
arr = load_golden("gat3_train_grads.npz")
dev = "cuda"
x = torch.from_numpy(arr["x"]).to(dev)
ei = torch.from_numpy(arr["edge_index"]).to(dev)
W = torch.from_numpy(arr["w.gat_layers.0.lin_src.weight"]).to(dev)
a_s = torch.from_numpy(arr["w.gat_layers.0.att_src"]).to(dev).reshape(-1)
a_d = torch.from_numpy(arr["w.gat_layers.0.att_dst"]).to(dev).reshape(-1)
b = torch.from_numpy(arr["w.gat_layers.0.bias"]).to(dev)
N, F = x.shape
g = get_graph(ei, N)
plan = g.plan()
lib = _lib.load()
res = {}
for pitch in (F, (F + 3) // 4 * 4):
    xb = torch.zeros((N, pitch), device=dev)
    xb[:, :F] = x
    xv = xb[:, :F]
    out = torch.empty((N, 64), device=dev)
    st = torch.empty((N, 16), device=dev)
    stats = torch.empty((N, 16), device=dev)
    ws = _ws(lib.gfd_gat_fwd_workspace_size(N, N, F, 8, 64, plan.num_hubs, plan.num_chunks), dev)
    _lib.call("gfd_gat_fwd", xv.data_ptr(), 0, N, F, pitch, g.rowptr.data_ptr(), g.col.data_ptr(),
              W.data_ptr(), a_s.data_ptr(), a_d.data_ptr(), b.data_ptr(), 8, 64, 0.2, 0.0, 0,
              plan.cstruct(), out.data_ptr(), st.data_ptr(), stats.data_ptr(), ws.data_ptr(),
              ws.numel(), _lib.stream_handle(dev))
    torch.cuda.synchronize()
    res[f"out_{pitch}"] = out.cpu().numpy()
    res[f"st_{pitch}"] = st.cpu().numpy()
    res[f"stats_{pitch}"] = stats.cpu().numpy()
res["rowptr"] = g.rowptr.cpu().numpy()
res["order"] = plan.row_order.cpu().numpy()
res["split"] = plan.class_split.cpu().numpy()
os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(REPO, "gpurun_out", f"{tag}.npz"), **res)
print("saved", tag, {k: v.shape for k, v in res.items()})
