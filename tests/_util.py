"""Shared test helpers (weights from fixtures, oracle CSR, tolerances)."""
import numpy as np
import torch

# Parity bar from BASELINE.json north_star: outputs within 1e-4 (fp32) of the
# PyG-dataflow CPU forward on identical weights.
FWD_ATOL = 1e-4
FWD_RTOL = 1e-4
# Gradients: fp32 sums in a different order (and BatchNorm's batch statistics in
# train mode) -- still 1e-4 relative to the tensor's scale.
GRAD_RTOL = 1e-4


def state_dict_from(arrays: dict, prefix: str) -> dict:
    sd = {}
    for k, v in arrays.items():
        if not k.startswith(prefix):
            continue
        name = k[len(prefix):]
        sd[name] = torch.from_numpy(np.array(v))
        if name.endswith("lin_src.weight"):
            sd[name.replace("lin_src", "lin_dst")] = sd[name]
    return sd


def assert_close(got, ref, atol=FWD_ATOL, rtol=FWD_RTOL, what=""):
    got = got.detach().cpu().double().numpy() if torch.is_tensor(got) else np.asarray(got, np.float64)
    ref = ref.detach().cpu().double().numpy() if torch.is_tensor(ref) else np.asarray(ref, np.float64)
    assert got.shape == ref.shape, f"{what}: shape {got.shape} != {ref.shape}"
    err = np.abs(got - ref)
    bound = atol + rtol * np.abs(ref)
    bad = err > bound
    assert not bad.any(), (f"{what}: {bad.sum()} / {bad.size} elements off; max abs err "
                           f"{err.max():.3e} (ref scale {np.abs(ref).max():.3e})")


def assert_close_scaled(got, ref, rtol=GRAD_RTOL, what="", atol=0.0):
    """|got - ref| <= rtol * max|ref| + atol (for gradients whose entries span
    decades).  ``atol`` covers gradients that are zero up to fp32 noise, e.g.
    the GATConv bias feeding a train-mode BatchNorm (BN removes the shift)."""
    got = got.detach().cpu().double().numpy() if torch.is_tensor(got) else np.asarray(got, np.float64)
    ref = ref.detach().cpu().double().numpy() if torch.is_tensor(ref) else np.asarray(ref, np.float64)
    assert got.shape == ref.shape, f"{what}: shape {got.shape} != {ref.shape}"
    scale = max(np.abs(ref).max(), 1e-30)
    err = np.abs(got - ref).max()
    assert err <= rtol * scale + atol, f"{what}: max abs err {err:.3e} > {rtol} * {scale:.3e} + {atol}"


def csr_cpu(edge_index: torch.Tensor, num_nodes: int):
    """CPU CSR with PyG's self-loop policy (stable by destination, loops last)."""
    ei = edge_index.long()
    keep = ei[0] != ei[1]
    src, dst = ei[0][keep], ei[1][keep]
    loops = torch.arange(num_nodes)
    src = torch.cat([src, loops])
    dst = torch.cat([dst, loops])
    order = torch.argsort(dst, stable=True)
    rowptr = torch.zeros(num_nodes + 1, dtype=torch.long)
    rowptr[1:] = torch.cumsum(torch.bincount(dst, minlength=num_nodes), 0)
    return rowptr, src[order]
