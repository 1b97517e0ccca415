"""CPU restatement of gfd's neighbour sampler -- TEST INFRASTRUCTURE ONLY.

The sampler replaces PyG NeighborLoader (/root/reference/src/data/dataloader.py
:42-66): per hop, for every frontier node, min(k, in-degree) distinct
in-neighbours drawn uniformly without replacement; new sources appended in
order of first appearance (frontier order, then draw order).  PyG's own random
stream cannot be reproduced (PyG is not installed and uses another generator),
so this restatement fixes the draws: Robert Floyd's algorithm over
counter-based splitmix64 numbers keyed by (seed, hop, node, draw) -- the same
function the HIP kernel evaluates (gfd_sample.hip), so GPU and oracle agree
bit for bit; the distribution is what is pinned to PyG (uniform k-subsets).
"""
from __future__ import annotations

M64 = (1 << 64) - 1


def mix64(z: int) -> int:
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def draw(seed: int, hop: int, node: int, i: int, m: int) -> int:
    """Uniform integer in [0, m] for (seed, hop, node, draw i)."""
    z = mix64((seed & M64) ^ (((hop + 1) * 0x9E3779B97F4A7C15) & M64) ^
              ((node * 0xD1B54A32D192ED03) & M64) ^ (((i + 1) * 0x8CB92BA72F3D8DD7) & M64))
    return z % (m + 1)


def floyd(d: int, k: int, seed: int, hop: int, node: int):
    """k distinct positions of [0, d) (d > k), uniformly, in insertion order."""
    pick = []
    for i in range(k):
        j = d - k + i
        t = draw(seed, hop, node, i, j)
        pick.append(j if t in pick else t)
    return pick


def sample_ref(rowptr, col, seeds, fanouts, seed):
    """(n_id, level_ptr, edges [(src_local, dst_local, csr_pos)], edge_ptr) on
    the gfd CSR (rowptr / col with one self loop appended last per segment,
    which is not sampled)."""
    n_id = [int(s) for s in seeds]
    local = {s: i for i, s in enumerate(n_id)}
    level, edges, edge_ptr = [0, len(n_id)], [], [0]
    for hop, k in enumerate(fanouts):
        cands = []
        for f in range(level[hop], level[hop + 1]):
            node = n_id[f]
            e0 = int(rowptr[node])
            d = int(rowptr[node + 1]) - e0 - 1
            picks = range(d) if d <= k else floyd(d, k, seed, hop, node)
            cands += [(int(col[e0 + t]), f, e0 + t) for t in picks]
        for j, _, _ in cands:
            if j not in local:
                local[j] = len(n_id)
                n_id.append(j)
        level.append(len(n_id))
        edges += [(local[j], dl, eid) for j, dl, eid in cands]
        edge_ptr.append(len(edges))
    return n_id, level, edges, edge_ptr
