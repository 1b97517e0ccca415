"""gfd -- MI355X-native GAT/TGN message passing.

Drop-in for the reference's hot path (PyG ``GATConv`` as used by
/root/reference/src/models/gat.py and tgn.py).  Public surface:

* ``gfd.nn.GATConv`` / ``gfd.nn.gat_conv``  -- the operator (libgfd.so)
* ``gfd.models.GAT`` / ``gfd.models.TemporalGNN`` -- the reference model families
* ``gfd.graph``  -- COO -> cached CSR/CSC/hub plan on the GPU
* ``gfd.dist``   -- destination-sharded multi-GPU execution (RCCL)
* ``gfd.pyg_shim.install()`` -- run the reference's own model files on gfd
"""
__version__ = "0.1.0"

_LAZY = {"GATConv": "nn", "gat_conv": "nn", "GAT": "models", "TemporalGNN": "models"}


def __getattr__(name):
    if name in _LAZY:
        import importlib
        return getattr(importlib.import_module(f".{_LAZY[name]}", __name__), name)
    raise AttributeError(name)
