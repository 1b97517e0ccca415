"""Oracle package: CPU restatements of the reference's GATConv hot path and
model wiring.  TEST INFRASTRUCTURE ONLY -- imported by ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg, never by
the product package ``gfd``.  See oracle/gatconv_ref.py for the parity status.
"""
from .gatconv_ref import (GATConvRef, gatconv_forward, gatconv_forward_chunked,  # noqa: F401
                          gatconv_forward_at, gatconv_forward_sampled, gatconv_grads_chunked,
                          remove_then_add_self_loops, segment_softmax, glorot_)
from .models_ref import GATRef, TemporalGNNRef  # noqa: F401
from .ingest_ref import process_ref  # noqa: F401
from .sample_ref import floyd, sample_ref  # noqa: F401
from .temporal_ref import temporal_subgraph_loop, temporal_subgraph_ref  # noqa: F401
