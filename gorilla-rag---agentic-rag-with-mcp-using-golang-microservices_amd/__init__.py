"""MI355X-native exact top-k vector search for GoRilla-RAG's vector-service.

The product is the HIP library ``lib/libvsearch.so`` behind the C-ABI in
``include/vsearch.h``; :mod:`.engine` is its ctypes binding and
:mod:`.service` the host-side mirror of rag/vector-service's HTTP handlers.
"""
from .engine import (DTYPE_BF16, DTYPE_F32, FLAG_NO_PREFILTER, METRIC_COSINE, METRIC_DOT,
                     VectorEngine, VSError, build_id, device_count, keys_decode, load_library,
                     pack_allow)

__all__ = ["VectorEngine", "VSError", "build_id", "device_count", "keys_decode", "load_library", "pack_allow",
           "METRIC_COSINE", "METRIC_DOT", "DTYPE_F32", "DTYPE_BF16", "FLAG_NO_PREFILTER"]
