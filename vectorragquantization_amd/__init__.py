"""vectorragquantization_amd -- MI355X-native (gfx950) rebuild of the
aitrailblazer/VectorRAGQuantization hot path: CohereEnhancedVectorDB's
three-phase search (Phase I Hamming top-k, Phase II float x +-1 rescoring,
Phase III float x int8 cosine rescoring) and the VectorDBInt{4,8,16}{,Global}
quantise/packbits encode path, as hand-written HIP kernels behind a C ABI
(libvrq.so, include/vrq.h) with the reference's Python surface on top.
"""
from ._native import VrqNativeError, load as load_native  # noqa: F401

__all__ = ["VrqNativeError", "load_native", "CohereEnhancedVectorDB", "BinaryIndexIDMap2", "encode",
           "ShardedSearch", "CohereVectorDBFloat", "VectorDBInt8Global", "VectorDBInt16Global", "VectorDBInt4Global",
           "VectorDBInt8", "VectorDBInt4", "VectorDBInt16", "CohereVectorDBInt8"]

_VECTORDB = ("VectorDBInt8Global", "VectorDBInt16Global", "VectorDBInt4Global", "VectorDBInt8", "VectorDBInt4",
             "VectorDBInt16", "CohereVectorDBInt8")


def __getattr__(name):  # lazy: importing the package must not require a GPU
    if name == "CohereEnhancedVectorDB":
        from .enhanced import CohereEnhancedVectorDB
        return CohereEnhancedVectorDB
    if name == "BinaryIndexIDMap2":
        from .index import BinaryIndexIDMap2
        return BinaryIndexIDMap2
    if name == "encode":
        from .quant import encode
        return encode
    if name in _VECTORDB:
        from . import vectordb
        return getattr(vectordb, name)
    if name == "CohereVectorDBFloat":
        from .flat import CohereVectorDBFloat
        return CohereVectorDBFloat
    if name == "ShardedSearch":
        from .dist import ShardedSearch
        return ShardedSearch
    raise AttributeError(name)
