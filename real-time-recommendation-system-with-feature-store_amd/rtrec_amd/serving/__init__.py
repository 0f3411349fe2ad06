"""Serving: HBM-resident exact retrieval (reference src/serving/retrieval.py)."""
from .retrieval import FaissIndex, HipFlatIPIndex, IndexBase, RetrievalEngine, register_index

__all__ = ["IndexBase", "HipFlatIPIndex", "FaissIndex", "RetrievalEngine", "register_index"]
