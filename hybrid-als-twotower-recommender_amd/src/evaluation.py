"""Evaluation helpers the hot path calls.

Only `compute_f1_score` is provided: src/hybrid_system.py:15 imports it from
this module, where the reference never defines it; the
definition is the reference's own copy from src/als_model.py:171-177. The
offline quality metrics of src/evaluation.py (P@k, NDCG, plots) are outside
the hot path and not rebuilt.
"""
from .als_model import compute_f1_score  # noqa: F401
