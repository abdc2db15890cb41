"""Drop-in MI355X implementation of the reference package `src`
(HSoumi/hybrid-als-twotower-recommender, src/__init__.py:36-123).

Same module paths and class names as the reference — `src.als_model.ALSModel`,
`src.two_tower_model.TwoTowerModel`, `src.hybrid_system.HybridRecommendationSystem` —
with the ALS solves, two-tower towers and scoring/fusion running as hand-written
HIP kernels (libhrec.so, C-ABI in include/hrec.h). Put the directory that
contains this package on sys.path to use it in place of the reference.
"""
__version__ = "1.0.0"

# The reference's re-exports (src/__init__.py:39-42, __all__ :53-63) minus the
# out-of-scope src.utils helpers.
from .hybrid_system import HybridRecommendationSystem  # noqa: E402
from .als_model import ALSModel  # noqa: E402
from .two_tower_model import TwoTowerModel  # noqa: E402
from .evaluation import RecommenderEvaluator  # noqa: E402

__all__ = ["HybridRecommendationSystem", "ALSModel", "TwoTowerModel", "RecommenderEvaluator"]

DEFAULT_CONFIG = {
    "ALS_PARAMS": {"rank": 10, "max_iter": 10, "reg_param": 0.1, "cold_start_strategy": "drop"},
    "TWO_TOWER_PARAMS": {"embedding_size": 50, "learning_rate": 0.001},
    "EVALUATION_PARAMS": {"k_values": [5, 10, 15, 20], "top_k": 5},
}


def get_default_config():
    return DEFAULT_CONFIG.copy()
