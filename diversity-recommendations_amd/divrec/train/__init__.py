from .utils import (
    fused_adam_step,
    get_model_recommendations,
    pair_wise_score_loop,
    pair_wise_train_loop,
    point_wise_score_loop,
    point_wise_train_loop,
    recommendations_score_loop,
    recommendations_train_loop,
)

__all__ = [
    "point_wise_score_loop",
    "pair_wise_score_loop",
    "get_model_recommendations",
    "recommendations_score_loop",
    "point_wise_train_loop",
    "pair_wise_train_loop",
    "recommendations_train_loop",
    "fused_adam_step",
]
