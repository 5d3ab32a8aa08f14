from .base_models import RankingModel
from .matrix_factorization import MatrixFactorization
from .random_model import RandomModel

__all__ = ["MatrixFactorization", "RankingModel", "RandomModel"]
