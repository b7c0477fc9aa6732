"""CEO-Firm matching two-tower model -- MI355X-native training path.

Drop-in replacement for the hot path of SMaric93/CEO-Recommender's
``ceo_firm_matching`` package (model, training loop, data feeding); see
DESIGN.md / INTEGRATION.md at the repository root.
"""
from .config import Config
from .data import CEOFirmDataset, DataProcessor
from .engine import FusedTrainer
from .model import CEOFirmMatcher
from .synthetic import generate_pairs, generate_synthetic_data
from .training import train, train_model
from . import contrastive  # noqa: E402  (reference: Extension 2, contrastive learning)

__version__ = "0.4.0+mi355x"

__all__ = ["Config", "DataProcessor", "CEOFirmDataset", "CEOFirmMatcher", "train_model", "train",
           "FusedTrainer", "generate_synthetic_data", "generate_pairs"]
