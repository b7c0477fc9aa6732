"""CEO-Firm matching two-tower model -- MI355X-native training path.

Drop-in replacement for the hot path of SMaric93/CEO-Recommender's
``ceo_firm_matching`` package (model, training loop, data feeding); see
DESIGN.md / INTEGRATION.md at the repository root.
"""
from .config import Config
from .data import CEOFirmDataset, DataProcessor
from .engine import FusedTrainer
from .model import CEOFirmMatcher
from .explain import ModelWrapper, explain_model_pdp, explain_model_shap
from .synthetic import generate_pairs, generate_structural_synthetic_data, generate_synthetic_data
from .training import train, train_model
from .visualization import plot_interaction_heatmap
from . import contrastive  # noqa: E402  (reference: Extension 2, contrastive learning)

__version__ = "0.4.0+mi355x"

# the reference's two-tower names (reference __init__.py:7-13,44-55); its
# structural-distillation and research-extension modules are out of scope
# (INTEGRATION.md lists them)
__all__ = ["Config", "DataProcessor", "CEOFirmDataset", "CEOFirmMatcher", "train_model", "train",
           "ModelWrapper", "explain_model_pdp", "explain_model_shap", "plot_interaction_heatmap",
           "generate_synthetic_data", "generate_structural_synthetic_data",
           "FusedTrainer", "generate_pairs", "contrastive"]
