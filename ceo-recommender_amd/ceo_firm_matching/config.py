"""Configuration (mirrors the reference ``ceo_firm_matching/config.py:10-55``).

Same class-attribute surface.  Differences:
* ``DEVICE`` prefers the HIP device (``torch.cuda`` on ROCm) and prints as
  ``cuda`` (reference test ``test_config.py:13``); MPS does not exist on ROCm.
* ``OUTPUT_PATH`` defaults to ``$CEO_TT_OUTPUT`` or ``./Output`` instead of the
  author's home directory (``config.py:17``).
* ``DROPOUT_P`` (0.1, the value hard-coded at ``model.py:41,45,56,60``) is
  exposed so parity runs can disable dropout.
"""
import os
from typing import List

import torch


class Config:
    """Centralized configuration for the project."""
    # System
    DEVICE = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    DATA_PATH = "Data/ceo_types_v0.2.csv"
    OUTPUT_PATH = os.environ.get("CEO_TT_OUTPUT", os.path.join(os.getcwd(), "Output"))

    # Hyperparameters
    EPOCHS = 40
    LEARNING_RATE = 0.0004
    LATENT_DIM = 60
    BATCH_SIZE = 128
    DROPOUT_P = 0.1

    # Embedding Dimensions
    EMBEDDING_DIM_SMALL = 2
    EMBEDDING_DIM_MEDIUM = 8
    EMBEDDING_DIM_LARGE = 48

    # Feature Definitions
    ID_COLS = ['gvkey', 'match_exec_id']

    # CEO Features
    CEO_NUMERIC_COLS = ['Age']  # 'tenure' is derived
    CEO_CAT_COLS = ['Gender', 'maxedu', 'ivy', 'm', 'Output', 'Throghput', 'Peripheral']
    CEO_RAW_COLS = CEO_NUMERIC_COLS + CEO_CAT_COLS + ['ceo_year', 'dep_baby_ceo']

    # Firm Features
    FIRM_NUMERIC_COLS = ['ind_firms_60w', 'non_competition_score', 'boardindpw',
                         'boardsizew', 'busyw', 'pct_blockw', 'logatw', 'exp_roa',
                         'rdintw', 'capintw', 'leverage', 'divyieldw']
    FIRM_CAT_COLS = ['compindustry', 'ba_state', 'rd_control', 'dpayer']
    FIRM_RAW_COLS = FIRM_NUMERIC_COLS + FIRM_CAT_COLS + ['fiscalyear']

    # Target & Weights
    TARGET_COL = 'match_means'
    WEIGHT_COL = 'sd_match_means'

    @property
    def all_required_cols(self) -> List[str]:
        """All unique columns required from the CSV."""
        return sorted(set(self.ID_COLS + self.CEO_RAW_COLS + self.FIRM_RAW_COLS
                          + [self.TARGET_COL, self.WEIGHT_COL]))
