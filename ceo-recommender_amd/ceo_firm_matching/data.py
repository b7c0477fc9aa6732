"""Data preparation (mirrors the reference ``ceo_firm_matching/data.py``).

``DataProcessor`` keeps the reference's stages and outputs (``data.py:16-177``:
dropna, ``tenure``, ``weights = 1/(sd^2+1e-6)``, LabelEncoder codes with
unknown labels mapped to 0, StandardScaler on the numeric columns, the same
tensor dict + metadata keys) but encodes categories with one vectorised
``searchsorted`` per column instead of the reference's per-element Python
``encoder.transform([x])`` (``data.py:97-100``).  ``CEOFirmDataset`` is the
same per-sample dataset (``data.py:180-198``); the fused training loop never
calls ``__getitem__``: it uploads ``dataset.data`` once and gathers on the GPU.
"""
from typing import Any, Dict, List, Optional

import numpy as np
import pandas as pd
import torch
from sklearn.preprocessing import LabelEncoder, StandardScaler
from torch.utils.data import Dataset

from .config import Config


class DataProcessor:
    """Loading, cleaning, feature engineering, encoding and scaling."""

    def __init__(self, config: Config):
        self.cfg = config
        self.encoders: Dict[str, LabelEncoder] = {}
        self.scalers: Dict[str, StandardScaler] = {'firm': StandardScaler(), 'ceo': StandardScaler()}
        self.final_firm_numeric = list(self.cfg.FIRM_NUMERIC_COLS)
        self.final_ceo_numeric = list(self.cfg.CEO_NUMERIC_COLS) + ['tenure']
        self.processed_df: Optional[pd.DataFrame] = None

    def load_data(self) -> pd.DataFrame:
        print(f"Loading data from {self.cfg.DATA_PATH}...")
        try:
            df = pd.read_csv(self.cfg.DATA_PATH, on_bad_lines='skip')
        except FileNotFoundError:
            print(f"Error: File not found at {self.cfg.DATA_PATH}")
            return pd.DataFrame()
        missing = [c for c in self.cfg.all_required_cols if c not in df.columns]
        if missing:
            print(f"Error: Missing essential columns: {missing}")
            return pd.DataFrame()
        return df[self.cfg.all_required_cols].copy()

    def prepare_features(self, df: pd.DataFrame) -> pd.DataFrame:
        if df.empty:
            return df
        n0 = len(df)
        df = df.dropna().copy()
        print(f"Dropped {n0 - len(df)} rows with NaNs. Final count: {len(df)}")
        df['tenure'] = (df['fiscalyear'] - df['ceo_year']).clip(lower=0)
        df['weights'] = 1 / (df[self.cfg.WEIGHT_COL] ** 2 + 1e-6)
        return df

    def fit(self, df: pd.DataFrame):
        print("Fitting scalers and encoders on training data...")
        for col in list(self.cfg.FIRM_CAT_COLS) + list(self.cfg.CEO_CAT_COLS):
            enc = LabelEncoder()
            enc.fit(df[col].astype(str))
            self.encoders[col] = enc
        self.scalers['firm'].fit(df[self.final_firm_numeric])
        self.scalers['ceo'].fit(df[self.final_ceo_numeric])

    @staticmethod
    def _codes(encoder: LabelEncoder, values: pd.Series) -> np.ndarray:
        classes = np.asarray(encoder.classes_)
        v = values.to_numpy()
        pos = np.searchsorted(classes, v)
        pos_c = np.minimum(pos, len(classes) - 1)
        known = classes[pos_c] == v
        return np.where(known, pos_c, 0).astype(np.int64)

    def transform(self, df: pd.DataFrame) -> Dict[str, Any]:
        if df.empty:
            return {}
        df = df.copy()
        for col in list(self.cfg.FIRM_CAT_COLS) + list(self.cfg.CEO_CAT_COLS):
            df[f'{col}_code'] = self._codes(self.encoders[col], df[col].astype(str))
        df[self.final_firm_numeric] = self.scalers['firm'].transform(df[self.final_firm_numeric])
        df[self.final_ceo_numeric] = self.scalers['ceo'].transform(df[self.final_ceo_numeric])
        self.processed_df = df
        return self._to_tensors(df)

    def _to_tensors(self, df: pd.DataFrame) -> Dict[str, Any]:
        metadata = {
            'n_firm_numeric': len(self.final_firm_numeric),
            'firm_cat_counts': [len(self.encoders[c].classes_) for c in self.cfg.FIRM_CAT_COLS],
            'n_ceo_numeric': len(self.final_ceo_numeric),
            'ceo_cat_counts': [len(self.encoders[c].classes_) for c in self.cfg.CEO_CAT_COLS],
        }
        firm_cat = np.stack([df[f'{c}_code'].values for c in self.cfg.FIRM_CAT_COLS], axis=1)
        ceo_cat = np.stack([df[f'{c}_code'].values for c in self.cfg.CEO_CAT_COLS], axis=1)
        tensors = {
            'firm_numeric': torch.tensor(df[self.final_firm_numeric].values, dtype=torch.float32),
            'firm_cat': torch.tensor(firm_cat, dtype=torch.long),
            'ceo_numeric': torch.tensor(df[self.final_ceo_numeric].values, dtype=torch.float32),
            'ceo_cat': torch.tensor(ceo_cat, dtype=torch.long),
            'target': torch.tensor(df[self.cfg.TARGET_COL].values, dtype=torch.float32).view(-1, 1),
            'weights': torch.tensor(df['weights'].values, dtype=torch.float32).view(-1, 1),
        }
        return {**tensors, **metadata}

    def get_feature_names(self) -> List[str]:
        return (self.final_firm_numeric + list(self.cfg.FIRM_CAT_COLS)
                + self.final_ceo_numeric + list(self.cfg.CEO_CAT_COLS))

    def get_flat_features(self, df: pd.DataFrame) -> np.ndarray:
        d = self.transform(df)
        return np.hstack([d['firm_numeric'].numpy(), d['firm_cat'].numpy(),
                          d['ceo_numeric'].numpy(), d['ceo_cat'].numpy()])


class CEOFirmDataset(Dataset):
    """Per-sample dataset over the tensor dict (reference data.py:180-198)."""

    KEYS = ('firm_numeric', 'firm_cat', 'ceo_numeric', 'ceo_cat', 'target', 'weights')

    def __init__(self, data_dict: Dict[str, Any]):
        self.data = data_dict
        self.length = len(data_dict['target'])

    def __len__(self):
        return self.length

    def __getitem__(self, idx):
        return {k: self.data[k][idx] for k in self.KEYS}
