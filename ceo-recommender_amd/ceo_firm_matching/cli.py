"""Command line entry (reference ``cli.py:17-93``): ``python -m ceo_firm_matching.cli --synthetic``.

Runs the reference pipeline -- synthetic or CSV data, DataProcessor,
train/val split (0.2, random_state 42), DataLoader(bs=256, shuffle=True),
``train_model`` -- on the fused HIP engine.  The explainability / heatmap
consumers that follow training in the reference (``cli.py:61-89``) are outside
this build's scope; ``--save`` writes the trained
``state_dict`` instead.
"""
import argparse
import os

import torch
from sklearn.model_selection import train_test_split
from torch.utils.data import DataLoader

from .config import Config
from .data import CEOFirmDataset, DataProcessor
from .training import train_model


def main(argv=None):
    parser = argparse.ArgumentParser(description="Train Two Towers Model")
    parser.add_argument('--synthetic', action='store_true', help='Use synthetic data for verification')
    parser.add_argument('--epochs', type=int, default=None, help='override Config.EPOCHS')
    parser.add_argument('--save', type=str, default=None, help='write the trained state_dict here')
    args = parser.parse_args(argv)

    config = Config()
    if args.epochs is not None:
        config.EPOCHS = args.epochs
    print(f"Running Two Towers Model on {config.DEVICE}")
    processor = DataProcessor(config)
    if args.synthetic:
        print("Using SYNTHETIC data...")
        from .synthetic import generate_synthetic_data
        raw_df = generate_synthetic_data(1000)
    else:
        raw_df = processor.load_data()
    if raw_df.empty:
        return None
    df_clean = processor.prepare_features(raw_df)
    train_df, val_df = train_test_split(df_clean, test_size=0.2, random_state=42)
    print(f"Train size: {len(train_df)}, Val size: {len(val_df)}")
    processor.fit(train_df)
    train_data = processor.transform(train_df)
    val_data = processor.transform(val_df)
    train_loader = DataLoader(CEOFirmDataset(train_data), batch_size=256, shuffle=True)
    val_loader = DataLoader(CEOFirmDataset(val_data), batch_size=256, shuffle=False)
    model = train_model(train_loader, val_loader, train_data, config)
    if model is not None and args.save:
        os.makedirs(os.path.dirname(os.path.abspath(args.save)), exist_ok=True)
        torch.save(model.state_dict(), args.save)
        print(f"saved {args.save}")
    return model


if __name__ == "__main__":
    main()
