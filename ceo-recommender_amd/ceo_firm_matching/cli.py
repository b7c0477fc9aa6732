"""Command line entry (reference ``cli.py:17-93``): ``python -m ceo_firm_matching.cli --synthetic``.

Runs the reference pipeline -- synthetic or CSV data, DataProcessor,
train/val split (0.2, random_state 42), DataLoader(bs=256, shuffle=True),
``train_model`` on the fused HIP engine, then the reference's consumers
(``cli.py:61-89``): partial-dependence plots and the eleven interaction
heatmaps, each evaluated as one batched eval forward (``explain.py``,
``visualization.py``).  ``--no-plots`` skips them; ``--save`` writes the
trained ``state_dict``.
"""
import argparse
import os

import torch
from sklearn.model_selection import train_test_split
from torch.utils.data import DataLoader

from .config import Config
from .data import CEOFirmDataset, DataProcessor
from .training import train_model


# the interaction heatmaps the reference CLI draws after training (cli.py:75-89)
HEATMAPS = [
    ('logatw', 'Age', 'heatmap_size_age.svg'), ('logatw', 'Output', 'heatmap_size_skill.svg'),
    ('exp_roa', 'tenure', 'heatmap_perf_exp.svg'), ('rdintw', 'Output', 'heatmap_rd_skill.svg'),
    ('rdintw', 'Age', 'heatmap_rd_age.svg'), ('logatw', 'ivy', 'heatmap_size_ivy.svg'),
    ('tenure', 'boardindpw', 'heatmap_tenure_boardind.svg'), ('maxedu', 'rdintw', 'heatmap_maxedu_rd.svg'),
    ('maxedu', 'capintw', 'heatmap_maxedu_capx.svg'), ('logatw', 'm', 'heatmap_size_mover.svg'),
    ('leverage', 'Age', 'heatmap_leverage_age.svg'),
]


def main(argv=None):
    parser = argparse.ArgumentParser(description="Train Two Towers Model")
    parser.add_argument('--synthetic', action='store_true', help='Use synthetic data for verification')
    parser.add_argument('--epochs', type=int, default=None, help='override Config.EPOCHS')
    parser.add_argument('--save', type=str, default=None, help='write the trained state_dict here')
    parser.add_argument('--no-plots', action='store_true', help='skip the PDP / heatmap consumers')
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
    if model is not None and not args.no_plots:
        from .explain import ModelWrapper, explain_model_pdp
        from .visualization import plot_interaction_heatmap
        wrapper = ModelWrapper(model, processor)
        explain_model_pdp(wrapper, val_df, list(config.FIRM_NUMERIC_COLS) + list(config.CEO_NUMERIC_COLS) + ['tenure'])
        processor.transform(val_df)
        for fx, fy, name in HEATMAPS:
            plot_interaction_heatmap(model, processor, fx, fy, name)
    if model is not None and args.save:
        os.makedirs(os.path.dirname(os.path.abspath(args.save)), exist_ok=True)
        torch.save(model.state_dict(), args.save)
        print(f"saved {args.save}")
    return model


if __name__ == "__main__":
    main()
