"""Training entry point (drop-in for the reference ``training.py:15-64``).

``train_model(train_loader, val_loader, metadata, config)`` keeps the
reference signature, stdout lines and semantics: the model is built with the
same RNG draws, batches come in exactly the order the DataLoader would yield
them (its RandomSampler is driven from the same global generator), the last
partial batch is kept, Adam(lr=config.LEARNING_RATE), and every 5th epoch
prints the mean of the batch losses.

On a HIP device the loop runs on the fused engine (``engine.FusedTrainer``):
the dataset behind a ``CEOFirmDataset`` loader is uploaded to HBM once and
every step is one C-ABI call (six kernels) with no per-step host sync.  Any
other loader is consumed batch by batch (``.to(DEVICE)``) through the same
fused step.  On CPU the reference loop runs with ATen ops.
"""
from __future__ import annotations

from typing import Dict, List, Optional

import torch
import torch.optim as optim
from torch.utils.data import DataLoader

from .config import Config
from .engine import DATA_KEYS, FusedTrainer
from .model import CEOFirmMatcher


def sampler_batches(loader: DataLoader) -> List[List[int]]:
    """Index lists of one epoch of ``loader``, consuming the global RNG exactly
    as ``iter(loader)`` does (torch 2.10 ``_BaseDataLoaderIter.__init__`` draws
    the worker base seed first; the RandomSampler draws its seed lazily)."""
    torch.empty((), dtype=torch.int64).random_(generator=loader.generator)
    return [list(b) for b in loader.batch_sampler]


def _resident_data(loader: DataLoader) -> Optional[Dict[str, torch.Tensor]]:
    ds = loader.dataset
    data = getattr(ds, "data", None)
    if not isinstance(data, dict) or any(k not in data for k in DATA_KEYS):
        return None
    if loader.batch_sampler is None or getattr(loader, "_dataset_kind", 0) != 0:
        return None
    if loader.collate_fn is not torch.utils.data.default_collate:
        return None
    return {k: data[k] for k in DATA_KEYS}


def train_model(train_loader: DataLoader, val_loader: DataLoader,
                metadata: Dict[str, int], config: Config) -> Optional[CEOFirmMatcher]:
    """Train the CEOFirmMatcher model (reference training.py:15-64)."""
    model = CEOFirmMatcher(metadata, config).to(config.DEVICE)
    print(f"Starting training on {config.DEVICE} for {config.EPOCHS} epochs...")
    if torch.device(config.DEVICE).type == "cuda":
        return _train_fused(model, train_loader, config)
    return _train_cpu(model, train_loader, config)


train = train_model  # the north-star name


def _train_fused(model: CEOFirmMatcher, loader: DataLoader, config: Config) -> CEOFirmMatcher:
    dev = model.logit_scale.device
    bs = loader.batch_size or 1
    trainer = FusedTrainer(model, lr=config.LEARNING_RATE, max_batch=max(bs, 2))
    data = _resident_data(loader)
    if data is not None:
        trainer.set_data(data)
    for epoch in range(config.EPOCHS):
        model.train()
        n_batches = 0
        if data is not None:
            batches = sampler_batches(loader)
            flat = [i for b in batches for i in b]
            rows = torch.tensor(flat, dtype=torch.int64).to(dev, non_blocking=True)
            off = 0
            for b in batches:
                trainer.step(rows, off, len(b))
                off += len(b)
                n_batches += 1
        else:
            for batch in loader:
                batch = {k: v.to(dev) for k, v in batch.items()}
                trainer.set_data(batch)
                trainer.step(None, 0, batch["target"].shape[0])
                n_batches += 1
        if epoch % 5 == 0:
            avg_loss = trainer.pop_loss_sum() / max(n_batches, 1)
            print(f"Epoch {epoch}: Avg Train Loss = {avg_loss:.4f}")
        else:
            trainer.pop_loss_sum(read=False)
    trainer.check_exchange()
    model._trainer = trainer  # keeps optimizer state reachable for callers/tests
    return model


def _train_cpu(model: CEOFirmMatcher, loader: DataLoader, config: Config) -> CEOFirmMatcher:
    optimizer = optim.Adam(model.parameters(), lr=config.LEARNING_RATE)
    for epoch in range(config.EPOCHS):
        model.train()
        total_loss = 0.0
        for batch in loader:
            optimizer.zero_grad()
            preds = model(batch['firm_numeric'], batch['firm_cat'], batch['ceo_numeric'], batch['ceo_cat'])
            loss = (batch['weights'] * (preds - batch['target']) ** 2).mean()
            loss.backward()
            optimizer.step()
            total_loss += loss.item()
        avg_loss = total_loss / len(loader)
        if epoch % 5 == 0:
            print(f"Epoch {epoch}: Avg Train Loss = {avg_loss:.4f}")
    return model
