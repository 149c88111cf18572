"""Learning-rate and KL-annealing schedules (deterministic in the step, so
data-parallel ranks never need to communicate them)."""
from __future__ import annotations


def reference_lr(cfg, epoch: int) -> float:
    """Per-epoch exponential decay (``train.py:78``)."""
    return cfg.learning_rate * (cfg.decay_rate ** epoch)


def vae_lr(cfg, step: int) -> float:
    return (cfg.learning_rate - cfg.min_learning_rate) * (cfg.decay_rate ** step) + cfg.min_learning_rate


def kl_weight(cfg, step: int) -> float:
    """KL annealing: rises from ``kl_weight_start`` towards ``kl_weight``."""
    return cfg.kl_weight - (cfg.kl_weight - cfg.kl_weight_start) * (cfg.kl_decay_rate ** step)
