"""Seeding (reference utils/reproducibility.py:10-35)."""

import random

import numpy as np
import torch

SEED = 42


def set_random_seeds(seed=SEED, exact_reproducibility=False):
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed(seed)
        torch.cuda.manual_seed_all(seed)
    torch.backends.cudnn.deterministic = bool(exact_reproducibility)
    torch.backends.cudnn.benchmark = not exact_reproducibility


def get_device():
    if torch.cuda.is_available():
        return torch.device("cuda"), f"GPU: {torch.cuda.get_device_name(0)}"
    return torch.device("cpu"), "CPU"
