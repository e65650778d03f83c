"""MI355X-native Chen–Pelger–Zhu "Deep Learning in Asset Pricing" framework.

Same public surface as the reference package `/root/reference/src/__init__.py:8-39` (12 names +
``__version__``); the GPU path of every model/training call runs the native HIP engine
(``engine/``, ``csrc/``), the CPU path is a vectorised PyTorch implementation of the same
semantics. Distributed ensemble / sweep drivers live in ``parallel/``.
"""
from .models.gan import AssetPricingGAN, MomentNetwork, SDFNetwork, SimpleSDF
from .data.dataset import AssetPricingDataset, create_data_loaders, create_small_sample
from .train.trainer import evaluate, train_3phase, train_epoch


def download_all_data(*args, **kwargs):
    """Download the real dataset (see ``data.download``; needs ``gdown`` + network)."""
    from .data.download import download_all_data as _dl
    return _dl(*args, **kwargs)


def check_data_exists(*args, **kwargs):
    """Which of the six required ``.npz`` files exist under a data directory."""
    from .data.download import check_data_exists as _chk
    return _chk(*args, **kwargs)


__version__ = "0.1.0"
__all__ = [
    "AssetPricingGAN", "SDFNetwork", "MomentNetwork", "SimpleSDF",
    "AssetPricingDataset", "create_data_loaders", "create_small_sample",
    "train_3phase", "train_epoch", "evaluate",
    "download_all_data", "check_data_exists",
]
