"""Drop-in module paths of the reference package (``src.train``, ``src.model`` ...).

Every module here re-exports the MI355X-native implementation from
``deeplearninginassetpricing_paperreplication_amd`` so code and commands written for the
reference (``python -m src.train --data_dir ...``) run unchanged.
"""
from deeplearninginassetpricing_paperreplication_amd import (  # noqa: F401
    AssetPricingDataset, AssetPricingGAN, MomentNetwork, SDFNetwork, SimpleSDF, __version__,
    check_data_exists, create_data_loaders, create_small_sample, download_all_data, evaluate,
    train_3phase, train_epoch)

__all__ = [
    "AssetPricingGAN", "SDFNetwork", "MomentNetwork", "SimpleSDF",
    "AssetPricingDataset", "create_data_loaders", "create_small_sample",
    "train_3phase", "train_epoch", "evaluate",
    "download_all_data", "check_data_exists",
]
