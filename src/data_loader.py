"""``src.data_loader``: npz panel datasets."""
from deeplearninginassetpricing_paperreplication_amd.data.dataset import (  # noqa: F401
    AssetPricingDataset, create_data_loaders, create_small_sample)
