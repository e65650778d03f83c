"""``src.model``: the GAN modules (native engine on CUDA tensors)."""
from deeplearninginassetpricing_paperreplication_amd.models.gan import (  # noqa: F401
    AssetPricingGAN, MacroLSTM, MomentNetwork, SDFNetwork, SimpleSDF)
