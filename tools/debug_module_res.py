"""Module API, phase 'moment' with a residual term: the GPU forward's loss components against the
CPU modules (debug print for tests/test_module_autograd_gpu.py::test_moment_phase_with_residual_term)."""
import copy
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from deeplearninginassetpricing_paperreplication_amd.config import default_cli_config  # noqa: E402
from deeplearninginassetpricing_paperreplication_amd.data.synthetic import generate_panel_fast  # noqa: E402
from deeplearninginassetpricing_paperreplication_amd.models.gan import AssetPricingGAN  # noqa: E402
from deeplearninginassetpricing_paperreplication_amd.ops import fused  # noqa: E402

fused.set_precision("fp32")
ret, feats, mask, mac = generate_panel_fast(30, 120, 46, 8, seed=4)
mac = (mac - mac.mean(0)) / (mac.std(0, unbiased=False) + 1e-8)
cfg = default_cli_config(8, 46, dropout=0.0)
cfg["residual_loss_factor"] = 0.5
torch.manual_seed(3)
cpu = AssetPricingGAN(cfg)
gpu = copy.deepcopy(cpu).cuda()
for phase in ("moment", "conditional", "unconditional"):
    oc = cpu(mac, feats, ret, mask, phase=phase)
    og = gpu(mac.cuda(), feats.cuda(), ret.cuda(), mask.cuda(), phase=phase)
    for k in ("loss", "loss_conditional", "loss_unconditional", "loss_residual"):
        print(phase, k, float(oc[k]), float(og[k]))
    print(phase, "weights", float((og["weights"].detach().cpu() - oc["weights"].detach()).abs().max()))
    print(phase, "P", float((og["portfolio_returns"].detach().cpu() - oc["portfolio_returns"].detach()).abs().max()))
