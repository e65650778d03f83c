"""Per-tensor LSTM gradient errors of the fp32 engine vs torch autograd (debug aid)."""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
from deeplearninginassetpricing_paperreplication_amd.config import default_cli_config
from deeplearninginassetpricing_paperreplication_amd.data.synthetic import generate_panel_fast
from deeplearninginassetpricing_paperreplication_amd.models.gan import AssetPricingGAN
from deeplearninginassetpricing_paperreplication_amd.engine.runner import GANEngine, flatten_state

for T in (36, 120):
    ret, feats, mask, mac = generate_panel_fast(T, 160, 46, 8, seed=0)
    mac = (mac - mac.mean(0)) / (mac.std(0, unbiased=False) + 1e-8)
    b = {"returns": ret, "individual_features": feats, "mask": mask, "macro_features": mac}
    cfg = default_cli_config(8, 46, dropout=0.0)
    for phase, pname in ((1, "unconditional"), (3, "conditional")):
        torch.manual_seed(0)
        model = AssetPricingGAN(cfg)
        eng = GANEngine(model.spec, 1, max_epochs=8, precision="fp32")
        eng.set_data(b)
        eng.set_model(0, model, 7)
        eng.eng.backward_only(phase)
        got = eng.eng.get_grads(0)
        model.zero_grad()
        o = model(b["macro_features"], b["individual_features"], b["returns"], b["mask"], phase=pname)
        o["loss"].backward()
        ref = flatten_state({k: (p.grad if p.grad is not None else torch.zeros_like(p))
                             for k, p in model.named_parameters()}, model.spec)
        off = 0
        for k, s in model.spec.param_layout():
            n = int(np.prod(s))
            if "macro_lstm" in k or k.endswith("fc_layers.0.weight"):
                g, r = got[off:off + n], ref[off:off + n]
                print(f"T={T} ph={phase} {k:45s} rel={np.linalg.norm(g - r) / (np.linalg.norm(r) + 1e-30):.2e} |r|={np.linalg.norm(r):.3e}")
            off += n
