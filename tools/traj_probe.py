"""fp32 engine trajectory vs the CPU trainer for one config branch under engine switches (numerics
triage). Usage: python tools/traj_probe.py '{"num_condition_moment": 32}' [ENV=VAL ...]
Prints per-step relative errors of (loss, grad norm) and the worst parameter tensor."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    upd = json.loads(sys.argv[1])
    for kv in sys.argv[2:]:
        k, v = kv.split("=", 1)
        os.environ[k] = v
    import copy
    import numpy as np
    import torch
    from deeplearninginassetpricing_paperreplication_amd.config import default_cli_config
    from deeplearninginassetpricing_paperreplication_amd.models.gan import AssetPricingGAN
    import test_engine_fp32_gpu as T
    from deeplearninginassetpricing_paperreplication_amd.ops import native
    native.load(required=True)
    splits = T._splits()
    cfg = default_cli_config(8, 46, dropout=0.0)
    cfg.update(upd)
    torch.manual_seed(0)
    model = AssetPricingGAN(cfg)
    gm = copy.deepcopy(model)
    eng, got = T._gpu_trajectory(gm, splits, T.SCHED, 1e-3)
    ref = T._cpu_trajectory(model, splits[0], T.SCHED, 1e-3)
    rel = np.abs(got - ref) / np.maximum(np.abs(ref), 1e-30)
    errs = T._tensor_errors(eng.state_dict(0), model)
    worst = sorted(errs, key=errs.get)[-3:]
    print(json.dumps({"env": sys.argv[2:], "rel_loss": [float(x) for x in rel[:, 0]],
                      "rel_gn": [float(x) for x in rel[:, 1]],
                      "worst": {k: errs[k] for k in worst}, "info": {k: v for k, v in eng.eng.fused_info().items()
                                                                      if k in ("split_graphs", "fused_tail", "adam_in_tail")}}))


if __name__ == "__main__":
    main()
