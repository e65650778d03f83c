"""Time the UNMODIFIED reference (read-only oracle at /root/reference) on the bench config.

Measures seconds per epoch of each phase exactly as `train_3phase` runs them
(phase 1/3 epoch = train_epoch + evaluate(valid) + evaluate(test); phase 2 = train_epoch)
on the synthetic real-sized panel used by bench.py, and derives epochs/sec for the standard
256/64/1024 schedule mix. CPU only; writes JSON to stdout.
"""
import argparse
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, "/root/repo")
sys.path.append("/root/reference")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=3)
    ap.add_argument("--threads", type=int, default=8)
    a = ap.parse_args()
    torch.set_num_threads(a.threads)
    from src import model as RM, train as RT  # reference package (oracle)
    from bench import make_panel, BENCH
    from deeplearninginassetpricing_paperreplication_amd.config import default_cli_config
    tr, va, te = make_panel(seed=0)
    cfg = default_cli_config(BENCH["M"], BENCH["F"])
    torch.manual_seed(0)
    model = RM.AssetPricingGAN(cfg)
    opt_s = torch.optim.Adam(model.sdf_net.parameters(), lr=1e-3)
    opt_m = torch.optim.Adam(model.moment_net.parameters(), lr=1e-3)
    dev = torch.device("cpu")
    res = {}
    for phase, opt, scope, evals in (("unconditional", opt_s, "sdf", True), ("moment", opt_m, "moment", False),
                                     ("conditional", opt_s, "sdf", True)):
        ts = []
        for e in range(a.epochs + 1):
            t0 = time.time()
            RT.train_epoch(model, opt, tr, dev, phase=phase, scope=scope)
            if evals:
                RT.evaluate(model, va, dev)
                RT.evaluate(model, te, dev)
            if e > 0:
                ts.append(time.time() - t0)
        res[phase] = float(np.median(ts))
    mix = 256 * res["unconditional"] + 64 * res["moment"] + 1024 * res["conditional"]
    res["epochs_per_s_3phase_mix"] = 1344 / mix
    res["full_schedule_min"] = mix / 60
    res["threads"] = a.threads
    print(json.dumps(res))


if __name__ == "__main__":
    main()
