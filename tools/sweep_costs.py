"""Measure the per-epoch cost of every architecture bucket of the sweep grids on one MI355X and
write `deeplearninginassetpricing_paperreplication_amd/parallel/sweep_costs.json`, the table the
sweep's longest-processing-time-first rank assignment reads (`parallel/sweep.py:bucket_cost`).

For each distinct architecture: an 8-member engine on the 600 x 3000 x 46 (M = 178) panel, a
short warmup (graph capture), then timed epochs of each phase; the recorded cost is the
schedule-weighted epoch time (256 : 64 : 1024) in ms.

Usage (GPU box): python tools/sweep_costs.py [--grid paper|baseline|both] [--epochs 12]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", choices=["paper", "baseline", "both"], default="both")
    ap.add_argument("--epochs", type=int, default=12)
    ap.add_argument("--out", default=None)
    ap.add_argument("--only", default=None, help="architectures whose key contains this string")
    a = ap.parse_args()
    from bench import make_panel
    from deeplearninginassetpricing_paperreplication_amd.config import ModelSpec
    from deeplearninginassetpricing_paperreplication_amd.engine.runner import GANEngine
    from deeplearninginassetpricing_paperreplication_amd.models.gan import AssetPricingGAN
    from deeplearninginassetpricing_paperreplication_amd.parallel import sweep
    torch.cuda.set_device(0)
    tr, va, te = make_panel(seed=0, device="cuda:0")
    entries = []
    if a.grid in ("paper", "both"):
        entries += sweep.paper_grid(178, 46)
    if a.grid in ("baseline", "both"):
        entries += sweep.baseline_grid(178, 46)
    seen = {}
    for cfg, _, _ in entries:
        spec = ModelSpec.from_config(cfg)
        seen.setdefault(sweep.arch_key(spec), cfg)
    out = {}
    n = a.epochs
    for key, cfg in seen.items():
        if a.only and a.only not in key:
            continue
        spec = ModelSpec.from_config(cfg)
        t0 = time.perf_counter()
        eng = GANEngine(spec, n_models=8, max_epochs=4 * n + 16)
        eng.set_data(tr, va, te)
        for g in range(8):
            torch.manual_seed(g)
            eng.set_model(g, AssetPricingGAN(cfg), g)
        for ph in (1, 2, 3):                     # warmup + graph capture
            eng.eng.begin_phase(ph)
            eng.run(ph, 2, 1e-3, 0)
        eng.eng.sync()
        per = []
        for ph in (1, 2, 3):
            eng.eng.begin_phase(ph)
            eng.eng.sync()
            tp = time.perf_counter()
            eng.run(ph, n, 1e-3, 0)
            eng.eng.sync()
            per.append((time.perf_counter() - tp) / n * 1e3)
        ms = (256 * per[0] + 64 * per[1] + 1024 * per[2]) / 1344
        out[key] = round(ms, 4)
        print(f"{key:28s} {ms:8.3f} ms/epoch  phases {[round(x, 3) for x in per]}  "
              f"(setup {time.perf_counter() - t0:.1f} s)", flush=True)
        del eng
        torch.cuda.empty_cache()
    rec = {"what": "schedule-weighted epoch time (ms) of an 8-member engine, 600x3000x46 panel, M=178",
           "device": torch.cuda.get_device_name(0), "epochs_timed_per_phase": n, "ms_per_epoch": out}
    path = a.out or os.path.join(ROOT, "deeplearninginassetpricing_paperreplication_amd", "parallel",
                                 "sweep_costs.json")
    with open(path, "w") as fh:
        json.dump(rec, fh, indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
