"""Probe of the SDF tower backward on the bench panel (600x3000x46, M = 178): runs the phase-3
backward ``--iters`` times through ``Engine.backward_only`` and prints the one-pass kernel's
in-kernel timestamps (k_tbwd.hip g_tb_ts: start, staged, loop done, slab stored for the first and
the last workgroup). Used under ``rocprofv3 --pmc`` for counter passes of the backward alone.

    python tools/tbwd_probe.py [--iters 20] [--models 1] [--sliced]
"""
from __future__ import annotations

import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--models", type=int, default=1)
    ap.add_argument("--sliced", action="store_true", help="DLAP_TBWD=0: the sliced k_mlp_bwd_sdf")
    ap.add_argument("--hidden", type=int, nargs="+", default=[64, 64])
    a = ap.parse_args()
    if a.sliced:
        os.environ["DLAP_TBWD"] = "0"
    import torch
    from bench import make_panel
    from deeplearninginassetpricing_paperreplication_amd.config import default_cli_config
    from deeplearninginassetpricing_paperreplication_amd.engine.runner import GANEngine
    from deeplearninginassetpricing_paperreplication_amd.models.gan import AssetPricingGAN
    from deeplearninginassetpricing_paperreplication_amd.ops import native
    mod = native.load(required=True)
    tr, va, te = make_panel(seed=0, device="cuda", keep_on_device=True)
    cfg = default_cli_config(178, 46, hidden_dim=a.hidden)
    eng = GANEngine(AssetPricingGAN(cfg).spec, a.models, max_epochs=8)
    eng.set_data(tr, va, te)
    for g in range(a.models):
        torch.manual_seed(g)
        eng.set_model(g, AssetPricingGAN(cfg), g)
    for _ in range(a.iters):
        eng.eng.backward_only(3)
    ts = mod.Engine.tbwd_timestamps() if hasattr(mod.Engine, "tbwd_timestamps") else []
    if ts and not a.sliced:
        us = lambda x, y: (ts[y] - ts[x]) / 100.0      # 100 MHz wall clock -> us
        print(f"tbwd first wg: stage {us(0, 1):.2f} loop {us(1, 2):.2f} reduce+store {us(2, 3):.2f} us")
        print(f"tbwd last  wg: stage {us(4, 5):.2f} loop {us(5, 6):.2f} reduce+store {us(6, 7):.2f} us; "
              f"first start -> last end {(ts[7] - ts[0]) / 100.0:.2f} us")
    print("desc", {k: eng.desc[k] for k in ("tbwd", "tps_s", "ntile_s")})


if __name__ == "__main__":
    main()
