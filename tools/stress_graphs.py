"""Engine / epoch-graph churn stress test: build an engine, run pipelined epoch graphs of all
three phases, destroy it, repeat. Prints per-iteration process resources (threads, open fds,
RSS) so a resource leak in the runtime (graph executors, streams, queues) shows up as a trend.

    python tools/stress_graphs.py [iterations] [wide]
"""
from __future__ import annotations

import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _res():
    with open("/proc/self/status") as f:
        st = dict(l.split(":", 1) for l in f if ":" in l)
    return (int(st["Threads"]), len(os.listdir("/proc/self/fd")), int(st["VmRSS"].split()[0]) // 1024)


def main():
    import torch
    from deeplearninginassetpricing_paperreplication_amd.config import default_cli_config
    from deeplearninginassetpricing_paperreplication_amd.data.synthetic import generate_panel_fast
    from deeplearninginassetpricing_paperreplication_amd.engine.runner import GANEngine
    from deeplearninginassetpricing_paperreplication_amd.models.gan import AssetPricingGAN
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    mode = sys.argv[2] if len(sys.argv) > 2 else "fused"     # fused | wide | alt
    torch.cuda.set_device(0)
    ret, feats, mask, mac = generate_panel_fast(36, 160, 46, 8, seed=0)
    b = {"returns": ret, "individual_features": feats, "mask": mask, "macro_features": mac}
    cfg = default_cli_config(8, 46)
    t0 = time.time()
    eng = None
    for it in range(n):
        wide = mode == "wide" or (mode == "alt" and it % 2 == 1)
        os.environ["DLAP_WIDE"] = "1" if wide else "0"
        torch.manual_seed(0)
        new = GANEngine(AssetPricingGAN(cfg).spec, 1, max_epochs=64)
        new.set_data(b, b, b)
        new.set_model(0, AssetPricingGAN(cfg), 7)
        eng = new                                  # the previous engine dies here
        for ph, k in ((1, 4), (2, 2), (3, 4)):
            eng.eng.begin_phase(ph)
            eng.run(ph, k, 1e-3, 1, 1.0, True)
        eng.eng.sync()
        th, fd, rss = _res()
        print(f"iter {it} threads {th} fds {fd} rss_mb {rss} t {time.time() - t0:.1f}s", flush=True)


if __name__ == "__main__":
    main()
