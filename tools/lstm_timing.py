"""In-kernel phase timing of the serial LSTM kernels at the bench config (GPU).

Prints, for the last launch of each kernel: staging / recurrence / tail durations in us
(wall_clock64 at 100 MHz), with the eval branch pipelined or not.
"""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from deeplearninginassetpricing_paperreplication_amd.config import default_cli_config  # noqa: E402
from deeplearninginassetpricing_paperreplication_amd.engine.runner import GANEngine  # noqa: E402
from deeplearninginassetpricing_paperreplication_amd.models.gan import AssetPricingGAN  # noqa: E402
from deeplearninginassetpricing_paperreplication_amd.ops import native  # noqa: E402


def main():
    tr, va, te = bench.make_panel(seed=0, device="cuda")
    cfg = default_cli_config(bench.BENCH["M"], bench.BENCH["F"])
    eng = GANEngine(AssetPricingGAN(cfg).spec, 1, max_epochs=64)
    eng.set_data(tr, va, te)
    torch.manual_seed(0)
    eng.set_model(0, AssetPricingGAN(cfg), 1)
    mod = native.load()
    for pipe in (False, True):
        eng.eng.set_pipeline(pipe)
        eng.eng.begin_phase(3)
        eng.run(3, 6, 1e-3, 1, 1.0, True)
        eng.eng.sync()
        ts = np.array(mod.Engine.rnn_timestamps(), dtype=np.int64)
        us = lambda a, b: (ts[b] - ts[a]) / 100.0  # noqa: E731
        print(f"pipeline={pipe}")
        print(f"  k_lstm_gl train: stage {us(0, 1):7.1f}  recur {us(1, 2):7.1f}  tail {us(2, 3):7.1f}  total {us(0, 3):7.1f}")
        print(f"  k_lstm_gl eval : stage {us(4, 5):7.1f}  recur {us(5, 6):7.1f}  tail {us(6, 7):7.1f}  total {us(4, 7):7.1f}")
        print(f"  k_lstm_bwd     : stage {us(8, 9):7.1f}  bptt  {us(9, 10):7.1f}  grads {us(10, 11):7.1f} total {us(8, 11):7.1f}")
        if ts[13] > ts[9] and ts[15] > ts[13]:     # dense-state path: step matrices | chain | gates
            print(f"    dense-state  : matrices {us(9, 13):7.1f}  chain {us(13, 15):7.1f}  gates {us(15, 10):7.1f}")
        if eng.eng.fused_info()["fused_tail"] and ts[16] > ts[9]:    # k_lstm_tail: dpp wait, W_ih
            print(f"    fused tail   : pre-pass->dpp in LDS {us(9, 16):7.1f}  pair maps {us(16, 13):7.1f}  "
                  f"W_hh grads {us(10, 11):7.1f}  last W_ih block done {us(10, 17):7.1f} after the gates")
        if eng.eng.fused_info().get("adam_in_tail") and pipe and ts[20] > ts[18]:
            print(f"    tail Adam    : last arrival {us(10, 18):7.1f} after the gates  Adam block 0 released "
                  f"{us(18, 19):7.1f}  update done {us(19, 20):7.1f} later")
        print(f"  k_proj tile0   : total {us(12, 14):7.1f}")
        m = np.array(mod.Engine.mlp_timestamps(), dtype=np.int64)
        um = lambda a, b: (m[b] - m[a]) / 100.0  # noqa: E731
        print(f"  k_mlp_fwd blk0 : stage {um(0, 1):7.1f}  tile1 {um(1, 2):7.1f}  rest {um(2, 3):7.1f}")
        print(f"  k_mlp_fwd last : stage {um(4, 5):7.1f}  tile1 {um(5, 6):7.1f}  rest {um(6, 7):7.1f}  "
              f"start-lag {(m[4] - m[0]) / 100.0:7.1f}  end-lag {(m[7] - m[3]) / 100.0:7.1f}")
        if eng.eng.fused_forward(3):
            print(f"  fused fwd blk0 : start->recur {um(8, 9):7.1f}  recur {um(9, 10):7.1f}  flush {um(10, 11):7.1f}  "
                  f"publisher-end {um(8, 12):7.1f}  first tower start {(m[0] - m[8]) / 100.0:7.1f}  "
                  f"last tower end {(max(m[3], m[7]) - m[8]) / 100.0:7.1f}")
            if len(m) > 20 and m[18] > m[17] > 0:
                print(f"  fused fwd eval : last evaluation WG start {um(8, 16):7.1f}  first tile {um(16, 20):7.1f} "
                      f"(weights requested {um(16, 21):7.1f})  recurrence start {um(16, 17):7.1f}  recur {um(17, 18):7.1f}  "
                      f"end {um(8, 18):7.1f} (from blk0 start)")
        lt = np.array(mod.Engine.loss_timestamps(), dtype=np.int64)
        ul = lambda a, b: (lt[b] - lt[a]) / 100.0  # noqa: E731
        print(f"  k_job_metrics  : losses {ul(0, 1):7.1f}  pass0 {ul(1, 2):7.1f}  pass1 {ul(2, 3):7.1f}")


if __name__ == "__main__":
    main()
