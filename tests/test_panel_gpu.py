"""Device-side split preparation (csrc/k_panel.hip, ``Engine.set_split_dense``) against the host
compaction ``engine.panel.prepare_split`` (the layout contract, `/root/reference/src/
data_loader.py:42-65` masking): bitwise-equal compacted rows, indices and dense arrays, the same
per-period / per-asset constants, on edge panels (an all-masked period, single-observation
assets, N not a multiple of the block) and in both tower precisions."""
import numpy as np
import pytest
import torch

from deeplearninginassetpricing_paperreplication_amd.config import default_cli_config
from deeplearninginassetpricing_paperreplication_amd.data.synthetic import generate_panel_fast
from deeplearninginassetpricing_paperreplication_amd.engine.panel import prepare_split
from deeplearninginassetpricing_paperreplication_amd.models.gan import AssetPricingGAN

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from deeplearninginassetpricing_paperreplication_amd.ops import native
    native.load(required=True)


def _panel(T, N, F, M, seed):
    ret, feats, mask, mac = generate_panel_fast(T, N, F, M, seed=seed)
    mask = mask.clone()
    mask[3] = False                      # an all-masked period
    mask[:, 7] = False
    mask[5, 7] = True                    # an asset observed once
    ret = ret.clone()
    ret[~mask] = float("nan")            # masked entries must never leak into anything
    return {"returns": ret, "individual_features": feats, "mask": mask, "macro_features": mac}


@pytest.mark.parametrize("precision,N", [("bf16", 777), ("fp32", 300)])
def test_device_compaction_equals_host(precision, N):
    from deeplearninginassetpricing_paperreplication_amd.engine.runner import GANEngine
    T, F, M = 40, 46, 8
    b = _panel(T, N, F, M, seed=2)
    cfg = default_cli_config(M, F)
    eng = GANEngine(AssetPricingGAN(cfg).spec, 1, max_epochs=4, precision=precision)
    dev = {k: v.cuda() for k, v in b.items()}
    eng.set_data(dev)
    got = eng.eng.read_split(0)
    ref = prepare_split(b, eng.KP, fp32=precision == "fp32")
    assert got["R"] == ref.R == int(b["mask"].sum())
    np.testing.assert_array_equal(np.asarray(got["X"]).view(np.uint16), ref.X.reshape(-1))
    np.testing.assert_array_equal(got["rowti"], ref.rowti.reshape(-1))
    np.testing.assert_array_equal(got["row_ptr"], ref.row_ptr)
    np.testing.assert_array_equal(got["Rm"], ref.Rm)
    np.testing.assert_array_equal(got["mask"], ref.mask)
    np.testing.assert_array_equal(got["macro"], ref.macro.reshape(-1))
    ti = ref.rowti
    np.testing.assert_array_equal(got["Rc"], ref.Rm.reshape(T, N)[ti[:, 0], ti[:, 1]])
    m = ref.mask.reshape(T, N).astype(np.float64)
    r = ref.Rm.reshape(T, N).astype(np.float64)
    nt = m.sum(1)
    nc = np.maximum(nt, 1)
    np.testing.assert_array_equal(got["Nt"], nt.astype(np.float32))
    np.testing.assert_array_equal(got["invNt"], (1.0 / nc).astype(np.float32))
    np.testing.assert_allclose(got["meanR"], ((r * m).sum(1) / nc).astype(np.float32), rtol=2e-7, atol=0)
    np.testing.assert_allclose(got["RR"], (r * r * m).sum(1).astype(np.float32), rtol=2e-7, atol=0)
    np.testing.assert_array_equal(got["invT"], (1.0 / np.maximum(m.sum(0), 1)).astype(np.float32))
    assert got["Nbar"] == np.float32(nc.mean())
    # host inputs take the same device path: identical engine state
    eng2 = GANEngine(AssetPricingGAN(cfg).spec, 1, max_epochs=4, precision=precision)
    eng2.set_data(b)
    got2 = eng2.eng.read_split(0)
    for k in got:
        np.testing.assert_array_equal(np.asarray(got[k]), np.asarray(got2[k]))


def test_compaction_is_fast_on_the_bench_panel():
    """The bench panel (240/60/300 x 3000 x 46, M = 178) is prepared in a few milliseconds per
    split (the eager torch compaction it replaces took ~0.05-0.14 s for the three splits)."""
    import os
    import sys
    import time
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import make_panel
    from deeplearninginassetpricing_paperreplication_amd.engine.runner import GANEngine
    tr, va, te = make_panel(seed=0, device="cuda", keep_on_device=True)
    cfg = default_cli_config(178, 46)
    eng = GANEngine(AssetPricingGAN(cfg).spec, 1, max_epochs=4)
    eng.set_data(tr, va, te)                    # warm-up (first launches)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.set_data(tr, va, te)
    dt = time.perf_counter() - t0
    print(f"device compaction of the three bench splits: {dt * 1e3:.2f} ms")
    assert dt < 0.05
