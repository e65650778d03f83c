"""Gram-matrix loss mode of the native engine (csrc/k_gram.hip) on an MI355X.

While the moments are frozen (phases 1 and 3, every evaluation split) the reference losses
(`/root/reference/src/model.py:346-433`) are quadratic forms in the SDF vector s = 1 + P:
L_cond = s^T Gc s / (K N) and L_unc = s^T Gu s / N. These tests check the HIP Gram build against
an fp64 numpy construction from the engine's own cached moments, and the per-epoch quadratic
forms against the dense fp32 asset passes (DLAP_GRAM=0) over a phase 1 -> 2 -> 3 trajectory.
"""
import copy
import os

import numpy as np
import pytest
import torch

from deeplearninginassetpricing_paperreplication_amd.config import default_cli_config
from deeplearninginassetpricing_paperreplication_amd.data.synthetic import generate_panel_fast
from deeplearninginassetpricing_paperreplication_amd.models.gan import AssetPricingGAN

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from deeplearninginassetpricing_paperreplication_amd.ops import native
    native.load(required=True)


def _splits(T=(70, 20, 45), N=203, F=46, M=8, seed=3):
    ret, feats, mask, mac = generate_panel_fast(sum(T), N, F, M, seed=seed)
    mac = (mac - mac[:T[0]].mean(0)) / (mac[:T[0]].std(0, unbiased=False) + 1e-8)
    cuts = [(0, T[0]), (T[0], T[0] + T[1]), (T[0] + T[1], sum(T))]
    return [{"returns": ret[a:b].contiguous(), "individual_features": feats[a:b].contiguous(),
             "mask": mask[a:b].contiguous(), "macro_features": mac[a:b].contiguous()} for a, b in cuts]


def _engine(model, splits, gram, precision="fp32", G=1):
    from deeplearninginassetpricing_paperreplication_amd.engine.runner import GANEngine
    old = os.environ.get("DLAP_GRAM")
    os.environ["DLAP_GRAM"] = "1" if gram else "0"
    try:
        eng = GANEngine(model.spec, G, max_epochs=64, precision=precision)
    finally:
        if old is None:
            os.environ.pop("DLAP_GRAM")
        else:
            os.environ["DLAP_GRAM"] = old
    eng.set_data(*splits)
    for g in range(G):
        eng.set_model(g, model, 7 + g)
    return eng


@pytest.mark.parametrize("K", [8, 4])
def test_gram_matrices_match_fp64_numpy(K):
    """Gc / Gu of every split from the HIP fp64-MFMA build vs numpy fp64 on the same cached
    moments (T not a multiple of the 32-row tiles, N*K not a multiple of the 16-wide chunks)."""
    splits = _splits()
    cfg = default_cli_config(8, 46, dropout=0.0)
    cfg["num_condition_moment"] = K
    torch.manual_seed(0)
    model = AssetPricingGAN(cfg)
    eng = _engine(model, splits, True, G=2)
    eng.eng.refresh_gram()
    for s, b in enumerate(splits):
        T, N = b["mask"].shape
        R = (b["returns"] * b["mask"]).double().numpy()
        Ti = np.maximum(b["mask"].double().sum(0).numpy(), 1.0)
        invT = (1.0 / Ti).astype(np.float32).astype(np.float64)  # the engine's fp32 1/T_i
        a = R * invT[None, :]                                   # [T, N]
        for g in range(2):
            h = eng.eng.read_ws(g, s, "h").astype(np.float64).reshape(T, N, K)
            A = (a[:, :, None] * h).reshape(T, N * K)
            Gc = A @ A.T
            Gu = a @ a.T
            got = eng.eng.read_gram(g, s).reshape(2, T, T)
            assert np.abs(got[1] - Gu).max() <= 1e-12 * np.abs(Gu).max(), (s, g)
            assert np.abs(got[0] - Gc).max() <= 1e-12 * np.abs(Gc).max(), (s, g)


def test_gram_trajectory_matches_dense_losses():
    """Phases 1 -> 2 -> 3 with evaluation: every history row's train / valid / test losses in Gram
    mode (fp64 quadratic forms) within 1e-6 of the dense fp32 asset passes, and the final
    parameters within 1e-5 (the two loss reductions round differently; Adam amplifies it)."""
    from deeplearninginassetpricing_paperreplication_amd.engine.runner import HIST
    splits = _splits()
    cfg = default_cli_config(8, 46, dropout=0.0)
    torch.manual_seed(1)
    model = AssetPricingGAN(cfg)
    hs, ps = [], []
    for gram in (True, False):
        eng = _engine(copy.deepcopy(model), splits, gram)
        assert eng.eng.gram_enabled(1) == gram and eng.eng.gram_enabled(3) == gram
        for phase, n in ((1, 5), (2, 3), (3, 5)):
            eng.eng.begin_phase(phase)
            eng.run(phase, n, 1e-3, 0)
        eng.eng.sync()
        hs.append(eng.history_rows(0))
        ps.append(eng.params(0))
    a, b = hs
    for key in ("train_loss", "valid_loss", "test_loss", "valid_loss_unc", "valid_loss_cond", "test_loss_unc",
                "test_loss_cond", "train_loss_unc", "train_loss_cond"):
        x, y = a[:, HIST[key]], b[:, HIST[key]]
        rel = np.abs(x - y) / np.maximum(np.abs(y), 1e-30)
        assert np.nanmax(rel) < 1e-6, (key, np.nanmax(rel))
    assert np.linalg.norm(ps[0] - ps[1]) <= 1e-5 * np.linalg.norm(ps[1])


def test_gram_first_step_losses_match_fp64_reference():
    """Phase-1 and phase-3 training losses of the first step against the reference module run in
    float64 on the CPU (same weights, dropout 0): within 1e-6 relative -- the tower outputs are
    fp32, the quadratic forms fp64."""
    splits = _splits()
    cfg = default_cli_config(8, 46, dropout=0.0)
    torch.manual_seed(2)
    model = AssetPricingGAN(cfg)
    m64 = copy.deepcopy(model).double()
    b = {k: (v.double() if v.is_floating_point() else v) for k, v in splits[0].items()}
    from deeplearninginassetpricing_paperreplication_amd.engine.runner import HIST
    for phase, name in ((1, "loss_unconditional"), (3, "loss_conditional")):
        eng = _engine(copy.deepcopy(model), splits, True)
        eng.eng.begin_phase(phase)
        eng.run(phase, 1, 1e-3, 0)
        eng.eng.sync()
        got = eng.history_rows(0)[0, HIST["train_loss"]]
        with torch.no_grad():
            out = m64(b["macro_features"], b["individual_features"], b["returns"], b["mask"],
                      phase="unconditional" if phase == 1 else "conditional")
        ref = float(out[name])
        assert abs(got - ref) <= 1e-6 * abs(ref), (phase, got, ref)
