"""The one-pass SDF tower backward (``csrc/k_tbwd.hip``) on a real MI355X.

It replaces the sliced k_mlp_bwd_sdf for the bf16 fused-layer-0 shapes (1..3 hidden layers, a
64-column panel row). Both kernels multiply the same bf16 operands -- the activations, dz and
panel rows go through an LDS transpose (``ds_read_b64_tr_b16``) instead of selector MFMAs, both
exact -- and differ only in the fp32 summation order of the weight gradients, so the gradients
must agree to fp32 rounding (reference op: the autograd of `SDFNetwork.forward`,
`/root/reference/src/model.py:208-219,253-279`). Against the fp32 PyTorch model the bf16 tolerance
of ``test_engine_gpu.test_gradients_match_autograd`` applies."""
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


def _batch(T=48, N=700, F=46, M=8, seed=0):
    ret, feats, mask, mac = generate_panel_fast(T, N, F, M, seed=seed)
    mac = (mac - mac.mean(0)) / (mac.std(0, unbiased=False) + 1e-8)
    return {"returns": ret, "individual_features": feats, "mask": mask, "macro_features": mac}


def _grads(cfg, b, tbwd, phase, G=1, monkeypatch=None):
    from deeplearninginassetpricing_paperreplication_amd.engine.runner import GANEngine
    monkeypatch.setenv("DLAP_TBWD", "1" if tbwd else "0")
    eng = GANEngine(AssetPricingGAN(cfg).spec, G, max_epochs=8)
    assert int(eng.desc["tbwd"]) == int(tbwd)
    eng.set_data(b, b, b)
    for g in range(G):
        torch.manual_seed(100 + g)
        eng.set_model(g, AssetPricingGAN(cfg), 11 + g)
    eng.eng.backward_only(phase)
    return [eng.eng.get_grads(g) for g in range(G)], AssetPricingGAN(cfg).spec.param_counts()[0]


def _rel(a, b):
    return float(np.linalg.norm(a - b) / (np.linalg.norm(b) + 1e-30))


CASES = [
    ([64, 64], [4], 0.0),        # the paper / bench architecture
    ([64, 64], [4], 0.05),       # with dropout (pre-generated keep words)
    ([64], [8], 0.05),           # SMV = 8 of the paper grid, one hidden layer
    ([64, 64, 64], [4], 0.05),   # HL = 3
    ([48, 32], [2, 2], 0.0),     # narrow layers (zero-padded units), two-layer LSTM of width 2
    ([64] * 4, [4], 0.05),       # HL = 4 (the paper grid's deepest SDF)
]


@pytest.mark.parametrize("hidden,rnn,dropout", CASES)
@pytest.mark.parametrize("phase", [1, 3])
def test_one_pass_backward_equals_sliced_kernel(monkeypatch, hidden, rnn, dropout, phase):
    cfg = default_cli_config(8, 46, hidden_dim=hidden, rnn_dim=rnn, dropout=dropout)
    b = _batch()
    (ref,), P_sdf = _grads(cfg, b, False, phase, monkeypatch=monkeypatch)
    (got,), _ = _grads(cfg, b, True, phase, monkeypatch=monkeypatch)
    sl = slice(0, P_sdf)
    assert np.isfinite(got[sl]).all()
    assert np.abs(ref[sl]).max() > 0
    # same bf16 operands, different fp32 summation order: rounding-level agreement, every parameter
    assert _rel(got[sl], ref[sl]) < 1e-4, _rel(got[sl], ref[sl])
    np.testing.assert_allclose(got[sl], ref[sl], rtol=2e-3, atol=1e-6 * np.abs(ref[sl]).max())


def test_one_pass_backward_batched_members_equal_solo(monkeypatch):
    """Model batching: member g of a 3-model launch has the bits of the same model alone (the
    fine-slab partition and the fixed wave tree depend on R only)."""
    cfg = default_cli_config(8, 46, dropout=0.05)
    b = _batch(seed=4)
    batched, _ = _grads(cfg, b, True, 3, G=3, monkeypatch=monkeypatch)
    from deeplearninginassetpricing_paperreplication_amd.engine.runner import GANEngine
    for g in range(3):
        eng = GANEngine(AssetPricingGAN(cfg).spec, 1, max_epochs=8)
        eng.set_data(b, b, b)
        torch.manual_seed(100 + g)
        eng.set_model(0, AssetPricingGAN(cfg), 11 + g)
        eng.eng.backward_only(3)
        np.testing.assert_array_equal(eng.eng.get_grads(0), batched[g])


def test_one_pass_backward_matches_fp32_autograd(monkeypatch):
    from deeplearninginassetpricing_paperreplication_amd.engine.runner import flatten_state
    cfg = default_cli_config(8, 46, dropout=0.0)
    b = _batch(seed=2)
    torch.manual_seed(100)
    model = AssetPricingGAN(cfg)
    (got,), P_sdf = _grads(cfg, b, True, 3, monkeypatch=monkeypatch)
    model.zero_grad()
    o = model(b["macro_features"], b["individual_features"], b["returns"], b["mask"], phase="conditional")
    o["loss"].backward()
    ref = flatten_state({k: (p.grad if p.grad is not None else torch.zeros_like(p))
                         for k, p in model.named_parameters()}, model.spec)
    sl = slice(0, P_sdf)
    err = np.linalg.norm(got[sl] - ref[sl]) / np.linalg.norm(ref[sl])
    cos = np.dot(got[sl], ref[sl]) / (np.linalg.norm(got[sl]) * np.linalg.norm(ref[sl]))
    # (bf16 GEMM operands: ~5% whole-scope L2 error on this panel, the sliced kernel's too -- the two
    # agree to 1e-4 above)
    assert err < 0.08 and cos > 0.998, (err, cos)


WIDE_CASES = [
    ([64, 64], [4], 0.05, 46),   # the scaled panel's architecture (wide path forced)
    ([64], [4], 0.0, 46),
    ([64, 64, 64], [4], 0.05, 46),
    ([48, 32], [2, 2], 0.0, 46),
    ([64] * 4, [4], 0.05, 46),
    ([64, 64], [4], 0.05, 200),  # F + LSTM columns > 128: wide by size
]


@pytest.mark.parametrize("hidden,rnn,dropout,F", WIDE_CASES)
@pytest.mark.parametrize("phase", [1, 3])
def test_one_pass_backward_wide_path_equals_sliced_kernel(monkeypatch, hidden, rnn, dropout, F, phase):
    """Wide layer-0 path (ZIN): the one-pass backward starts from the stored layer-0 pre-activations
    (k_mlp_fwd_zx), its layer-0 gradient tile is the per-period input columns only, and the layer-0
    dz it stores (in the sliced kernel's row order) feeds k_wgrad0 -- so the whole SDF gradient,
    the streamed panel columns of W0 included, must agree with the sliced kernel to fp32 rounding."""
    monkeypatch.setenv("DLAP_WIDE", "1")
    cfg = default_cli_config(8, F, hidden_dim=hidden, rnn_dim=rnn, dropout=dropout)
    b = _batch(F=F, seed=5)
    (ref,), P_sdf = _grads(cfg, b, False, phase, monkeypatch=monkeypatch)
    (got,), _ = _grads(cfg, b, True, phase, monkeypatch=monkeypatch)
    assert np.isfinite(got[:P_sdf]).all()
    assert np.abs(ref[:P_sdf]).max() > 0
    # every SDF parameter, and layer 0's weight (k_wgrad0 from the stored dz) on its own
    lay = dict(AssetPricingGAN(cfg).spec.param_layout())
    o0 = sum(int(np.prod(shp)) for k, shp in AssetPricingGAN(cfg).spec.param_layout()
             if k.startswith("sdf_net.macro_lstm"))
    w0 = slice(o0, o0 + int(np.prod(lay["sdf_net.fc_layers.0.weight"])))
    for sl in (slice(0, P_sdf), w0):
        assert _rel(got[sl], ref[sl]) < 1e-4, _rel(got[sl], ref[sl])
        np.testing.assert_allclose(got[sl], ref[sl], rtol=2e-3, atol=1e-6 * np.abs(ref[sl]).max())
