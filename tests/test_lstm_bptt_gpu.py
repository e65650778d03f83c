"""Dense-state LSTM BPTT (`k_lstm_bwd`, H = 4: the backward recurrence as one 8x8 mat-vec per
step with alternating reduction layouts, csrc/k_rnn.hip) against the gate-per-lane chain it
replaces (DLAP_LSTM_SCAN=0) and against fp32 autograd of the reference LSTM
(`/root/reference/src/model.py:21-84`, the macro `nn.LSTM`): same gradients to fp32 rounding, the
tower gradients untouched (bitwise), every time-length parity and block remainder, stacked
layers, and the initial-state gradient of the module API path."""
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


def _batch(T, N=160, F=46, M=8, seed=0):
    ret, feats, mask, mac = generate_panel_fast(T, N, F, M, seed=seed)
    mac = (mac - mac.mean(0)) / (mac.std(0, unbiased=False) + 1e-8)
    return {"returns": ret, "individual_features": feats, "mask": mask, "macro_features": mac}


def _lstm_count(spec):
    return sum(int(np.prod(s)) for k, s in spec.param_layout() if "macro_lstm" in k)


def _grads(cfg, b, phase, scan, monkeypatch, precision="fp32"):
    from deeplearninginassetpricing_paperreplication_amd.engine.runner import GANEngine
    monkeypatch.setenv("DLAP_LSTM_SCAN", scan)
    torch.manual_seed(0)
    model = AssetPricingGAN(cfg)
    eng = GANEngine(model.spec, 1, max_epochs=8, precision=precision)
    eng.set_data(b, b, b)
    eng.set_model(0, model, 7)
    eng.eng.backward_only(phase)
    return eng.eng.get_grads(0), model


@pytest.mark.parametrize("T", [36, 37, 240, 9])
@pytest.mark.parametrize("phase", [1, 3])
def test_dense_state_bptt_equals_gate_per_lane(T, phase, monkeypatch):
    cfg = default_cli_config(8, 46, dropout=0.0)
    b = _batch(T)
    g0, model = _grads(cfg, b, phase, "0", monkeypatch)
    g1, _ = _grads(cfg, b, phase, "1", monkeypatch)
    n = _lstm_count(model.spec)
    np.testing.assert_array_equal(g1[n:], g0[n:])          # the towers never see the LSTM backward
    err = np.linalg.norm(g1[:n] - g0[:n]) / np.linalg.norm(g0[:n])
    assert np.isfinite(g1).all() and err < 2e-6, err


def test_dense_state_bptt_stacked_layers(monkeypatch):
    cfg = default_cli_config(8, 46, rnn_dim=[4, 4], dropout=0.0)
    b = _batch(60)
    g0, model = _grads(cfg, b, 3, "0", monkeypatch)
    g1, _ = _grads(cfg, b, 3, "1", monkeypatch)
    n = _lstm_count(model.spec)
    err = np.linalg.norm(g1[:n] - g0[:n]) / np.linalg.norm(g0[:n])
    assert err < 2e-6, err


def test_dense_state_bptt_matches_autograd(monkeypatch):
    """fp32 engine LSTM gradients (phase 3) against torch autograd of the reference model. (At
    T = 36 the loss is well conditioned: the whole gradient agrees to ~3e-7. Longer random panels
    sit near a cancellation of the conditional loss where every parameter's gradient -- the
    towers' as much as the LSTM's, either BPTT -- moves by ~1e-3 relative between fp32 orders,
    tools/dbg/lstm_grad_check.py.)"""
    from deeplearninginassetpricing_paperreplication_amd.engine.runner import flatten_state
    cfg = default_cli_config(8, 46, dropout=0.0)
    b = _batch(36)
    got, model = _grads(cfg, b, 3, "1", monkeypatch)
    model.zero_grad()
    o = model(b["macro_features"], b["individual_features"], b["returns"], b["mask"], phase="conditional")
    o["loss"].backward()
    ref = flatten_state({k: (p.grad if p.grad is not None else torch.zeros_like(p))
                         for k, p in model.named_parameters()}, model.spec)
    n = _lstm_count(model.spec)
    err = np.linalg.norm(got[:n] - ref[:n]) / np.linalg.norm(ref[:n])
    assert err < 1e-5, err
