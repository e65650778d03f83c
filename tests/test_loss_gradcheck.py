"""fp64 gradient checks of the vectorised loss formulas (SURVEY §7.4 "gradient checks"): the
analytic gradients the native engine implements (k_loss.hip) are validated against these
through the fp32 PyTorch model, so the autograd of the reference formulas must itself be exact."""
import torch

from deeplearninginassetpricing_paperreplication_amd.models import losses as L


def _panel(T=7, N=9, K=3, seed=0):
    g = torch.Generator().manual_seed(seed)
    mask = torch.rand(T, N, generator=g) > 0.35
    mask[2] = False                      # an all-masked period
    mask[:, 4] = False
    mask[5, 4] = True                    # an asset with a single observation
    r = torch.randn(T, N, generator=g, dtype=torch.float64) * 0.1 * mask
    w = torch.randn(T, N, generator=g, dtype=torch.float64, requires_grad=True)
    h = torch.tanh(torch.randn(K, T, N, generator=g, dtype=torch.float64)).requires_grad_(True)
    return w, r, mask, h


def test_unconditional_loss_gradcheck():
    w, r, m, _ = _panel()
    for weighted in (True, False):
        assert torch.autograd.gradcheck(lambda x: L.unconditional_loss(L.zero_mean_normalize(x, m), r, m,
                                                                       weighted)[0], (w,))


def test_conditional_loss_gradcheck():
    w, r, m, h = _panel()
    f = lambda x, hh: L.conditional_loss(L.zero_mean_normalize(x, m), r, m, hh, True)[0]  # noqa: E731
    assert torch.autograd.gradcheck(f, (w, h))


def test_residual_loss_gradcheck():
    w, r, m, _ = _panel(seed=3)
    assert torch.autograd.gradcheck(lambda x: L.residual_loss(x * m, r, m), (w,))


def test_l1_normalize_and_sharpe_gradcheck():
    w, r, m, _ = _panel(seed=5)
    assert torch.autograd.gradcheck(lambda x: L.sharpe_monitor(
        L.portfolio_returns(L.l1_normalize(x * m, m), r, m, False)), (w,))
