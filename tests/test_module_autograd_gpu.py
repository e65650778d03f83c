"""Module API on CUDA tensors: autograd through every output, caller-supplied LSTM state, the
'moment' phase with a residual term, and SimpleSDF without hidden layers (VERDICT r2 "what's
missing" 1, 2, 4, 5).

The reference returns ``weights``, ``moments`` and ``portfolio_returns`` inside the autograd
graph and threads ``hidden`` into its LSTM (`/root/reference/src/model.py:68,244,511,553-563,
579`). The GPU path runs the native engine at reference precision (``ops.fused.set_precision
('fp32')``) and every gradient is compared with the CPU modules (which reproduce the reference)
within 1e-5 relative.
"""
import copy

import numpy as np
import pytest
import torch

from deeplearninginassetpricing_paperreplication_amd.config import default_cli_config
from deeplearninginassetpricing_paperreplication_amd.data.synthetic import generate_panel_fast
from deeplearninginassetpricing_paperreplication_amd.models.gan import AssetPricingGAN, SimpleSDF

pytestmark = pytest.mark.gpu

TOL = 1e-5


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from deeplearninginassetpricing_paperreplication_amd.ops import fused, native
    native.load(required=True)
    fused.set_precision("fp32")
    yield
    fused.set_precision("bf16")


def _batch(T=30, N=120, F=46, M=8, seed=4):
    ret, feats, mask, mac = generate_panel_fast(T, N, F, M, seed=seed)
    mac = (mac - mac.mean(0)) / (mac.std(0, unbiased=False) + 1e-8)
    return {"returns": ret, "individual_features": feats, "mask": mask, "macro_features": mac}


def _cuda(b):
    return {k: v.cuda() for k, v in b.items()}


def _args(b):
    return b["macro_features"], b["individual_features"], b["returns"], b["mask"]


def _grads(model):
    return {k: (p.grad.detach().double().cpu() if p.grad is not None else torch.zeros(p.shape, dtype=torch.float64))
            for k, p in model.named_parameters()}


def _close(ga, gb, tol=TOL, skip=("sdf_net.output_proj.bias",)):
    """Per-parameter relative error (the SDF output bias cancels out of the normalised weights:
    its exact gradient is 0, both sides only see rounding noise)."""
    for k in ga:
        if k in skip:
            continue
        a, b = ga[k], gb[k]
        nb = float(b.norm())
        err = float((a - b).norm()) / max(nb, 1e-30)
        assert err < tol or float((a - b).abs().max()) < 1e-9, (k, err, nb)


def _close_out(g, c, tol=TOL):
    """An output tensor within tol in relative norm and 1e-6 elementwise (fp32 sums in another
    order: an entry near zero carries ~1e-7 absolute rounding noise, which a per-entry rtol
    cannot absorb)."""
    a, b = g.detach().double().cpu(), c.detach().double()
    err = float((a - b).norm()) / max(float(b.norm()), 1e-30)
    mx = float((a - b).abs().max())
    assert err < tol and mx < 1e-6, (err, mx)


def _pair(cfg_extra=None, seed=0):
    cfg = default_cli_config(8, 46, dropout=0.0)
    cfg.update(cfg_extra or {})
    torch.manual_seed(seed)
    cpu = AssetPricingGAN(cfg)
    gpu = copy.deepcopy(cpu).cuda()
    return cpu, gpu


@pytest.mark.parametrize("output", ["weights", "moments", "portfolio_returns"])
def test_custom_loss_of_outputs_backpropagates(output):
    """A loss built from out[output] only: the engine's tower backward (xs_backward) gives the
    parameter gradients of the CPU modules."""
    b = _batch()
    cpu, gpu = _pair()
    bc = _cuda(b)
    w = torch.randn(b["mask"].shape)

    def custom(out, wt):
        x = out[output]
        if output == "weights":
            return (x * wt).sum() + (x ** 2).sum()
        if output == "moments":
            return (x * wt[None]).sum() + 0.5 * (x ** 2).mean()
        return (x * wt[:, 0]).sum() + (x ** 2).sum()

    out_c = cpu(*_args(b), phase="conditional")
    custom(out_c, w).backward()
    out_g = gpu(*_args(bc), phase="conditional")
    custom(out_g, w.cuda()).backward()
    _close_out(out_g[output], out_c[output])
    _close(_grads(gpu), _grads(cpu))


def test_combined_loss_accumulates_paths():
    """loss + lambda * f(weights) + mu * g(moments): the fused-loss backward and both tower
    backwards accumulate into the same parameter gradients."""
    b = _batch()
    cpu, gpu = _pair(seed=1)
    bc = _cuda(b)
    for model, bb in ((cpu, b), (gpu, bc)):
        out = model(*_args(bb), phase="conditional")
        (out["loss"] + 0.1 * (out["weights"] ** 2).sum() + 0.01 * out["moments"].abs().sum()).backward()
    _close(_grads(gpu), _grads(cpu))


def test_hidden_state_forward_and_gradient():
    """A caller-supplied (h0, c0) changes the SDF (reference: nn.LSTM(x, hidden)); outputs,
    the parameter gradient and dL/d(h0, c0) match the CPU modules."""
    b = _batch()
    cpu, gpu = _pair(seed=2)
    bc = _cuda(b)
    torch.manual_seed(7)
    h0 = 0.5 * torch.randn(1, 1, 4)
    c0 = 0.5 * torch.randn(1, 1, 4)
    hc = (h0.clone().requires_grad_(True), c0.clone().requires_grad_(True))
    hg = (h0.cuda().requires_grad_(True), c0.cuda().requires_grad_(True))
    out_c = cpu(*_args(b), hidden=hc, phase="conditional")
    out_g = gpu(*_args(bc), hidden=hg, phase="conditional")
    assert torch.allclose(out_g["weights"].detach().cpu(), out_c["weights"].detach(), rtol=1e-5, atol=1e-7)
    for a, c in zip(out_g["hidden"], out_c["hidden"]):
        assert torch.allclose(a.detach().cpu(), c.detach(), rtol=1e-5, atol=1e-6)
    zero = cpu(*_args(b), phase="conditional")["weights"]
    assert float((zero - out_c["weights"]).abs().max()) > 1e-6          # the state matters
    (out_c["loss"] + (out_c["weights"] ** 2).sum()).backward()
    (out_g["loss"] + (out_g["weights"] ** 2).sum()).backward()
    _close(_grads(gpu), _grads(cpu))
    for a, c in zip(hg, hc):
        err = float((a.grad.cpu().double() - c.grad.double()).norm() / c.grad.double().norm())
        assert err < TOL, err


def test_moment_phase_with_residual_term():
    """phase='moment' with residual_loss_factor > 0: the SDF gradient of -L_cond + r L_res and
    the moment gradient (reference `src/model.py:524-548`)."""
    b = _batch()
    cpu, gpu = _pair({"residual_loss_factor": 0.5}, seed=3)
    bc = _cuda(b)
    out_c = cpu(*_args(b), phase="moment")
    out_g = gpu(*_args(bc), phase="moment")
    assert abs(float(out_g["loss"]) - float(out_c["loss"])) <= TOL * abs(float(out_c["loss"]))
    assert abs(float(out_g["loss_residual"]) - float(out_c["loss_residual"])) <= TOL * abs(float(out_c["loss_residual"]))
    out_c["loss"].backward()
    out_g["loss"].backward()
    _close(_grads(gpu), _grads(cpu))


def test_get_weights_differentiable():
    b = _batch()
    cpu, gpu = _pair(seed=5)
    bc = _cuda(b)
    wc, _ = cpu.get_weights(b["macro_features"], b["individual_features"], b["mask"], normalized=True)
    wg, _ = gpu.get_weights(bc["macro_features"], bc["individual_features"], bc["mask"], normalized=True)
    assert torch.allclose(wg.detach().cpu(), wc.detach(), rtol=1e-5, atol=1e-7)
    r = torch.randn(wc.shape, generator=torch.Generator().manual_seed(1))
    ((wc * r).sum() + (wc ** 2).sum()).backward()
    ((wg * r.cuda()).sum() + (wg ** 2).sum()).backward()
    _close(_grads(gpu), _grads(cpu))


def test_simple_sdf_without_hidden_layers():
    """SimpleSDF(hidden_dims=[]) (reference `src/model.py:639-646`): a single Linear; on CUDA it
    is one library GEMV plus the loss math (no tower to fuse)."""
    b = _batch()
    torch.manual_seed(6)
    cpu = SimpleSDF(8, 46, hidden_dims=[], dropout=0.0)
    gpu = copy.deepcopy(cpu).cuda()
    out_c = cpu(*_args(b))
    out_g = gpu(*_args(_cuda(b)))
    assert abs(float(out_g["loss"]) - float(out_c["loss"])) <= TOL * abs(float(out_c["loss"]))
    out_c["loss"].backward()
    out_g["loss"].backward()
    # (the Linear's bias cancels out of the zero-mean weights: its gradient is rounding noise)
    gc, gg = cpu.net[-1].weight.grad, gpu.net[-1].weight.grad.cpu()
    assert float((gg - gc).norm() / gc.norm()) < TOL


def test_param_cache_sees_data_edits_after_invalidation():
    """the engine skips re-uploading unchanged parameters (storage + autograd version);
    an in-place edit through ``p.data`` keeps the version, so ``invalidate_param_cache`` is the
    documented way to make the next call see it. Either way the outputs match the CPU modules
    after the same edit."""
    from deeplearninginassetpricing_paperreplication_amd.ops import fused
    b = _batch()
    cpu, gpu = _pair()
    bc = _cuda(b)
    with torch.no_grad():
        gpu(*_args(bc), phase="conditional")            # parameters uploaded and cached
    for m in (cpu, gpu):
        for p in m.sdf_net.parameters():
            p.data.mul_(0.5)
    fused.invalidate_param_cache()
    with torch.no_grad():
        out_g = gpu(*_args(bc), phase="conditional")
        out_c = cpu(*_args(b), phase="conditional")
    _close_out(out_g["weights"], out_c["weights"])


def test_new_panel_at_a_reused_address_is_uploaded():
    """a loop that moves a new host batch of the same shape to the GPU every step gets
    the freed block back at the same address with version 0. The panel cache key holds weak
    references to the tensor objects (``ops.fused._PanelKey``), so the second batch is uploaded
    and the outputs follow it (checked against the CPU module on each batch)."""
    cpu, gpu = _pair()
    outs = []
    for seed in (4, 5):
        b = _batch(seed=seed)
        bc = _cuda(b)
        with torch.no_grad():
            out_g = gpu(*_args(bc), phase="conditional")
            out_c = cpu(*_args(b), phase="conditional")
        _close_out(out_g["weights"], out_c["weights"])
        outs.append((bc["individual_features"].data_ptr(), out_g["weights"].detach().cpu()))
        del bc, out_g
        torch.cuda.synchronize()
    assert not torch.equal(outs[0][1], outs[1][1])
