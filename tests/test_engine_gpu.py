"""Native engine on a real MI355X: numerics vs the fp32 PyTorch model, determinism, model
batching and the pipelined epoch graph. All tests need the GPU and the in-tree extension
(they fail loudly if it is missing: no eager fallback)."""
import numpy as np
import pytest
import torch

from deeplearninginassetpricing_paperreplication_amd.config import default_cli_config
from deeplearninginassetpricing_paperreplication_amd.data.synthetic import generate_panel_fast
from deeplearninginassetpricing_paperreplication_amd.models.gan import AssetPricingGAN

pytestmark = pytest.mark.gpu


def _batch(T=36, N=160, F=46, M=8, seed=0):
    ret, feats, mask, mac = generate_panel_fast(T, N, F, M, seed=seed)
    mac = (mac - mac.mean(0)) / (mac.std(0, unbiased=False) + 1e-8)
    return {"returns": ret, "individual_features": feats, "mask": mask, "macro_features": mac}


def _engine(cfg, n_models=1, seeds=(7,), data=None, max_epochs=64):
    from deeplearninginassetpricing_paperreplication_amd.engine.runner import GANEngine
    b = data or _batch(M=cfg["macro_feature_dim"], F=cfg["individual_feature_dim"])
    torch.manual_seed(0)
    model = AssetPricingGAN(cfg)
    eng = GANEngine(model.spec, n_models, max_epochs=max_epochs)
    eng.set_data(b, b, b)
    for g in range(n_models):
        torch.manual_seed(g)
        eng.set_model(g, AssetPricingGAN(cfg), seeds[g % len(seeds)])
    return eng, b


def _rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / (np.abs(b).max() + 1e-30))


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from deeplearninginassetpricing_paperreplication_amd.ops import native
    native.load(required=True)


def test_extension_is_native():
    from deeplearninginassetpricing_paperreplication_amd.ops import native
    mod = native.load(required=True)
    assert mod.__file__.endswith(".so")


@pytest.mark.parametrize("rnn,hidden,K", [([4], [64, 64], 8), ([2, 2], [32], 4), ([8], [64, 48, 32], 12)])
def test_forward_matches_fp32_reference(rnn, hidden, K):
    cfg = default_cli_config(8, 46, hidden_dim=hidden, rnn_dim=rnn, num_moments=K, dropout=0.0)
    eng, b = _engine(cfg)
    torch.manual_seed(0)
    model = AssetPricingGAN(cfg)
    eng.set_model(0, model, 7)
    with torch.no_grad():
        out = model(b["macro_features"], b["individual_features"], b["returns"], b["mask"], phase="conditional")
        lh, _ = model.sdf_net.macro_lstm(b["macro_features"])
    eng.eng.forward_split(0, False, True)
    T, N = b["mask"].shape
    m = b["mask"].numpy()
    assert _rel(eng.eng.read_ws(0, 0, "pp").reshape(T, -1), lh.numpy()) < 1e-4
    assert _rel(eng.eng.read_ws(0, 0, "wn").reshape(T, N), out["weights"].numpy()) < 3e-2
    h = eng.eng.read_ws(0, 0, "h").reshape(T, N, K)
    assert _rel(h[m], out["moments"].permute(1, 2, 0).numpy()[m]) < 3e-2
    sc = eng.eng.read_ws(0, 0, "scal")
    assert _rel(sc[0], out["loss_conditional"].item()) < 3e-2
    assert _rel(sc[1], out["loss_unconditional"].item()) < 3e-2


@pytest.mark.parametrize("phase,pname", [(1, "unconditional"), (3, "conditional"), (2, "moment")])
def test_gradients_match_autograd(phase, pname):
    from deeplearninginassetpricing_paperreplication_amd.engine.runner import flatten_state
    cfg = default_cli_config(8, 46, dropout=0.0)
    eng, b = _engine(cfg)
    torch.manual_seed(0)
    model = AssetPricingGAN(cfg)
    eng.set_model(0, model, 7)
    model.zero_grad()
    o = model(b["macro_features"], b["individual_features"], b["returns"], b["mask"], phase=pname)
    o["loss"].backward()
    ref = flatten_state({k: (p.grad if p.grad is not None else torch.zeros_like(p))
                         for k, p in model.named_parameters()}, model.spec)
    eng.eng.backward_only(phase)
    got = eng.eng.get_grads(0)
    P_sdf = model.spec.param_counts()[0]
    sl = slice(0, P_sdf) if phase != 2 else slice(P_sdf, None)
    # bf16 tower GEMMs: whole-scope relative L2 error and direction
    err = np.linalg.norm(got[sl] - ref[sl]) / np.linalg.norm(ref[sl])
    cos = np.dot(got[sl], ref[sl]) / (np.linalg.norm(got[sl]) * np.linalg.norm(ref[sl]))
    assert err < 0.05 and cos > 0.998, (err, cos)


def test_training_is_deterministic_and_finite():
    cfg = default_cli_config(8, 46)
    runs = []
    for _ in range(2):
        eng, _ = _engine(cfg)
        for ph, n in ((1, 4), (2, 2), (3, 4)):
            eng.eng.begin_phase(ph)
            eng.run(ph, n, 1e-3, 1, 1.0, True)
        eng.eng.sync()
        runs.append((eng.history_rows(0), eng.params(0)))
    (h0, p0), (h1, p1) = runs
    assert np.isfinite(h0[:, 1]).all()
    np.testing.assert_array_equal(p0, p1)
    np.testing.assert_array_equal(np.nan_to_num(h0), np.nan_to_num(h1))


def test_pipelined_epochs_equal_sequential():
    cfg = default_cli_config(8, 46)
    res = []
    for pipe in (False, True):
        eng, _ = _engine(cfg)
        eng.eng.set_pipeline(pipe)
        for ph, n in ((1, 5), (2, 2), (3, 6)):
            eng.eng.begin_phase(ph)
            eng.run(ph, n, 1e-3, 2, 1.0, True)
        eng.eng.sync()
        res.append((eng.history_rows(0), eng.params(0), eng.params(0, "loss"), eng.params(0, "sharpe")))
    for a, b in zip(res[0], res[1]):
        np.testing.assert_array_equal(np.nan_to_num(a), np.nan_to_num(b))


def test_graph_replay_equals_eager_launches():
    cfg = default_cli_config(8, 46)
    res = []
    for use_graph in (False, True):
        eng, _ = _engine(cfg)
        for ph, n in ((1, 3), (3, 3)):
            eng.eng.begin_phase(ph)
            eng.run(ph, n, 1e-3, 1, 1.0, use_graph)
        eng.eng.sync()
        res.append(eng.params(0))
    np.testing.assert_array_equal(res[0], res[1])


def test_model_batching_matches_single_models():
    cfg = default_cli_config(8, 46)
    data = _batch()
    eng2, _ = _engine(cfg, n_models=2, seeds=(11, 12), data=data)
    for ph, n in ((1, 3), (3, 3)):
        eng2.eng.begin_phase(ph)
        eng2.run(ph, n, 1e-3, 1, 1.0, True)
    eng2.eng.sync()
    for g, seed in ((0, 11), (1, 12)):
        from deeplearninginassetpricing_paperreplication_amd.engine.runner import GANEngine
        torch.manual_seed(0)
        model = AssetPricingGAN(cfg)
        e1 = GANEngine(model.spec, 1, max_epochs=64)
        e1.set_data(data, data, data)
        torch.manual_seed(g)
        e1.set_model(0, AssetPricingGAN(cfg), seed)
        for ph, n in ((1, 3), (3, 3)):
            e1.eng.begin_phase(ph)
            e1.run(ph, n, 1e-3, 1, 1.0, True)
        e1.eng.sync()
        np.testing.assert_array_equal(e1.params(0), eng2.params(g))


def test_dropout_changes_with_step_and_seed():
    cfg = default_cli_config(8, 46, dropout=0.3)
    eng, _ = _engine(cfg, n_models=2, seeds=(1, 2))
    eng.eng.backward_only(3)
    g0, g1 = eng.eng.get_grads(0), eng.eng.get_grads(1)
    assert not np.array_equal(g0, g1)           # same weights, different dropout streams
    assert np.isfinite(g0).all() and np.isfinite(g1).all()


def test_module_forward_and_backward_run_the_engine():
    """nn.Module API on CUDA tensors: forward through the native engine, loss.backward() through
    the engine's analytic gradients; compared with the fp32 CPU module."""
    cfg = default_cli_config(8, 46, dropout=0.0)
    b = _batch()
    torch.manual_seed(0)
    cpu = AssetPricingGAN(cfg)
    gpu = AssetPricingGAN(cfg)
    gpu.load_state_dict(cpu.state_dict())
    gpu.cuda()
    dev = {k: (v.cuda() if v is not None else None) for k, v in b.items()}
    for phase in ("unconditional", "conditional", "moment"):
        cpu.zero_grad(); gpu.zero_grad()
        oc = cpu(b["macro_features"], b["individual_features"], b["returns"], b["mask"], phase=phase)
        og = gpu(dev["macro_features"], dev["individual_features"], dev["returns"], dev["mask"], phase=phase)
        assert og["weights"].is_cuda and og["moments"].shape == oc["moments"].shape
        assert _rel(og["loss"].item(), oc["loss"].item()) < 3e-2
        oc["loss"].backward()
        og["loss"].backward()
        gc = torch.cat([p.grad.reshape(-1) if p.grad is not None else torch.zeros(p.numel())
                        for p in cpu.parameters()])
        gg = torch.cat([p.grad.reshape(-1).cpu() if p.grad is not None else torch.zeros(p.numel())
                        for p in gpu.parameters()])
        cos = float(torch.dot(gc, gg) / (gc.norm() * gg.norm() + 1e-30))
        assert cos > 0.995, (phase, cos)


def test_module_train_epoch_one_host_sync_and_engine_hidden():
    """``train_epoch(model, opt, data, 'cuda')``: after the first call (panel upload) a step issues
    no host-blocking engine call and exactly one torch synchronisation (the metrics read-back);
    the module's ``hidden`` is the engine LSTM's final (h_n, c_n), equal to nn.LSTM's."""
    import warnings
    from deeplearninginassetpricing_paperreplication_amd.ops import native
    from deeplearninginassetpricing_paperreplication_amd.train.trainer import train_epoch
    cfg = default_cli_config(8, 46, dropout=0.0, rnn_dim=[3, 4])
    b = _batch()
    torch.manual_seed(0)
    cpu = AssetPricingGAN(cfg)
    gpu = AssetPricingGAN(cfg)
    gpu.load_state_dict(cpu.state_dict())
    gpu.cuda()
    dev = {k: v.cuda() for k, v in b.items()}
    opt_c = torch.optim.Adam(cpu.sdf_net.parameters(), lr=1e-3)
    opt_g = torch.optim.Adam(gpu.sdf_net.parameters(), lr=1e-3)
    rc = [train_epoch(cpu, opt_c, b, "cpu", "conditional", scope="sdf")]
    rg = [train_epoch(gpu, opt_g, dev, "cuda", "conditional", scope="sdf")]
    n0 = native.load().Engine.blocking_calls()
    torch.cuda.set_sync_debug_mode("warn")
    try:
        with warnings.catch_warnings(record=True) as w:
            warnings.simplefilter("always")
            rg.append(train_epoch(gpu, opt_g, dev, "cuda", "conditional", scope="sdf"))
    finally:
        torch.cuda.set_sync_debug_mode("default")
    syncs = [x for x in w if "synchroniz" in str(x.message).lower()]
    assert len(syncs) == 1, [str(x.message) for x in syncs]
    assert native.load().Engine.blocking_calls() == n0
    rc.append(train_epoch(cpu, opt_c, b, "cpu", "conditional", scope="sdf"))
    for a, c in zip(rg, rc):
        assert _rel(a["loss"], c["loss"]) < 3e-2 and _rel(a["grad_norm"], c["grad_norm"]) < 5e-2
    with torch.no_grad():
        o = gpu(dev["macro_features"], dev["individual_features"], dev["returns"], dev["mask"])
        _, (h_ref, c_ref) = gpu.sdf_net.macro_lstm.cpu()(b["macro_features"])
        gpu.sdf_net.macro_lstm.cuda()
    h_n, c_n = o["hidden"]
    assert h_n.is_cuda and h_n.shape == h_ref.shape == (2, 1, 4)
    assert _rel(h_n.cpu().numpy(), h_ref.numpy()) < 1e-4 and _rel(c_n.cpu().numpy(), c_ref.numpy()) < 1e-4


def test_simple_sdf_runs_the_engine():
    """SimpleSDF (`/root/reference/src/model.py:620-694`) on CUDA tensors: the engine's SDF tower
    with the [macro ; x] column order, unweighted unconditional loss; forward and gradients vs the
    CPU module."""
    from deeplearninginassetpricing_paperreplication_amd.models.gan import SimpleSDF
    from deeplearninginassetpricing_paperreplication_amd.ops import native
    b = _batch()
    torch.manual_seed(0)
    cpu = SimpleSDF(8, 46, [64, 64], dropout=0.0)
    gpu = SimpleSDF(8, 46, [64, 64], dropout=0.0)
    gpu.load_state_dict(cpu.state_dict())
    gpu.cuda()
    dev = {k: v.cuda() for k, v in b.items()}
    oc = cpu(b["macro_features"], b["individual_features"], b["returns"], b["mask"])
    og = gpu(dev["macro_features"], dev["individual_features"], dev["returns"], dev["mask"])
    assert og["weights"].is_cuda
    assert _rel(og["weights"].detach().cpu().numpy(), oc["weights"].detach().numpy()) < 3e-2
    assert _rel(og["loss"].item(), oc["loss"].item()) < 3e-2
    assert _rel(og["sharpe"].item(), oc["sharpe"].item()) < 5e-2
    oc["loss"].backward()
    og["loss"].backward()
    for pc, pg in zip(cpu.parameters(), gpu.parameters()):
        a, c = pg.grad.cpu().reshape(-1), pc.grad.reshape(-1)
        if c.norm() > 0:
            cos = float(torch.dot(a, c) / (a.norm() * c.norm() + 1e-30))
            assert cos > 0.99, cos
    assert native.load() is not None


def test_per_model_learning_rates_batch_exactly():
    cfg = default_cli_config(8, 46)
    data = _batch()
    from deeplearninginassetpricing_paperreplication_amd.engine.runner import GANEngine
    lrs = (1e-3, 2e-4)
    eng2, _ = _engine(cfg, n_models=2, seeds=(5, 5), data=data)
    for g, lr in enumerate(lrs):
        eng2.eng.set_lr(g, lr)
    for ph, n in ((1, 3), (3, 3)):
        eng2.eng.begin_phase(ph)
        eng2.run(ph, n, 1e-3, 1, 1.0, True)
    for g, lr in enumerate(lrs):
        torch.manual_seed(0)
        model = AssetPricingGAN(cfg)
        e1 = GANEngine(model.spec, 1, max_epochs=64)
        e1.set_data(data, data, data)
        torch.manual_seed(g)
        e1.set_model(0, AssetPricingGAN(cfg), 5)
        for ph, n in ((1, 3), (3, 3)):
            e1.eng.begin_phase(ph)
            e1.run(ph, n, lr, 1, 1.0, True)
        np.testing.assert_array_equal(e1.params(0), eng2.params(g))


def test_batched_ensemble_weights_match_cpu():
    from deeplearninginassetpricing_paperreplication_amd.analysis.ensemble import (
        get_weights_from_model, weights_batched_gpu)
    cfg = default_cli_config(8, 46, dropout=0.0)
    b = _batch()
    models = []
    for s in (1, 2, 3):
        torch.manual_seed(s)
        models.append(AssetPricingGAN(cfg).eval())
    got = weights_batched_gpu(models, {"train": b, "valid": b, "test": b})
    assert got["test"].is_cuda and tuple(got["test"].shape) == (3,) + tuple(b["mask"].shape)
    for i, m in enumerate(models):
        ref = get_weights_from_model(m, b, "cpu")
        assert _rel(got["test"][i].cpu().numpy(), ref) < 3e-2


def test_evaluate_ensemble_cuda_matches_cpu(tmp_path):
    """``evaluate_ensemble --device cuda`` (batched engine forward + K11 on the device) against
    the CPU path (the reference's per-model forward + numpy averaging), from saved checkpoints."""
    import json
    from deeplearninginassetpricing_paperreplication_amd.analysis.ensemble import evaluate_ensemble
    from deeplearninginassetpricing_paperreplication_amd.data.synthetic import generate_all_splits
    data = tmp_path / "data"
    generate_all_splits(str(data), 30, 10, 20, n_stocks=200, seed=3, quiet=True)
    cfg = default_cli_config(8, 46, dropout=0.0)
    dirs = []
    for s in (1, 2, 3):
        torch.manual_seed(s)
        d = tmp_path / f"m{s}"
        d.mkdir()
        (d / "config.json").write_text(json.dumps(cfg))
        torch.save(AssetPricingGAN(cfg).state_dict(), d / "best_model_sharpe.pt")
        dirs.append(str(d))
    cpu = evaluate_ensemble(dirs, str(data), "cpu", verbose=False)
    gpu = evaluate_ensemble(dirs, str(data), "cuda", verbose=False)
    for k in ("train_sharpe", "valid_sharpe", "test_sharpe"):
        assert abs(gpu[k] - cpu[k]) < 3e-2 * max(1.0, abs(cpu[k])), (k, gpu[k], cpu[k])
    np.testing.assert_allclose(gpu["individual_sharpes"], cpu["individual_sharpes"], rtol=3e-2, atol=3e-2)


def test_device_ensemble_portfolios_match_numpy():
    """K11 on the device (k_ensemble: average, L1 re-normalisation, portfolio returns) against the
    numpy post-processing of `/root/reference/src/evaluate_ensemble.py:137-171`."""
    from deeplearninginassetpricing_paperreplication_amd.analysis.portfolio import (
        ensemble_sharpes, ensemble_sharpes_device)
    rng = np.random.default_rng(0)
    G, T, N = 5, 30, 257
    batches, ws, wd = {}, [dict() for _ in range(G)], {}
    for sp in ("train", "valid", "test"):
        m = rng.random((T, N)) < 0.6
        m[3] = False                                       # an all-masked period
        R = (rng.standard_normal((T, N)) * 0.05 * m).astype(np.float32)
        W = rng.standard_normal((G, T, N)).astype(np.float32) * m
        W /= np.maximum(np.abs(W).sum(2, keepdims=True), 1e-8)
        batches[sp] = {"returns": R, "mask": m}
        for g in range(G):
            ws[g][sp] = W[g]
        wd[sp] = torch.from_numpy(W).cuda()
    ref = ensemble_sharpes(ws, batches)
    got = ensemble_sharpes_device(wd, batches)
    for k in ("train_sharpe", "valid_sharpe", "test_sharpe"):
        assert abs(got[k] - ref[k]) < 1e-5 * max(1.0, abs(ref[k])), (k, got[k], ref[k])
    np.testing.assert_allclose(got["individual_sharpes"], ref["individual_sharpes"], rtol=1e-5, atol=1e-6)


def _rccl_worker(rank, world, port, out):
    import os
    os.environ.update(WORLD_SIZE=str(world), RANK=str(rank), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    from deeplearninginassetpricing_paperreplication_amd.parallel import comm
    d = comm.init(backend="nccl", use_gpu=True, timeout_s=120)
    mine = comm.shard(9, d.rank, d.world)
    loc = torch.stack([torch.full((4, 5), float(i), device=d.device) for i in mine])
    g = comm.all_gather_rows_tensor(d, loc, 9, mine)
    assert g.is_cuda and torch.equal(g[:, 0, 0].cpu(), torch.arange(9, dtype=torch.float32))
    h = comm.all_gather_rows(d, loc.cpu().numpy(), 9, mine)
    assert (h[:, 0, 0] == np.arange(9)).all()
    comm.shutdown(d)
    out.put(rank)


@pytest.mark.skipif(not torch.cuda.is_available() or torch.cuda.device_count() < 2,
                    reason="needs 2 GPUs (one RCCL rank per GPU)")
def test_rccl_two_rank_ensemble_all_gather():
    """The ensemble's weight all-gather over RCCL with one rank per GPU (9 seeds over 2 ranks)."""
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_rccl_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(timeout=120)
    assert all(p.exitcode == 0 for p in ps)
    assert sorted(q.get(timeout=5) for _ in range(2)) == [0, 1]


def test_cli_and_ensemble_driver_on_gpu(tmp_path):
    from deeplearninginassetpricing_paperreplication_amd.data.synthetic import generate_all_splits
    from deeplearninginassetpricing_paperreplication_amd.parallel.ensemble import run_ensemble
    from deeplearninginassetpricing_paperreplication_amd.parallel import comm
    from deeplearninginassetpricing_paperreplication_amd.train import cli
    data = tmp_path / "data"
    generate_all_splits(str(data), 24, 8, 12, n_stocks=80, n_features=46, n_macro=8, seed=1, quiet=True)
    cli.main(["--data_dir", str(data), "--epochs_unc", "4", "--epochs_moment", "2", "--epochs", "4",
              "--ignore_epoch", "0", "--print_freq", "2", "--device", "cuda", "--save_dir", str(tmp_path / "ck")])
    for f in ("config.json", "best_model_loss.pt", "best_model_sharpe.pt", "final_model.pt", "history.npz"):
        assert (tmp_path / "ck" / f).exists(), f
    from deeplearninginassetpricing_paperreplication_amd.data.dataset import load_splits
    batches = {k: d.get_full_batch() for k, d in zip(("train", "valid", "test"), load_splits(str(data)))}
    d = comm.Dist(device=torch.device("cuda", 0))
    res = run_ensemble(default_cli_config(8, 46), batches, seeds=(1, 2, 3), dist=d, epochs=(3, 1, 3),
                       ignore_epoch=0, save_root=str(tmp_path / "ens"))
    assert res["failed"] == [] and np.isfinite(res["test_sharpe"])
    assert (tmp_path / "ens" / "seed_2" / "best_model_sharpe.pt").exists()


@pytest.mark.parametrize("stop", [(1, 3), (2, 1), (3, 4)])
def test_gpu_resume_equals_uninterrupted(tmp_path, stop):
    """An interrupted GPU run continued from resume.pt reproduces the uninterrupted run
    bitwise (parameters, Adam state, dropout stream, trackers, history, checkpoint files)."""
    from deeplearninginassetpricing_paperreplication_amd.engine.runner import train_3phase_gpu
    b = _batch(T=30, N=120)
    cfg = default_cli_config(8, 46)
    kw = dict(num_epochs_unc=5, num_epochs_moment=3, num_epochs=6, print_freq=2, ignore_epoch=0,
              seed=11, verbose=False)
    out = {}
    for name, extra in (("a", {}), ("b", {"stop_after": stop})):
        d = tmp_path / name
        d.mkdir()
        torch.manual_seed(0)
        out[name] = train_3phase_gpu(cfg, b, b, b, save_dir=str(d), **kw, **extra)
    assert out["b"] is None and (tmp_path / "b" / "resume.pt").exists()
    torch.manual_seed(0)
    mb, hb = train_3phase_gpu(cfg, b, b, b, save_dir=str(tmp_path / "b"), resume=True, **kw)
    ma, ha = out["a"]
    for k in ha:
        assert np.array_equal(np.nan_to_num(np.array(ha[k], dtype=object if k == "phase" else float)),
                              np.nan_to_num(np.array(hb[k], dtype=object if k == "phase" else float))), k
    for k, v in ma.state_dict().items():
        assert torch.equal(v.cpu(), mb.state_dict()[k].cpu()), k
    for f in ("best_model_sharpe.pt", "best_model_loss.pt", "final_model.pt"):
        sa = torch.load(tmp_path / "a" / f, weights_only=True)
        sb = torch.load(tmp_path / "b" / f, weights_only=True)
        assert all(torch.equal(sa[k], sb[k]) for k in sa), f


def test_gpu_nonfinite_guard(tmp_path):
    from deeplearninginassetpricing_paperreplication_amd.engine.runner import train_3phase_gpu
    from deeplearninginassetpricing_paperreplication_amd.utils.guards import NonFiniteError
    b = _batch(T=20, N=96)
    b["individual_features"] = b["individual_features"].clone()
    b["individual_features"][3, 5, 0] = float("inf")
    b["mask"] = b["mask"].clone()
    b["mask"][3, 5] = True
    cfg = default_cli_config(8, 46)
    with pytest.raises(NonFiniteError):
        train_3phase_gpu(cfg, b, b, b, num_epochs_unc=3, num_epochs_moment=1, num_epochs=2,
                         print_freq=100, ignore_epoch=0, seed=1, verbose=False, nan_policy="raise")


# ---- wide panels: layer 0 as the streaming k_proj0 / k_wgrad0 GEMMs (F + Dm > 128) ----------
def _wide_engine(monkeypatch, cfg, data, force, seeds=(7,), n_models=1):
    monkeypatch.setenv("DLAP_WIDE", "1" if force else "0")
    eng, b = _engine(cfg, n_models=n_models, seeds=seeds, data=data)
    assert int(eng.desc["wide"]) == 1
    return eng, b


@pytest.mark.parametrize("F,M,force,rnn,hm,K", [(46, 8, True, [4], [], 8), (200, 8, False, [4], [], 8),
                                                (300, 12, False, [2, 3], [16], 4), (140, 6, False, [], [], 8)])
def test_wide_forward_and_gradients_match_fp32_reference(monkeypatch, F, M, force, rnn, hm, K):
    from deeplearninginassetpricing_paperreplication_amd.engine.runner import flatten_state
    cfg = default_cli_config(M, F, rnn_dim=rnn or [4], use_lstm=bool(rnn), num_moments=K,
                             hidden_dim_moment=hm, dropout=0.0)
    data = _batch(T=30, N=150, F=F, M=M)
    eng, b = _wide_engine(monkeypatch, cfg, data, force)
    torch.manual_seed(0)
    model = AssetPricingGAN(cfg)
    eng.set_model(0, model, 7)
    with torch.no_grad():
        out = model(b["macro_features"], b["individual_features"], b["returns"], b["mask"], phase="conditional")
    eng.eng.forward_split(0, False, True)
    T, N = b["mask"].shape
    m = b["mask"].numpy()
    assert _rel(eng.eng.read_ws(0, 0, "wn").reshape(T, N), out["weights"].numpy()) < 3e-2
    h = eng.eng.read_ws(0, 0, "h").reshape(T, N, K)
    assert _rel(h[m], out["moments"].permute(1, 2, 0).numpy()[m]) < 3e-2
    sc = eng.eng.read_ws(0, 0, "scal")
    assert _rel(sc[0], out["loss_conditional"].item()) < 3e-2
    P_sdf = model.spec.param_counts()[0]
    for phase, pname in ((1, "unconditional"), (3, "conditional"), (2, "moment")):
        model.zero_grad()
        o = model(b["macro_features"], b["individual_features"], b["returns"], b["mask"], phase=pname)
        o["loss"].backward()
        ref = flatten_state({k: (p.grad if p.grad is not None else torch.zeros_like(p))
                             for k, p in model.named_parameters()}, model.spec)
        eng.eng.backward_only(phase)
        got = eng.eng.get_grads(0)
        sl = slice(0, P_sdf) if phase != 2 else slice(P_sdf, None)
        err = np.linalg.norm(got[sl] - ref[sl]) / np.linalg.norm(ref[sl])
        cos = np.dot(got[sl], ref[sl]) / (np.linalg.norm(got[sl]) * np.linalg.norm(ref[sl]))
        # bf16 layer-0 operands over F up to 300 inputs: slightly looser than the F=46 bound
        assert err < 0.08 and cos > 0.997, (phase, err, cos)


def test_wide_path_tracks_fused_path_and_is_deterministic(monkeypatch):
    cfg = default_cli_config(8, 46)
    data = _batch()
    runs = {}
    for force in (False, True, True):
        monkeypatch.setenv("DLAP_WIDE", "1" if force else "0")
        eng, _ = _engine(cfg, data=data)
        for ph, n in ((1, 4), (2, 2), (3, 4)):
            eng.eng.begin_phase(ph)
            eng.run(ph, n, 1e-3, 1, 1.0, True)
        eng.eng.sync()
        runs.setdefault(force, []).append((eng.history_rows(0), eng.params(0)))
    (hw0, pw0), (hw1, pw1) = runs[True]
    np.testing.assert_array_equal(pw0, pw1)                       # bitwise reproducible
    np.testing.assert_array_equal(np.nan_to_num(hw0), np.nan_to_num(hw1))
    hf, pf = runs[False][0]
    assert np.isfinite(hw0[:, 1]).all()
    # same math, different rounding (fp32 per-period terms): close, not bitwise
    assert np.abs(pw0 - pf).max() < 5e-3, np.abs(pw0 - pf).max()


def test_device_eval_metrics_match_numpy():
    """Sharpe (unbiased std), mean/std and the scan-based max drawdown of the device metric
    kernel vs the numpy formulas of `/root/reference/src/train.py:29-42` on its own portfolio."""
    from deeplearninginassetpricing_paperreplication_amd.train.metrics import compute_max_drawdown
    cfg = default_cli_config(8, 46)
    for T in (36, 300):
        eng, _ = _engine(cfg, data=_batch(T=T, N=120))
        ev = eng.evaluate(0)[0]
        port = ev["portfolio_returns"].astype(np.float64)
        assert abs(ev["max_drawdown"] - compute_max_drawdown(port)) < 1e-5
        assert abs(ev["mean_return"] - port.mean()) < 1e-6
        assert abs(ev["std_return"] - port.std()) < 1e-5


def test_wide_periods_use_chunked_loss_passes():
    """Periods with more valid rows than one register block (>4096 fwd / >2048 bwd) take the
    chunked streaming paths of k_period_fwd / k_period_bwd: same results as the fp32 model."""
    from deeplearninginassetpricing_paperreplication_amd.engine.runner import flatten_state
    cfg = default_cli_config(8, 46, dropout=0.0)
    b = _batch(T=8, N=12000)
    assert b["mask"].sum(1).min() > 4096
    eng, _ = _engine(cfg, data=b)
    torch.manual_seed(0)
    model = AssetPricingGAN(cfg)
    eng.set_model(0, model, 7)
    with torch.no_grad():
        out = model(b["macro_features"], b["individual_features"], b["returns"], b["mask"], phase="conditional")
    eng.eng.forward_split(0, False, True)
    T, N = b["mask"].shape
    assert _rel(eng.eng.read_ws(0, 0, "wn").reshape(T, N), out["weights"].numpy()) < 3e-2
    assert _rel(eng.eng.read_ws(0, 0, "scal")[0], out["loss_conditional"].item()) < 3e-2
    model.zero_grad()
    o = model(b["macro_features"], b["individual_features"], b["returns"], b["mask"], phase="conditional")
    o["loss"].backward()
    ref = flatten_state({k: (p.grad if p.grad is not None else torch.zeros_like(p))
                         for k, p in model.named_parameters()}, model.spec)
    eng.eng.backward_only(3)
    got = eng.eng.get_grads(0)
    sl = slice(0, model.spec.param_counts()[0])
    cos = np.dot(got[sl], ref[sl]) / (np.linalg.norm(got[sl]) * np.linalg.norm(ref[sl]))
    assert cos > 0.998, cos


def test_wide_model_batching_matches_single_models(monkeypatch):
    monkeypatch.setenv("DLAP_WIDE", "1")
    test_model_batching_matches_single_models()


@pytest.mark.parametrize("wide", ["0", "1"])
def test_edge_panels_all_masked_period_single_observation_asset(monkeypatch, wide):
    """SURVEY §7.4 edge cases through the native engine: a fully masked period, an asset with a
    single observation, N not a multiple of the tile, T = 2 (the shortest split with a Sharpe)."""
    from deeplearninginassetpricing_paperreplication_amd.engine.runner import flatten_state
    monkeypatch.setenv("DLAP_WIDE", wide)
    cfg = default_cli_config(8, 46, dropout=0.0)
    for T, N in ((7, 77), (2, 45)):
        b = _batch(T=T, N=N, seed=3)
        mask = b["mask"].clone()
        mask[T // 2] = False                          # no valid stock in this period
        mask[:, 5] = False
        mask[0, 5] = True                             # one observation for asset 5
        b["mask"] = mask
        b["returns"] = b["returns"] * mask
        b["individual_features"] = b["individual_features"] * mask[..., None]
        eng, _ = _engine(cfg, data=b)
        torch.manual_seed(0)
        model = AssetPricingGAN(cfg)
        eng.set_model(0, model, 7)
        with torch.no_grad():
            out = model(b["macro_features"], b["individual_features"], b["returns"], b["mask"], phase="conditional")
        eng.eng.forward_split(0, False, True)
        assert _rel(eng.eng.read_ws(0, 0, "wn").reshape(T, N), out["weights"].numpy()) < 3e-2
        sc = eng.eng.read_ws(0, 0, "scal")
        assert _rel(sc[0], out["loss_conditional"].item()) < 3e-2
        assert _rel(sc[1], out["loss_unconditional"].item()) < 3e-2
        model.zero_grad()
        o = model(b["macro_features"], b["individual_features"], b["returns"], b["mask"], phase="conditional")
        o["loss"].backward()
        ref = flatten_state({k: (p.grad if p.grad is not None else torch.zeros_like(p))
                             for k, p in model.named_parameters()}, model.spec)
        eng.eng.backward_only(3)
        got = eng.eng.get_grads(0)
        sl = slice(0, model.spec.param_counts()[0])
        assert np.isfinite(got).all()
        cos = np.dot(got[sl], ref[sl]) / (np.linalg.norm(got[sl]) * np.linalg.norm(ref[sl]))
        assert cos > 0.995, (T, N, cos)


def test_epochs_past_history_capacity_are_dropped_not_written_out_of_bounds():
    """More epochs than ``max_epochs``: k_epoch_end keeps the first max_epochs history rows and
    sends later rows to scratch (no write past the history buffer); training itself continues."""
    cfg = default_cli_config(8, 46)
    eng, _ = _engine(cfg, max_epochs=4)
    before = eng.params(0).copy()
    for ph, n in ((1, 3), (3, 4)):
        eng.eng.begin_phase(ph)
        eng.run(ph, n, 1e-3, 0, 1.0, True)
    eng.eng.sync()
    h = eng.history_rows(0)
    assert h.shape[0] == 4
    assert np.isfinite(h[:, 1]).all()
    after = eng.params(0)
    assert np.isfinite(after).all() and np.abs(after - before).max() > 0


@pytest.mark.parametrize("rnn,G,dropout", [([4], 1, 0.05), ([8], 2, 0.05), ([4, 4], 1, 0.3)])
def test_fused_lstm_tower_forward_equals_two_launches(monkeypatch, rnn, G, dropout):
    """k_mlp_fwd_rnn (the LSTM on workgroup 0 publishing its periods, the towers trailing it)
    against the separate LSTM + tower launches: bitwise-equal parameters and history through
    all three phases (graph replays, pipelined), and no spin wait ever gave up."""
    cfg = default_cli_config(8, 46, rnn_dim=rnn, dropout=dropout)
    data = _batch()
    res = []
    for overlap in ("0", "1"):
        monkeypatch.setenv("DLAP_RNN_OVERLAP", overlap)
        eng, _ = _engine(cfg, n_models=G, seeds=(5, 6), data=data)
        assert eng.eng.fused_forward(1) == (overlap == "1")
        assert not eng.eng.fused_forward(2)   # phase 2 keeps the two launches (engine.cpp fused_fwd)
        for ph, n in ((1, 4), (2, 2), (3, 5)):
            eng.eng.begin_phase(ph)
            eng.run(ph, n, 1e-3, 1, 1.0, True)
        eng.eng.backward_only(3)
        eng.eng.sync()
        assert eng.eng.prog_timeouts() == 0
        res.append([(eng.history_rows(g), eng.params(g), eng.eng.get_grads(g)) for g in range(G)])
    for a, b in zip(res[0], res[1]):
        for x, y in zip(a, b):
            np.testing.assert_array_equal(np.nan_to_num(x), np.nan_to_num(y))
