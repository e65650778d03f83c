"""Cross-sectionally sharded training with the local towers on the native engine (MI355X):
``XSectionGAN.attach_engine`` vs the same model with PyTorch towers -- losses, gradients of every
phase's scope and a train step, one rank (the cross-sectional sums are then local; the
multi-rank all-reduce algebra is covered on the CPU by tests/test_xsection.py)."""
import numpy as np
import pytest
import torch

from deeplearninginassetpricing_paperreplication_amd.config import default_cli_config
from deeplearninginassetpricing_paperreplication_amd.data.synthetic import generate_panel_fast
from deeplearninginassetpricing_paperreplication_amd.parallel import comm, xsection as X

pytestmark = pytest.mark.gpu
SPLITS = ("train", "valid", "test")


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from deeplearninginassetpricing_paperreplication_amd.ops import native
    native.load(required=True)


def _shards(dev, T=(24, 8, 10), N=96, F=46, M=8, seed=5):
    ret, feats, mask, mac = generate_panel_fast(sum(T), N, F, M, seed=seed)
    mac = (mac - mac[:T[0]].mean(0)) / (mac[:T[0]].std(0, unbiased=False) + 1e-8)
    mask[:, 0] = False
    cuts = {"train": (0, T[0]), "valid": (T[0], T[0] + T[1]), "test": (T[0] + T[1], sum(T))}
    out = []
    for k in SPLITS:
        a, b = cuts[k]
        sh = X.shard_batch({"returns": ret[a:b].contiguous(), "individual_features": feats[a:b].contiguous(),
                            "mask": mask[a:b].contiguous(), "macro_features": mac[a:b].contiguous()}, 0, 1)
        out.append({k2: (v.to(dev) if isinstance(v, torch.Tensor) else v) for k2, v in sh.items()})
    return out


def _pair(cfg, sh, dev, precision):
    d = comm.Dist(device=dev)
    torch.manual_seed(0)
    mt = X.XSectionGAN(cfg, d).to(dev)
    torch.manual_seed(0)
    me = X.XSectionGAN(cfg, d).to(dev).attach_engine(sh, dev, precision=precision)
    for s, b in enumerate(sh):
        me.et.register(s, b["mask"])
    return mt, me


def _args(b):
    return b["macro_features"], b["individual_features"], b["returns"], b["mask"]


def _scope(model, phase):
    return [p for n, p in model.named_parameters()
            if (n.startswith("moment_net.") if phase == "moment" else n.startswith("sdf_net."))]


@pytest.mark.parametrize("precision,tol", [("fp32", 2e-4), ("bf16", 4e-2)])
def test_engine_towers_match_torch_towers(precision, tol):
    dev = torch.device("cuda:0")
    sh = _shards(dev)
    cfg = default_cli_config(8, 46, dropout=0.0)
    mt, me = _pair(cfg, sh, dev, precision)
    mt.train()
    me.train()
    for phase in ("unconditional", "moment", "conditional"):
        for m in (mt, me):
            m.zero_grad()
        ot = mt(*_args(sh[0]), phase=phase)
        oe = me(*_args(sh[0]), phase=phase)
        lt, le = ot["loss"].item(), oe["loss"].item()
        assert abs(le - lt) <= tol * abs(lt) + 1e-9, (phase, le, lt)
        np.testing.assert_allclose(oe["portfolio_returns"].detach().cpu().numpy(),
                                   ot["portfolio_returns"].detach().cpu().numpy(), rtol=tol, atol=tol * 1e-2)
        ot["loss"].backward()
        oe["loss"].backward()
        gt = torch.cat([p.grad.reshape(-1) for p in _scope(mt, phase)])
        ge = torch.cat([p.grad.reshape(-1) for p in _scope(me, phase)])
        err = float((ge - gt).norm() / gt.norm())
        assert err < (1e-3 if precision == "fp32" else 6e-2), (phase, err)
    # evaluation path (no autograd) on the valid / test shards
    with torch.no_grad():
        mt.eval()
        me.eval()
        for b in sh[1:]:
            wt, _ = mt.get_weights(b["macro_features"], b["individual_features"], b["mask"], normalized=True)
            we, _ = me.get_weights(b["macro_features"], b["individual_features"], b["mask"], normalized=True)
            assert float((we - wt).abs().max() / wt.abs().max()) < tol * 5


def test_engine_xsection_train_3phase_runs():
    """The sharded trainer on the engine: a short full schedule, finite history, parameters move."""
    dev = torch.device("cuda:0")
    sh = _shards(dev)
    cfg = default_cli_config(8, 46)
    d = comm.Dist(device=dev)
    model, hist = X.train_3phase_xsection(cfg, sh[0], sh[1], sh[2], d, device=dev, num_epochs_unc=3,
                                          num_epochs_moment=2, num_epochs=3, print_freq=100, ignore_epoch=0,
                                          verbose=False)
    assert model.et is not None
    assert np.isfinite(np.asarray(hist["train_loss"], dtype=float)).all()


def _rank_worker(rank, world, port, out_path):
    import json
    import os
    os.environ.update(WORLD_SIZE=str(world), RANK=str(rank), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), DLAP_SHARE_GPU="1")
    d = comm.init(backend="gloo", use_gpu=True, timeout_s=120)
    dev = d.device
    full = _shards(dev)
    sh = []
    for b in full:
        s = X.shard_batch({k: v for k, v in b.items() if k != "n_total"}, d.rank, d.world)
        sh.append(s)
    cfg = default_cli_config(8, 46, dropout=0.0)
    torch.manual_seed(0)
    me = X.XSectionGAN(cfg, d).to(dev).attach_engine(sh, dev, precision="fp32")
    for s, b in enumerate(sh):
        me.et.register(s, b["mask"])
    me.train()
    res = {}
    for phase in ("unconditional", "moment", "conditional"):
        me.zero_grad()
        o = me(*_args(sh[0]), phase=phase, n_total=sh[0]["n_total"])
        (o["loss"] / d.world).backward()
        g = torch.cat([p.grad.reshape(-1) for p in _scope(me, phase)])
        torch.distributed.all_reduce(g)
        res[phase] = {"loss": o["loss"].item(), "grad": g.cpu().tolist()}
    if d.rank == 0:
        with open(out_path, "w") as f:
            json.dump(res, f)
    comm.shutdown(d)


def test_engine_xsection_two_ranks_equal_unsharded(tmp_path):
    """Two ranks (gloo, sharing the GPU) with engine towers on half the stocks each reproduce
    the unsharded model's losses and gradients (fp32 engine towers)."""
    import json
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    out = tmp_path / "r0.json"
    mp.start_processes(_rank_worker, args=(2, port, str(out)), nprocs=2, join=True, start_method="spawn")
    res = json.loads(out.read_text())
    dev = torch.device("cuda:0")
    sh = _shards(dev)
    cfg = default_cli_config(8, 46, dropout=0.0)
    torch.manual_seed(0)
    mt = X.XSectionGAN(cfg, comm.Dist(device=dev)).to(dev)
    mt.train()
    for phase in ("unconditional", "moment", "conditional"):
        mt.zero_grad()
        o = mt(*_args(sh[0]), phase=phase)
        o["loss"].backward()
        gt = torch.cat([p.grad.reshape(-1) for p in _scope(mt, phase)]).cpu()
        ge = torch.tensor(res[phase]["grad"])
        assert abs(res[phase]["loss"] - o["loss"].item()) <= 2e-4 * abs(o["loss"].item()), phase
        assert float((ge - gt).norm() / gt.norm()) < 1e-3, phase


def test_tower_dropout_independent_across_ranks():
    """every rank's EngineTowers used the same dropout seed, so local stock i of two
    shards drew the same tower masks. The towers are now salted per rank (the LSTM keeps the
    shared seed): equal salts reproduce the masks, different salts give independent ones."""
    from deeplearninginassetpricing_paperreplication_amd.models.gan import AssetPricingGAN
    from deeplearninginassetpricing_paperreplication_amd.ops.fused import _ordered_params
    dev = torch.device("cuda:0")
    sh = _shards(dev)
    cfg = default_cli_config(8, 46, dropout=0.3)
    torch.manual_seed(0)
    model = AssetPricingGAN(cfg).to(dev)
    params = _ordered_params(model)
    outs = {}
    for salt in (1, 1, 2):
        et = X.EngineTowers(model, sh, dev, seed=11, precision="fp32", tower_salt=salt)
        et.sync_params(params, True)
        w, _ = et.forward(0, True, False)
        outs.setdefault(salt, []).append(w.clone())
        torch.cuda.synchronize()
    m = sh[0]["mask"]
    a, b, c = outs[1][0][m], outs[1][1][m], outs[2][0][m]
    assert torch.equal(a, b)
    frac = float((a != c).float().mean())
    assert frac > 0.5, frac                # different masks change (almost) every row's output


# ---- the whole epoch on the engine (XSEngine: all-reduce callbacks between the engine's passes)
_SCHED = dict(num_epochs_unc=4, num_epochs_moment=3, num_epochs=4, print_freq=100, ignore_epoch=0,
              precision="fp32", verbose=False)


def _full_splits(dev):
    full = _shards(dev)
    return [{k: v for k, v in b.items() if k != "n_total"} for b in full]


def _plain_run(dev):
    from deeplearninginassetpricing_paperreplication_amd.engine.runner import flatten_state, train_3phase_gpu
    from deeplearninginassetpricing_paperreplication_amd.models.gan import AssetPricingGAN
    cfg = default_cli_config(8, 46, dropout=0.0)
    torch.manual_seed(42)
    model = AssetPricingGAN(cfg)
    m, hist = train_3phase_gpu(cfg, *_full_splits(dev), device=dev, seed=42, models=[model], seeds=[42], **_SCHED)
    return flatten_state(m, m.spec), hist, m.engine_final_eval


def test_xs_engine_one_rank_matches_engine():
    """One rank: the sharded epoch (staged period passes, Gram losses, unfused tail, eager epochs)
    trains the same model as the production engine (fp32: rounding-level differences only)."""
    from deeplearninginassetpricing_paperreplication_amd.engine.runner import flatten_state
    dev = torch.device("cuda:0")
    ref, href, fref = _plain_run(dev)
    cfg = default_cli_config(8, 46, dropout=0.0)
    m, hist = X.train_3phase_xsection_engine(cfg, *_full_splits(dev), comm.Dist(device=dev), device=dev, seed=42,
                                             **_SCHED)
    assert X.train_3phase_xsection_engine.last_xs.n_calls > 0        # the callbacks fired
    got = flatten_state(m, m.spec)
    np.testing.assert_allclose(got, ref, rtol=1e-4, atol=2e-6)
    np.testing.assert_allclose(hist["train_loss"], href["train_loss"], rtol=1e-4)
    np.testing.assert_allclose(hist["valid_sharpe"], href["valid_sharpe"], rtol=1e-3, atol=1e-4)
    for s in fref:
        assert abs(m.engine_final_eval[s]["sharpe"] - fref[s]["sharpe"]) < 1e-3


def _xs_rank_worker(rank, world, port, out_path):
    import json
    import os
    os.environ.update(WORLD_SIZE=str(world), RANK=str(rank), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), DLAP_SHARE_GPU="1")
    from deeplearninginassetpricing_paperreplication_amd.engine.runner import flatten_state
    d = comm.init(backend="gloo", use_gpu=True, timeout_s=120)
    dev = d.device
    cfg = default_cli_config(8, 46, dropout=0.0)
    m, hist = X.train_3phase_xsection_engine(cfg, *_full_splits(dev), d, device=dev, seed=42, **_SCHED)
    p = flatten_state(m, m.spec)
    allp = [torch.zeros_like(torch.from_numpy(p)) for _ in range(world)]
    torch.distributed.all_gather(allp, torch.from_numpy(p))
    if d.rank == 0:
        with open(out_path, "w") as f:
            json.dump({"params": p.tolist(), "replicas_equal": all(torch.equal(allp[0], q) for q in allp),
                       "train_loss": hist["train_loss"], "valid_sharpe": hist["valid_sharpe"],
                       "sharpe": {str(s): float(v["sharpe"]) for s, v in m.engine_final_eval.items()}}, f)
    comm.shutdown(d)


def test_xs_engine_two_ranks_equal_unsharded(tmp_path):
    """Two ranks (gloo, sharing the GPU), half the stocks each, the whole 3-phase schedule on the
    engine with the all-reduce callbacks: the replicas stay bit-identical and train the unsharded
    model (fp32; the cross-rank sums only reorder fp32 additions)."""
    import json
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    out = tmp_path / "r0.json"
    mp.start_processes(_xs_rank_worker, args=(2, port, str(out)), nprocs=2, join=True, start_method="spawn")
    res = json.loads(out.read_text())
    dev = torch.device("cuda:0")
    ref, href, fref = _plain_run(dev)
    assert res["replicas_equal"]
    np.testing.assert_allclose(np.asarray(res["params"], dtype=np.float32), ref, rtol=1e-4, atol=5e-6)
    np.testing.assert_allclose(res["train_loss"], href["train_loss"], rtol=2e-4)
    for s, v in res["sharpe"].items():
        assert abs(v - fref[int(s)]["sharpe"]) < 2e-3
