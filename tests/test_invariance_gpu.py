"""Batching / sharding invariance and the fused forward's safety guarantees on a real MI355X.

* A member's trajectory is a function of its seed and hyperparameters only: the same seed trained
  alone or batched with 1, 2 or 8 other models (at any position) gives bitwise-identical
  parameters, history and snapshots (the backward's fine-slab partition and the
  Gram split-K partition depend on R / T only). The reference's ensemble is defined by its seeds
  (`/root/reference/src/evaluate_ensemble.py:112-157`), so the same 9 seeds must give the same
  ensemble on 1, 2, 4 or 8 GPUs.
* Per-member dropout: a batched member with rate p equals a solo engine built with p
  (`/root/reference/src/model.py:314`; BASELINE config 4's dropout axis).
* The fused LSTM + tower launch only runs when its whole grid is co-resident (occupancy query),
  and a wait that gives up poisons the model on the device: no update, NaN epochs, the host raises.

Panel: the bench size (T = 240 / 60 / 300, N = 3000, F = 46, M = 178), large enough that no grid
cap of the engine binds (256 fine slabs per model)."""
import os
import sys

import numpy as np
import pytest
import torch

from deeplearninginassetpricing_paperreplication_amd.config import default_cli_config
from deeplearninginassetpricing_paperreplication_amd.models.gan import AssetPricingGAN

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PHASES = ((1, 5), (2, 3), (3, 5))


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from deeplearninginassetpricing_paperreplication_amd.ops import native
    native.load(required=True)


@pytest.fixture(scope="module")
def big():
    sys.path.insert(0, ROOT)
    from bench import make_panel
    tr, va, te = make_panel(seed=3, device="cuda", keep_on_device=True)
    return tr, va, te


def _train(data, cfg, seeds, G, phases=PHASES, dropouts=None, pipeline=True):
    from deeplearninginassetpricing_paperreplication_amd.engine.runner import GANEngine
    eng = GANEngine(AssetPricingGAN(cfg).spec, G, max_epochs=64)
    eng.set_data(*data)
    eng.eng.set_pipeline(pipeline)
    for g in range(G):
        torch.manual_seed(1000 + seeds[g])             # init weights follow the seed, not the slot
        eng.set_model(g, AssetPricingGAN(cfg), seeds[g])
        if dropouts is not None:
            eng.eng.set_dropout(g, dropouts[g])
    for ph, n in phases:
        eng.eng.begin_phase(ph)
        eng.run(ph, n, 1e-3, 1, 1.0, True)
    eng.eng.sync()
    assert eng.eng.prog_timeouts() == 0
    out = {seeds[g]: (eng.params(g), np.nan_to_num(eng.history_rows(g), nan=-7.0), eng.params(g, "sharpe"),
                      eng.params(g, "loss")) for g in range(G)}
    return eng, out


def _same(a, b):
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)


def test_member_is_bitwise_independent_of_batch_size_and_position(big):
    cfg = default_cli_config(178, 46)
    _, solo = _train(big, cfg, [123], 1)
    layouts = {2: [7, 123], 3: [7, 8, 123], 9: [0, 1, 2, 3, 123, 5, 6, 7, 8]}
    for G, seeds in layouts.items():
        eng, res = _train(big, cfg, seeds, G)
        _same(solo[123], res[123])
        info = eng.eng.fused_info()
        for ph in (1, 3):            # a fused launch never asks for more than is resident at once
            gx = info[f"train_gx_p{ph}"]
            assert gx == 0 or (1 + gx) * G <= info["cap_train"], info
        del eng


def test_nine_seeds_same_members_on_any_sharding(big):
    """The 9-seed ensemble split 9 / 5+4 / 3+2+2+2 over engines (what 1, 2 or 4 ranks run):
    identical member trajectories."""
    cfg = default_cli_config(178, 46)
    seeds = list(range(9))
    _, whole = _train(big, cfg, seeds, 9)
    for parts in ((seeds[:5], seeds[5:]), (seeds[:3], seeds[3:5], seeds[5:7], seeds[7:])):
        for p in parts:
            _, res = _train(big, cfg, p, len(p))
            for s in p:
                _same(whole[s], res[s])


def test_per_member_dropout_equals_solo_engines(big):
    rates = [0.0, 0.05, 0.2]
    seeds = [31, 32, 33]
    cfg = default_cli_config(178, 46, dropout=0.05)
    eng, res = _train(big, cfg, seeds, 3, dropouts=rates)
    assert [eng.eng.get_dropout(g) for g in range(3)] == pytest.approx(rates)
    for s, p in zip(seeds, rates):
        _, solo = _train(big, default_cli_config(178, 46, dropout=p), [s], 1)
        _same(solo[s], res[s])
    # the rates matter: the 0.2 member differs from the same seed at 0.05
    _, other = _train(big, cfg, [33], 1)
    assert not np.array_equal(other[33][0], res[33][0])


def test_fused_forward_capped_grid_equals_two_launches(big, monkeypatch):
    """A co-residency capacity smaller than the tuned grid caps the fused launch (bitwise the
    same results: the forward is per row); below a minimum grid the engine uses two launches."""
    cfg = default_cli_config(178, 46)
    monkeypatch.setenv("DLAP_RNN_OVERLAP", "0")
    _, ref = _train(big, cfg, [5, 6], 2)
    monkeypatch.setenv("DLAP_RNN_OVERLAP", "1")
    monkeypatch.setenv("DLAP_FUSED_CAP", "80")           # 2 jobs x (1 + 39)
    eng, res = _train(big, cfg, [5, 6], 2)
    info = eng.eng.fused_info()
    assert info["train_gx_p1"] == 39 and info["train_gx_p3"] == 39, info
    for s in (5, 6):
        _same(ref[s], res[s])
    monkeypatch.setenv("DLAP_FUSED_CAP", "20")           # 2 x (1 + 9): below the minimum grid
    eng, _ = _train(big, cfg, [5, 6], 2, phases=())
    assert not eng.eng.fused_forward(1) and not eng.eng.fused_forward(3)


def test_eval_recurrences_in_fused_forward_equal_separate_branch(big, monkeypatch):
    """The pipelined epoch with the evaluation splits' projections and recurrences inside the
    training prologue / fused forward (one launch, workgroups 1 .. 2 of each model) gives the bits
    of the round-4 graph whose evaluation branch ran its own LSTM launches."""
    cfg = default_cli_config(178, 46)
    monkeypatch.setenv("DLAP_EVAL_IN_FWD", "0")
    e0, ref = _train(big, cfg, [21, 22], 2)
    assert not e0.eng.fused_info()["eval_in_fwd_p3"]
    monkeypatch.setenv("DLAP_EVAL_IN_FWD", "1")
    e1, res = _train(big, cfg, [21, 22], 2)
    info = e1.eng.fused_info()
    assert info["eval_in_fwd_p1"] and info["eval_in_fwd_p3"], info
    for ph in (1, 3):       # (1 recurrence + 2 evaluation recurrences + towers) per model, resident
        assert (1 + info["eval_per_model"] + info[f"all_gx_p{ph}"]) * 2 <= info["cap_all"], info
    for s in (21, 22):
        _same(ref[s], res[s])


def test_fused_backward_tail_equals_separate_kernels(big, monkeypatch):
    """k_lstm_tail (the per-period sums, the LSTM BPTT with its weight gradients, the layer-0
    W_ih gradient and the weight-slab sums in ONE launch; the LSTM block waits for the period
    blocks in-kernel) gives the bits of k_finalize -> k_lstm_bwd -> k_wgrad, batched models
    included."""
    cfg = default_cli_config(178, 46)
    monkeypatch.setenv("DLAP_FUSED_TAIL", "0")
    e0, ref = _train(big, cfg, [51, 52], 2)
    assert not e0.eng.fused_info()["fused_tail"]
    monkeypatch.setenv("DLAP_FUSED_TAIL", "1")
    e1, res = _train(big, cfg, [51, 52], 2)
    assert e1.eng.fused_info()["fused_tail"]
    for s in (51, 52):
        _same(ref[s], res[s])


@pytest.mark.parametrize("rnn", [[8], [4, 4], [8, 8]])
def test_fused_backward_tail_other_lstm_shapes(big, monkeypatch, rnn):
    """The fused tail beyond one layer of width 4 (the paper grid's SMV = 8 and
    stacked LSTMs): k_lstm_bwd's serial chain inside the tail launch -- bits of the separate
    kernels -- and the split epoch graphs with the update in the tail on top of it."""
    cfg = default_cli_config(178, 46, rnn_dim=rnn, dropout=0.05)
    ph = ((1, 3), (2, 2), (3, 3))
    monkeypatch.setenv("DLAP_FUSED_TAIL", "0")
    e0, ref = _train(big, cfg, [61, 62], 2, phases=ph)
    assert not e0.eng.fused_info()["fused_tail"]
    monkeypatch.setenv("DLAP_FUSED_TAIL", "1")
    monkeypatch.setenv("DLAP_SPLIT_GRAPHS", "0")
    monkeypatch.setenv("DLAP_TAIL_ADAM", "0")
    e1, res = _train(big, cfg, [61, 62], 2, phases=ph)
    info = e1.eng.fused_info()
    assert info["fused_tail"] and not info["adam_in_tail"], info
    for s in (61, 62):
        _same(ref[s], res[s])
    monkeypatch.setenv("DLAP_SPLIT_GRAPHS", "1")
    monkeypatch.setenv("DLAP_TAIL_ADAM", "1")
    e2, res2 = _train(big, cfg, [61, 62], 2, phases=ph)
    info = e2.eng.fused_info()
    # (SMV = 8 on this panel: the fused forward's LDS cannot hold the 300-step test recurrence at
    # width 8, so the epochs run the one-graph pipeline with the update after the join)
    if rnn == [4, 4]:
        assert info["split_graphs"] and info["adam_in_tail"], info
    for s in (61, 62):
        _same(ref[s], res2[s])


@pytest.mark.parametrize("rnn,mom_hidden", [([4], []), ([8], [32]), ([4, 4], [])])
def test_phase2_tail_and_lstm_once_equal_separate_kernels(big, monkeypatch, rnn, mom_hidden):
    """Phase 2 as [k_proj (moment bias table)] -> towers -> losses -> moment backward -> ONE tail
    launch (per-period sums, the W_macro gradient, the train metrics and the moment network's
    clip + Adam) with the frozen SDF's LSTM state computed once per run instead of every epoch:
    the bits of k_finalize -> k_wgrad -> k_adam with the recurrence in every epoch."""
    cfg = default_cli_config(178, 46, rnn_dim=rnn, hidden_dim_moment=mom_hidden, dropout=0.05)
    ph = ((1, 2), (2, 5), (3, 2))
    monkeypatch.setenv("DLAP_MOM_TAIL", "0")
    monkeypatch.setenv("DLAP_P2_LSTM_CACHE", "0")
    e0, ref = _train(big, cfg, [91, 92], 2, phases=ph)
    info = e0.eng.fused_info()
    assert not info["mom_tail"] and not info["p2_lstm_cached"], info
    monkeypatch.setenv("DLAP_MOM_TAIL", "1")
    monkeypatch.setenv("DLAP_P2_LSTM_CACHE", "1")
    e1, res = _train(big, cfg, [91, 92], 2, phases=ph)
    info = e1.eng.fused_info()
    assert info["mom_tail"] and info["p2_lstm_cached"] == (len(rnn) == 1), info
    for s in (91, 92):
        _same(ref[s], res[s])


def test_adam_in_tail_equals_k_adam(big, monkeypatch):
    """The pipelined epoch's update in the backward tail's last blocks (waiting in-kernel for
    every gradient writer and for the evaluation branch's bookkeeping signal, the branches joined
    only at the graph end) gives the bits of the join + k_adam graphs: parameters, history rows
    (gradient norms, best-epoch flags) and snapshots, batched models included."""
    cfg = default_cli_config(178, 46)
    monkeypatch.setenv("DLAP_SPLIT_GRAPHS", "0")
    monkeypatch.setenv("DLAP_TAIL_ADAM", "0")
    e0, ref = _train(big, cfg, [71, 72], 2)
    assert not e0.eng.fused_info()["adam_in_tail"]
    # (the one-graph fallback runs the update in the tail only on request: DLAP_TAIL_ADAM=2)
    monkeypatch.setenv("DLAP_TAIL_ADAM", "1")
    e1, _ = _train(big, cfg, [71, 72], 2, phases=((1, 2),))
    assert not e1.eng.fused_info()["adam_in_tail"]
    monkeypatch.setenv("DLAP_TAIL_ADAM", "2")
    e1, res = _train(big, cfg, [71, 72], 2)
    assert e1.eng.fused_info()["adam_in_tail"]
    for s in (71, 72):
        _same(ref[s], res[s])


def test_split_epoch_graphs_equal_one_graph(big, monkeypatch):
    """The training chain and the evaluation branch as two graphs on two queues with no graph
    edge between them (in-kernel waits: the evaluation graph for the fused forward's evaluation
    recurrences, the tail's Adam blocks for the bookkeeping's signal) give the bits of the
    one-graph pipelined epoch, batched models included."""
    cfg = default_cli_config(178, 46)
    phases = ((1, 11), (2, 2), (3, 10))      # (9-10 body epochs: the unrolled graphs and singles)
    monkeypatch.setenv("DLAP_SPLIT_GRAPHS", "0")
    e0, ref = _train(big, cfg, [81, 82], 2, phases=phases)
    assert not e0.eng.fused_info()["split_graphs"]
    monkeypatch.setenv("DLAP_SPLIT_GRAPHS", "1")
    e1, res = _train(big, cfg, [81, 82], 2, phases=phases)
    assert e1.eng.fused_info()["split_graphs"]
    for s in (81, 82):
        _same(ref[s], res[s])


def test_eval_recurrences_on_the_eval_queue_equal_in_training_launch(big, monkeypatch):
    """Split epoch graphs with the evaluation splits' recurrences in the evaluation graph's own
    fused LSTM + tower forward (after an in-kernel wait for the previous update, k_wait_gen)
    instead of inside the training chain's fused forward: the bits of the round-5 split graphs,
    batched models included."""
    cfg = default_cli_config(178, 46)
    phases = ((1, 11), (2, 2), (3, 10))
    monkeypatch.setenv("DLAP_EVAL_SEP", "0")
    e0, ref = _train(big, cfg, [83, 84], 2, phases=phases)
    info = e0.eng.fused_info()
    assert info["split_graphs"] and not info["eval_sep"], info
    monkeypatch.setenv("DLAP_EVAL_SEP", "1")
    e1, res = _train(big, cfg, [83, 84], 2, phases=phases)
    info = e1.eng.fused_info()
    assert info["split_graphs"] and info["eval_sep"], info
    for s in (83, 84):
        _same(ref[s], res[s])


def test_train_gram_on_eval_stream_equals_in_chain(big, monkeypatch):
    """The train split's moment refresh and Gram build at a phase start on the evaluation stream,
    the head epoch's forward beside them and its loss pass waiting for them (two head graphs):
    the bits of the build on the training stream ahead of the head."""
    cfg = default_cli_config(178, 46)
    phases = ((1, 4), (2, 2), (3, 4), (3, 3))
    monkeypatch.setenv("DLAP_TRAIN_GRAM_SIDE", "0")
    _, ref = _train(big, cfg, [85, 86], 2, phases=phases)
    monkeypatch.setenv("DLAP_TRAIN_GRAM_SIDE", "1")
    _, res = _train(big, cfg, [85, 86], 2, phases=phases)
    for s in (85, 86):
        _same(ref[s], res[s])


def test_self_projecting_recurrences_equal_k_proj(big, monkeypatch):
    """The fused forward's recurrences computing their own layer-0 input projections tile by tile
    (spare waves of their workgroups, no k_proj launch) give the bits of k_proj + staged inputs."""
    cfg = default_cli_config(178, 46)
    monkeypatch.setenv("DLAP_SELF_PROJ", "0")
    _, ref = _train(big, cfg, [61, 62], 2)
    monkeypatch.setenv("DLAP_SELF_PROJ", "1")
    _, res = _train(big, cfg, [61, 62], 2)
    for s in (61, 62):
        _same(ref[s], res[s])


def test_fused_phase2_under_the_guarantee_equals_two_launches(big, monkeypatch):
    """Phase 2's fused forward (opt-in, DLAP_FUSED_PHASE2=1) runs on the capped grid and gives the
    same bits as the two-launch path."""
    cfg = default_cli_config(178, 46)
    _, ref = _train(big, cfg, [9], 1)
    monkeypatch.setenv("DLAP_FUSED_PHASE2", "1")
    eng, res = _train(big, cfg, [9], 1)
    assert eng.eng.fused_forward(2)
    gx = eng.eng.fused_info()["train_gx_p2"]
    assert 0 < gx and 1 + gx <= eng.eng.fused_info()["cap_train"]
    _same(ref[9], res[9])


def test_adam_fused_repack_equals_separate_pack(big, monkeypatch):
    """k_adam writing every updated parameter's packed copies itself (scatter lists built from
    k_pack_index) gives the bits of Adam followed by a full k_pack: parameters, history,
    snapshots, Adam moments and step counters, with per-member dropout scales in the blob."""
    cfg = default_cli_config(178, 46, dropout=0.05)
    monkeypatch.setenv("DLAP_FUSED_PACK", "0")
    e0, ref = _train(big, cfg, [41, 42], 2, dropouts=[0.0, 0.1])
    assert not e0.eng.fused_info()["fused_pack"]
    monkeypatch.setenv("DLAP_FUSED_PACK", "1")
    e1, res = _train(big, cfg, [41, 42], 2, dropouts=[0.0, 0.1])
    assert e1.eng.fused_info()["fused_pack"]
    for g, s in enumerate((41, 42)):
        _same(ref[s], res[s])
        a, b = e0.eng.get_opt_state(g), e1.eng.get_opt_state(g)
        for k in ("m", "v"):
            np.testing.assert_array_equal(a[k], b[k])
        assert [a[k] for k in ("step_sdf", "step_moment", "drop_step")] == \
            [b[k] for k in ("step_sdf", "step_moment", "drop_step")] == [10, 3, 13]


def test_fused_wait_give_up_poisons_the_model(monkeypatch):
    """Force every fused wait to give up (spin limit 0): the launch writes nothing, the model is
    never updated (parameters bit-identical to the initial ones), every epoch is recorded as NaN
    with no snapshot taken, and the GPU trainer raises at its next synchronisation."""
    from deeplearninginassetpricing_paperreplication_amd.data.synthetic import generate_panel_fast
    from deeplearninginassetpricing_paperreplication_amd.engine.runner import GANEngine, train_3phase_gpu
    ret, feats, mask, mac = generate_panel_fast(96, 600, 46, 8, seed=1)
    mac = (mac - mac.mean(0)) / (mac.std(0, unbiased=False) + 1e-8)
    b = {"returns": ret, "individual_features": feats, "mask": mask, "macro_features": mac}
    cfg = default_cli_config(8, 46)
    monkeypatch.setenv("DLAP_PROG_SPIN_LIMIT", "0")
    torch.manual_seed(0)
    eng = GANEngine(AssetPricingGAN(cfg).spec, 1, max_epochs=16)
    eng.set_data(b, b, b)
    eng.set_model(0, AssetPricingGAN(cfg), 3)
    assert eng.eng.fused_forward(1)
    p0 = eng.params(0).copy()
    eng.eng.begin_phase(1)
    eng.run(1, 4, 1e-3, 0, 1.0, True)
    eng.eng.sync()
    assert eng.eng.prog_timeouts() > 0
    np.testing.assert_array_equal(eng.params(0), p0)
    h = eng.history_rows(0)
    # every metric NaN, no best-model flag (columns 21, 22) raised
    assert h.shape[0] == 4 and np.isnan(h[:, 1:21]).all() and (h[:, 21:23] == 0).all()
    assert list(eng.eng.snap_flags(0)) == [0, 0]
    eng.eng.reset_prog_errors()
    assert eng.eng.prog_timeouts() == 0
    with pytest.raises(RuntimeError, match="spin wait gave up"):
        train_3phase_gpu(cfg, b, b, b, num_epochs_unc=4, num_epochs_moment=1, num_epochs=2, print_freq=2,
                         ignore_epoch=0, verbose=False, seed=3, wait_fallback=False)


def test_wait_give_up_falls_back_to_safe_mode(monkeypatch):
    """a spin wait that gives up no longer ends the run -- the GPU trainer
    restores the models to the start of the print interval and re-runs it (and the rest of the
    run) without cross-launch waits. Forced here with a zero spin limit for the first interval:
    the final state, history and snapshots are the bits of an undisturbed run."""
    from deeplearninginassetpricing_paperreplication_amd.data.synthetic import generate_panel_fast
    from deeplearninginassetpricing_paperreplication_amd.engine.runner import train_3phase_gpu
    ret, feats, mask, mac = generate_panel_fast(96, 600, 46, 8, seed=1)
    mac = (mac - mac.mean(0)) / (mac.std(0, unbiased=False) + 1e-8)
    b = {"returns": ret, "individual_features": feats, "mask": mask, "macro_features": mac}
    cfg = default_cli_config(8, 46)
    kw = dict(num_epochs_unc=6, num_epochs_moment=2, num_epochs=6, print_freq=3, ignore_epoch=0, verbose=False,
              seed=3)

    def run():
        torch.manual_seed(0)
        m, h = train_3phase_gpu(cfg, b, b, b, **kw)
        e = train_3phase_gpu.last_engine
        return (e.params(0), e.params(0, "sharpe"), e.params(0, "loss"), np.asarray(h["valid_sharpe"])), \
            dict(train_3phase_gpu.last_wait_fallback)

    ref, fb0 = run()
    assert fb0["reruns"] == 0
    monkeypatch.setenv("DLAP_PROG_SPIN_LIMIT", "0")
    got, fb1 = run()
    assert fb1["reruns"] == 1 and fb1["safe"], fb1
    assert train_3phase_gpu.last_engine.eng.prog_timeouts() == 0
    for x, y in zip(ref, got):
        np.testing.assert_array_equal(x, y)


def test_tail_adam_handoff_survives_a_new_train_split(big, monkeypatch):
    """The tail's Adam hand-off derives its launch index from running counts divided by the
    launch's block count, which depends on the train split: pipelined epochs, then
    set_data with a shorter train split, then more epochs on the same engine -- the bits of the
    join + k_adam engine doing the same (no running counts)."""
    from deeplearninginassetpricing_paperreplication_amd.engine.runner import GANEngine
    cfg = default_cli_config(178, 46)
    tr, va, te = big
    tr2 = {k: v[:200].contiguous() for k, v in tr.items()}

    def run(tail_adam):
        monkeypatch.setenv("DLAP_TAIL_ADAM", tail_adam)
        eng = GANEngine(AssetPricingGAN(cfg).spec, 2, max_epochs=64)
        eng.set_data(tr, va, te)
        for g, s in enumerate((91, 92)):
            torch.manual_seed(1000 + s)
            eng.set_model(g, AssetPricingGAN(cfg), s)
        eng.eng.begin_phase(1)
        eng.run(1, 11, 1e-3, 1, 1.0, True)
        eng.set_data(tr2, va, te)
        eng.eng.begin_phase(1)
        eng.run(1, 10, 1e-3, 1, 1.0, True)
        eng.eng.sync()
        assert eng.eng.prog_timeouts() == 0
        return eng, [(eng.params(g), np.nan_to_num(eng.history_rows(g), nan=-7.0)) for g in range(2)]

    e1, res = run("1")
    assert e1.eng.fused_info()["adam_in_tail"]
    _, ref = run("0")
    for a, b in zip(res, ref):
        _same(a, b)


def test_concurrent_engines_split_graphs_no_giveups(big):
    """Three live engines running split-graph epochs at the same time from three threads (the
    engine releases the GIL) beside a busy torch stream: no in-kernel wait gives up, and every
    member has the bits of its solo run (the evaluation queue of each engine is its
    own CU-masked stream, the runtime's queue pooling cannot put one engine's waits in front of
    the work they wait for)."""
    import threading
    from deeplearninginassetpricing_paperreplication_amd.engine.runner import GANEngine
    cfg = default_cli_config(178, 46)
    seeds = (101, 102, 103)
    phases = ((1, 9), (3, 9))
    _, solo = zip(*[_train(big, cfg, [s], 1, phases=phases) for s in seeds])
    engs = []
    for s in seeds:
        eng = GANEngine(AssetPricingGAN(cfg).spec, 1, max_epochs=64)
        eng.set_data(*big)
        torch.manual_seed(1000 + s)
        eng.set_model(0, AssetPricingGAN(cfg), s)
        assert eng.eng.fused_info()["split_graphs"]
        engs.append(eng)
    errs = []

    def work(eng):
        try:
            for ph, n in phases:
                eng.eng.begin_phase(ph)
                eng.run(ph, n, 1e-3, 1, 1.0, True)
            eng.eng.sync()
        except Exception as e:          # pragma: no cover - reported below
            errs.append(e)

    th = [threading.Thread(target=work, args=(e,)) for e in engs]
    x = torch.randn(2048, 2048, device="cuda")
    side = torch.cuda.Stream()
    for t in th:
        t.start()
    with torch.cuda.stream(side):        # a busy torch stream beside the three engines
        for _ in range(40):
            x = torch.tanh(x @ x * 1e-3)
    for t in th:
        t.join()
    torch.cuda.synchronize()
    assert not errs, errs
    for eng, s, ref in zip(engs, seeds, solo):
        assert eng.eng.prog_timeouts() == 0
        out = (eng.params(0), np.nan_to_num(eng.history_rows(0), nan=-7.0), eng.params(0, "sharpe"),
               eng.params(0, "loss"))
        _same(ref[s], out)
