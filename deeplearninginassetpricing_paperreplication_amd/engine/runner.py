"""Python driver of the native engine: model <-> flat parameters, the GPU ``train_3phase``.

``GANEngine`` trains G models of one architecture at once on one GPU (ensemble members or
sweep configurations that share a shape). The schedule is `/root/reference/src/train.py:156-426`
executed as hipGraph replays of one captured epoch per phase; the host only synchronises at
``print_freq`` boundaries and at phase ends, where it also writes the checkpoint files whose
final on-disk state equals the reference's "last writer wins" sequence.
"""
from __future__ import annotations

import os
import time
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from ..config import ModelSpec
from ..ops.native import load as load_native

HIST = dict(phase=0, train_loss=1, train_sharpe=2, valid_loss=3, valid_sharpe=4, test_loss=5,
            test_sharpe=6, train_loss_unc=7, train_loss_cond=8, grad_norm=9, valid_loss_unc=10,
            valid_loss_cond=11, valid_mdd=12, valid_mean=13, valid_std=14, test_loss_unc=15,
            test_loss_cond=16, test_mdd=17, test_mean=18, test_std=19, train_loss_res=20,
            best_loss=21, best_sharpe=22)
SC = dict(loss_cond=0, loss_unc=1, loss_res=2, train_sharpe=3, sharpe=4, mean=5, std=6, mdd=7)


def flatten_state(model_or_sd, spec: ModelSpec) -> np.ndarray:
    sd = model_or_sd.state_dict() if hasattr(model_or_sd, "state_dict") else model_or_sd
    parts = []
    for k, shp in spec.param_layout():
        t = sd[k].detach().float().cpu()
        if tuple(t.shape) != tuple(shp):
            raise ValueError(f"{k}: shape {tuple(t.shape)} != {shp}")
        parts.append(t.reshape(-1).numpy())
    return np.ascontiguousarray(np.concatenate(parts), dtype=np.float32)


def unflatten_state(flat: np.ndarray, spec: ModelSpec) -> Dict[str, torch.Tensor]:
    out, o = {}, 0
    for k, shp in spec.param_layout():
        n = int(np.prod(shp))
        out[k] = torch.from_numpy(np.array(flat[o:o + n], dtype=np.float32).reshape(shp))
        o += n
    return out


def _on_device(x, dtype: torch.dtype, dev: torch.device) -> torch.Tensor:
    t = x if isinstance(x, torch.Tensor) else torch.as_tensor(np.asarray(x))
    return t.detach().to(device=dev, dtype=dtype).contiguous()


class SplitInfo:
    """Shape of a split the engine holds (T, N, R valid rows); ``rowti`` [R, 2] is read back from
    the device on first use (tests)."""

    def __init__(self, eng, s: int, T: int, N: int, R: int):
        self._eng, self._s = eng, s
        self.T, self.N, self.R = T, N, R
        self._rowti = None

    @property
    def rowti(self) -> np.ndarray:
        if self._rowti is None:
            self._rowti = np.asarray(self._eng.read_split(self._s)["rowti"]).reshape(-1, 2)
        return self._rowti


class GANEngine:
    """Native multi-model trainer for one architecture (``spec``) on the current GPU.

    ``precision``: "bf16" (production: bf16 tower GEMM operands, fp32 accumulation / master
    weights / losses) or "fp32" (the reference's precision end to end: fp32 panel rows and
    weight fragments through fp32 MFMA tiles, the wide layer-0 path included)."""

    def __init__(self, spec: ModelSpec, n_models: int = 1, max_epochs: int = 4096, precision: str = "bf16"):
        if precision not in ("bf16", "fp32"):
            raise ValueError(f"precision must be 'bf16' or 'fp32', not {precision!r}")
        nat = load_native()
        self.spec = spec
        self.G = n_models
        self.fp32 = precision == "fp32"
        self.eng = nat.Engine(
            F=spec.individual_dim, M=spec.macro_dim, nrnn=spec.rnn_layers, H=spec.rnn_hidden,
            raw_macro_sdf=(spec.rnn_layers == 0 and spec.macro_dim > 0),
            hidden=list(spec.hidden), mom_hidden=list(spec.moment_hidden), K=spec.num_moments,
            dropout=spec.dropout, normalize_w=spec.normalize_w, weighted=spec.weighted_loss,
            residual=spec.residual_loss_factor, G=n_models, max_epochs=max_epochs, fp32=self.fp32)
        self.desc = self.eng.describe()
        self.KP = int(self.desc["KP"])
        self.splits: Dict[int, object] = {}

    # ---- data -----------------------------------------------------------------------
    # host splits whose dense fp32 features exceed this are compacted on the host and only the
    # compact bf16 rows are uploaded (a dense device copy of the scaled 600x30000x512 panel would
    # be ~37 GB of temporaries); smaller host splits take the device path (faster, same bits:
    # tests/test_panel_gpu.py)
    HOST_COMPACT_BYTES = 1 << 31

    def set_data(self, train: Dict, valid: Optional[Dict] = None, test: Optional[Dict] = None):
        """Upload the splits. The engine builds its compacted layout on the GPU from the dense
        split (``Engine.set_split_dense``, k_panel.hip): CUDA tensors are read in place, host
        arrays are copied to the device once (large host splits are compacted on the host
        instead, ``HOST_COMPACT_BYTES``); nothing comes back to the host but the row count."""
        from .panel import prepare_split
        dev = torch.device("cuda", torch.cuda.current_device())
        for s, b in enumerate((train, valid, test)):
            if b is None:
                continue
            f0 = b["individual_features"]
            on_dev = isinstance(f0, torch.Tensor) and f0.is_cuda
            if not on_dev and int(np.prod(tuple(f0.shape))) * 4 > self.HOST_COMPACT_BYTES:
                ps = prepare_split(b, self.KP, fp32=self.fp32)
                self.eng.set_split(s, ps.X, ps.rowti, ps.row_ptr, ps.Rm, ps.mask, ps.macro.reshape(-1),
                                   int(ps.T), int(ps.N))
                self.splits[s] = SplitInfo(self.eng, s, int(ps.T), int(ps.N), int(self.eng.split_rows(s)))
                del ps
                continue
            feats = _on_device(b["individual_features"], torch.float32, dev)
            ret = _on_device(b["returns"], torch.float32, dev)
            mask = _on_device(b["mask"], torch.bool, dev)
            T, N, F = feats.shape
            macro, mptr = None, 0
            if self.spec.macro_dim > 0:
                macro = _on_device(b["macro_features"], torch.float32, dev)
                if tuple(macro.shape) != (T, self.spec.macro_dim):
                    raise ValueError(f"macro_features must be [{T}, {self.spec.macro_dim}], not {tuple(macro.shape)}")
                mptr = macro.data_ptr()
            self.eng.set_split_dense(s, feats.data_ptr(), ret.data_ptr(), mask.data_ptr(), True, mptr,
                                     int(T), int(N), int(F), torch.cuda.current_stream(dev).cuda_stream)
            self.splits[s] = SplitInfo(self.eng, s, int(T), int(N), int(self.eng.split_rows(s)))
            if not on_dev:              # the dense device copies were temporaries: release them
                del feats, ret, mask, macro
                torch.cuda.empty_cache()

    # ---- parameters -----------------------------------------------------------------
    def set_model(self, g: int, model, seed: int):
        self.eng.set_params(g, flatten_state(model, self.spec))
        self.eng.set_seed(g, int(seed) & 0xFFFFFFFF)

    def params(self, g: int, which: str = "current") -> np.ndarray:
        if which == "current":
            return self.eng.get_params(g)
        return self.eng.get_snapshot(g, 0 if which == "loss" else 1)

    def state_dict(self, g: int, which: str = "current") -> Dict[str, torch.Tensor]:
        return unflatten_state(self.params(g, which), self.spec)

    # ---- execution ------------------------------------------------------------------
    def run(self, phase: int, n: int, lr: float, ignore_epoch: int, selection_sign: float = 1.0,
            use_graph: bool = True):
        self.eng.run_epochs(phase, n, lr, ignore_epoch, selection_sign, use_graph)

    def history_rows(self, g: int) -> np.ndarray:
        return self.eng.history(g)

    def evaluate(self, s: int, device_weights: bool = False) -> List[Dict]:
        """Eval-mode forward of split ``s`` for every model: metrics of `src/train.py:106-153`.
        ``device_weights``: the L1-normalised weights stay on the GPU (a CUDA tensor, for the
        ensemble all-gather) instead of a host copy of every [T, N] array."""
        self.eng.forward_split(s, False, True)
        out = []
        ps = self.splits[s]
        dev = torch.device("cuda", torch.cuda.current_device())
        for g in range(self.G):
            sc = self.eng.read_ws(g, s, "scal")
            port = self.eng.read_ws(g, s, "port")
            lres = sc[SC["loss_res"]] * self.spec.residual_loss_factor
            sd_u = float(np.std(port, ddof=1)) if len(port) > 1 else float("nan")
            sh = 0.0 if sd_u < 1e-8 else float(np.mean(port) / sd_u)
            if device_weights:
                w = torch.empty(ps.T * ps.N, dtype=torch.float32, device=dev)
                ts = torch.cuda.current_stream(dev).cuda_stream
                self.eng.join_from(ts)                 # (w may reuse memory torch still reads)
                self.eng.copy_ws(g, s, "wn", w.data_ptr())
                self.eng.join_to(ts)
                w = w.view(ps.T, ps.N)
                wn = w / w.abs().sum(dim=1, keepdim=True).clamp_min(1e-8)
            else:
                w = self.eng.read_ws(g, s, "wn").reshape(ps.T, ps.N)
                l1 = np.abs(w).sum(axis=1, keepdims=True)
                wn = torch.from_numpy((w / np.maximum(l1, 1e-8)).astype(np.float32))
            out.append({
                "loss": float(sc[SC["loss_cond"]] + lres), "loss_unc": float(sc[SC["loss_unc"]]),
                "loss_cond": float(sc[SC["loss_cond"]]), "sharpe": sh,
                "max_drawdown": float(sc[SC["mdd"]]), "mean_return": float(np.mean(port)),
                "std_return": float(np.std(port)), "weights": wn,
                "portfolio_returns": port,
            })
        return out


def _hist_to_dict(rows: np.ndarray, has_test: bool) -> Dict[str, list]:
    keep = rows[rows[:, HIST["phase"]] != 2]
    h = {
        "train_loss": keep[:, HIST["train_loss"]].astype(np.float64).tolist(),
        "train_sharpe": keep[:, HIST["train_sharpe"]].astype(np.float64).tolist(),
        "valid_loss": keep[:, HIST["valid_loss"]].astype(np.float64).tolist(),
        "valid_sharpe": keep[:, HIST["valid_sharpe"]].astype(np.float64).tolist(),
        "test_loss": keep[:, HIST["test_loss"]].astype(np.float64).tolist() if has_test else [],
        "test_sharpe": keep[:, HIST["test_sharpe"]].astype(np.float64).tolist() if has_test else [],
        "phase": ["unc" if p == 1 else "cond" for p in keep[:, HIST["phase"]]],
    }
    return h


def _save_sd(eng: GANEngine, g: int, which: str, path: str, template):
    template.load_state_dict(eng.state_dict(g, which))
    torch.save(template.state_dict(), path)


def train_3phase_gpu(config, train_data, valid_data, test_data=None, device=None,
                     num_epochs_unc=256, num_epochs_moment=64, num_epochs=1024, lr=1e-3,
                     print_freq=128, save_dir=None, ignore_epoch=64, seed=None,
                     precision="bf16", selection_sign=1.0, verbose=True, n_models=1,
                     models=None, seeds=None, save_dirs=None, lrs=None, dropouts=None, resume=False,
                     resume_path=None, nan_policy="warn", stop_after=None, final_weights_device=False,
                     engine_setup=None, wait_fallback=True):
    """GPU executor of the 3-phase schedule; with ``n_models > 1`` trains an ensemble batch.

    Returns ``(model, history)`` for a single model, or ``(models, histories)`` when
    ``n_models > 1`` (``models``/``seeds``/``save_dirs`` give per-member inputs; ``lrs`` gives
    per-member learning rates, e.g. the lr axis of a hyperparameter sweep; ``dropouts`` per-member
    dropout rates, the sweep's dropout axis -- a member trains exactly as a solo run with its rate).

    Fault tolerance (additions, see ``utils``):
      resume_path -- where the resume record is written at every print boundary and phase end
                     (default ``save_dir/resume.pt`` for a single model with a ``save_dir``);
      resume      -- continue from an existing record at ``resume_path`` (bit-identical to an
                     uninterrupted run: parameters, Adam state, dropout stream and trackers);
      nan_policy  -- 'warn' | 'raise' | 'ignore' for non-finite losses / gradient norms,
                     checked at the print boundaries (``history['nonfinite_epoch']``);
      stop_after  -- (phase, epochs) : stop once that many epochs of that phase are done
                     (used to test interruption; the resume record is written first).
    ``final_weights_device``: the final evaluation's L1-normalised weights stay on the GPU
    (``engine_final_eval[s]["weights"]`` is then a CUDA tensor; the ensemble all-gathers them).
    ``engine_setup``: called with the ``GANEngine`` once data and parameters are set, before the
    first epoch (the cross-sectional sharding installs its collectives there, parallel/xsection.py).
    ``wait_fallback``: when an in-kernel spin wait gives up (a fused launch or the split epoch
    graphs could not make progress -- e.g. the GPU shared with other work), the models are restored
    to the start of that print interval and the interval is re-run in the engine's safe mode (no
    cross-launch waits; bitwise the same results), instead of stopping the run.
    """
    from ..models.gan import AssetPricingGAN
    from ..utils import checkpoint as ckpt
    from ..utils.guards import NonFiniteMonitor
    from ..utils.tracing import Timers, trace_range
    say = print if verbose else (lambda *a, **k: None)
    dev = torch.device(device) if device is not None else torch.device("cuda")
    if dev.index is not None:
        torch.cuda.set_device(dev)
    if models is None:
        models = [AssetPricingGAN(config) for _ in range(n_models)]
    n_models = len(models)
    if seeds is None:
        base = torch.initial_seed() if seed is None else seed
        seeds = [int(base) + 7919 * g for g in range(n_models)]
    seeds = [int(x) for x in seeds]
    if save_dirs is None:
        save_dirs = [save_dir] * n_models if n_models == 1 else [None] * n_models
    spec = models[0].spec
    n_sdf, n_mom = spec.param_counts()
    say(f"Model has {n_sdf + n_mom:,} trainable parameters")
    say(f"  SDF network: {n_sdf:,}")
    say(f"  Moment network: {n_mom:,}")
    total = num_epochs_unc + num_epochs_moment + num_epochs
    timers = Timers()
    with trace_range("engine-build", timers):
        eng = GANEngine(spec, n_models, max_epochs=max(total, 1), precision=precision)
    with trace_range("panel-compaction", timers):
        eng.set_data(train_data, valid_data, test_data)
    with trace_range("set-params", timers):
        for g, m in enumerate(models):
            eng.set_model(g, m, seeds[g])
            if lrs is not None:
                eng.eng.set_lr(g, float(lrs[g]))
            if dropouts is not None:
                eng.eng.set_dropout(g, float(dropouts[g]))
        if engine_setup is not None:
            engine_setup(eng)
        eng.eng.sync()
    template = AssetPricingGAN(config)
    t_start = time.time()
    best_state = [False] * n_models
    schedule = (num_epochs_unc, num_epochs_moment, num_epochs)
    if resume_path is None and n_models == 1 and save_dirs[0]:
        resume_path = os.path.join(save_dirs[0], ckpt.RESUME_FILE)
    monitor = NonFiniteMonitor(n_models, HIST, nan_policy)
    fallback = {"safe": False, "reruns": 0}
    start = (1, 0)                  # (phase, epochs done in it) to continue from
    run_fp = ckpt.run_fingerprint(lr, ignore_epoch, selection_sign,
                                  ckpt.data_fingerprint(train_data, valid_data, test_data)) if resume_path else None
    if resume and resume_path:
        rec = ckpt.load_resume(resume_path, spec, schedule, run=run_fp)
        if rec is not None:
            if len(rec["models"]) != n_models:
                raise ValueError(f"{resume_path}: {len(rec['models'])} models, expected {n_models}")
            for g, st in enumerate(rec["models"]):
                ckpt.restore_model(eng.eng, g, st)
                seeds[g] = int(st["seed"])
            best_state = list(rec["best_state"])
            start = (int(rec["phase"]), int(rec["done"]))
            t_start -= float(rec["elapsed"])
            say(f"Resumed from {resume_path}: phase {start[0]}, {start[1]} epochs done")

    def write_resume(phase, done):
        if not resume_path:
            return
        with trace_range("resume-checkpoint", timers):
            lr_of = (lambda g: lrs[g]) if lrs is not None else (lambda g: None)
            ckpt.save_resume(resume_path, spec=spec, phase=phase, done=done, schedule=schedule,
                             models=[ckpt.capture_model(eng.eng, g, seeds[g], lr_of(g)) for g in range(n_models)],
                             best_state=best_state, elapsed=time.time() - t_start, run=run_fp)

    class _Stop(Exception):
        pass

    def check_fused(e):
        if e.eng.prog_timeouts():
            raise RuntimeError("fused LSTM + tower forward: a spin wait gave up, so the run stopped updating "
                               "(the GPU is shared with other processes?); rerun with DLAP_RNN_OVERLAP=0")

    def run_phase(phase, n, title, tag):
        if phase < start[0]:
            return
        if verbose:
            print("\n" + "=" * 70 + f"\n{title}\nEpochs: {n}\n" + "=" * 70 + "\n")
        done = start[1] if phase == start[0] else 0
        eng.eng.plan_phase(phase, n)          # dense or Gram losses for this phase (cost model)
        if done == 0:
            eng.eng.begin_phase(phase)
        ep0 = eng.eng.epoch_count(0) - done
        marks = sorted({0} | set(range(print_freq - 1, n, print_freq)) | {n - 1}) if n > 0 else []
        if stop_after is not None and stop_after[0] == phase and 0 < stop_after[1] < n:
            marks = sorted(set(marks) | {stop_after[1] - 1})
        for mk in marks:
            k = mk + 1 - done
            if k <= 0:
                continue
            saved = None
            if wait_fallback and not fallback["safe"]:
                lr_of = (lambda g: lrs[g]) if lrs is not None else (lambda g: None)
                saved = [ckpt.capture_model(eng.eng, g, seeds[g], lr_of(g)) for g in range(n_models)]
            t0 = time.time()
            with trace_range(f"phase{phase}-epochs", timers):
                eng.run(phase, k, lr, ignore_epoch, selection_sign)
                eng.eng.sync()
            if saved is not None and eng.eng.prog_timeouts():
                # a spin wait gave up (its model is poisoned: no update, NaN epochs): back to the
                # interval's start, the rest of the run without cross-launch waits
                say(f"[engine] an in-kernel wait gave up in phase {phase}; re-running epochs "
                    f"{done + 1}-{mk + 1} in safe mode")
                eng.eng.reset_prog_errors()
                for g in range(n_models):
                    ckpt.restore_model(eng.eng, g, saved[g])
                eng.eng.set_safe_mode(True)
                fallback["safe"] = True
                fallback["reruns"] += 1
                with trace_range(f"phase{phase}-epochs", timers):
                    eng.run(phase, k, lr, ignore_epoch, selection_sign)
                    eng.eng.sync()
            dt = (time.time() - t0) / k
            done = mk + 1
            # first: a fused forward that gave up a wait poisons its model on the device (no
            # update, NaN epochs) -- report that cause, not the NaN it leaves in the history
            check_fused(eng)
            for g in range(n_models):
                monitor.check(g, eng.history_rows(g), raise_ok=n_models == 1)
            write_resume(phase, done)
            if stop_after is not None and tuple(stop_after) == (phase, done):
                raise _Stop()
            if verbose and ((mk + 1) % print_freq == 0 or mk == 0):
                r = eng.history_rows(0)[ep0 + mk]
                if phase == 2:
                    print(f"Epoch {mk + 1:4d}/{n} ({dt:.4f}s) | Conditional loss: {r[HIST['train_loss_cond']]:.6f}")
                else:
                    msg = (f"Epoch {mk + 1:4d}/{n} ({dt:.4f}s) | Train: loss={r[HIST['train_loss']]:.4f} "
                           f"sharpe={r[HIST['train_sharpe']]:.2f} | Valid: loss={r[HIST['valid_loss']]:.4f} "
                           f"sharpe={r[HIST['valid_sharpe']]:.2f}")
                    if test_data is not None:
                        msg += f" | Test sharpe={r[HIST['test_sharpe']]:.2f}"
                    print(msg)
        # checkpoint files (final state of the reference's per-improvement writes)
        for g in range(n_models):
            fl = eng.eng.snap_flags(g)
            if fl[1]:
                best_state[g] = True
            d = save_dirs[g]
            if d:
                if fl[0]:
                    _save_sd(eng, g, "loss", os.path.join(d, "best_model_loss.pt"), template)
                if fl[1]:
                    _save_sd(eng, g, "sharpe", os.path.join(d, "best_model_sharpe.pt"), template)

    try:
        run_phase(1, num_epochs_unc, "PHASE 1: Training Unconditional Loss (E[w*R]^2)", "unc")
        if start[0] <= 1:
            say("\nPhase 1 Complete!")
            if verbose:      # the device tracker holds sel * Sharpe (`src/train.py:287`)
                b1 = float(eng.eng.get_tracker_state(0)["best_sharpe"])
                say(f"Best validation Sharpe (phase 1): {selection_sign * b1:.4f}")
            for g in range(n_models):
                if best_state[g]:
                    eng.eng.load_snapshot(g, 1)
            if best_state[0]:
                say("Loaded best model from Phase 1")
            write_resume(2, 0)
        run_phase(2, num_epochs_moment, "PHASE 2: Updating Moment Conditions", "mom")
        if start[0] <= 2:
            say("\nPhase 2 Complete!")
            write_resume(3, 0)
        run_phase(3, num_epochs, "PHASE 3: Training Conditional Loss (E[h*w*R]^2)", "cond")
    except _Stop:
        say(f"Stopped after {tuple(stop_after)}; resume record at {resume_path}")
        train_3phase_gpu.last_engine = eng
        return None
    elapsed = time.time() - t_start
    for g in range(n_models):
        if best_state[g]:
            eng.eng.load_snapshot(g, 1)
    say("\n" + "=" * 70 + "\nTraining Complete!")
    say(f"Total time: {elapsed / 60:.1f} minutes")
    say(f"Total epochs: {total} ({num_epochs_unc} + {num_epochs_moment} + {num_epochs})\n" + "=" * 70)
    with trace_range("final-eval", timers):
        finals = {s: eng.evaluate(s, device_weights=final_weights_device) for s in eng.splits}
    check_fused(eng)
    if verbose:
        print("\nBest Model Performance (normalized weights):")
        for s, name in ((0, "Train"), (1, "Valid"), (2, "Test ")):
            if s in finals:
                f = finals[s][0]
                print(f"  {name} - Sharpe: {f['sharpe']:7.3f}, MaxDD: {f['max_drawdown']:7.2%}")
        print("=" * 70)
    out_models, hists = [], []
    for g in range(n_models):
        m = models[g]
        m.load_state_dict(eng.state_dict(g, "current"))
        m.to(dev)
        m.engine_final_eval = {s: finals[s][g] for s in finals}
        if save_dirs[g]:
            torch.save(m.state_dict(), os.path.join(save_dirs[g], "final_model.pt"))
        hists.append(_hist_to_dict(eng.history_rows(g), test_data is not None))
        out_models.append(m)
    train_3phase_gpu.last_engine = eng
    train_3phase_gpu.last_elapsed = elapsed
    train_3phase_gpu.last_timers = timers
    # host time of the graph captures (inside the first run of every phase's epoch ranges)
    train_3phase_gpu.last_capture_s = float(eng.eng.capture_seconds())
    train_3phase_gpu.last_nonfinite = monitor.nonfinite_models
    train_3phase_gpu.last_wait_fallback = dict(fallback)
    if n_models == 1:
        return out_models[0], hists[0]
    return out_models, hists
