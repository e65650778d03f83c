"""Cross-sectional (N-) sharded training: one model, its panel split over the stocks of N ranks.

SURVEY.md §5.7 (the "context parallel" analogue of this workload). Every BASELINE panel fits in
one MI355X's 288 GB, so the single-GPU engine is the production path; this mode exists for
panels beyond one GPU (or beyond one host's RAM when every rank reads only its own stocks).

Decomposition (reference math: `/root/reference/src/model.py:271-279` zero-mean weights,
`:346-433` unconditional / conditional losses, `:435-483` residual loss, `:565-594` L1
normalisation; `/root/reference/src/train.py:45-153` step and evaluation):

  * parameters, the macro series and the LSTM state [T, H] are replicated;
  * each rank runs both towers on its own stocks [T, N_r, F];
  * every cross-sectional sum is a [T]-vector all-reduce: (Σ w·m, N_t) for the zero mean,
    Σ w·R·m for P_t, (Σ w², Σ R·w, Σ R²) for the residual loss, Σ |w|·m for the L1 norm;
  * E_{k,i} (a sum over t) is rank-local; the loss needs one all-reduce of Σ_i E²_{k,i} [K].

Gradients: every rank evaluates the same global loss L from the all-reduced sums and
back-propagates L / world; the all-reduce's backward is itself an all-reduce (sum), so each rank
gets dL/d(its local partial sums), and one flat all-reduce of the parameter gradients completes
dL/dθ = Σ_r (local paths). The replicated clip + Adam then keep the replicas bit-identical.

Collectives per training step: 3 forward ([2,T], [2,T], [K]; +[4,T] with a residual loss), their 3 backward mirrors and one
flat gradient all-reduce (~12k floats) — all latency-bound, a few µs each over xGMI.

Two executors:

* ``train_3phase_xsection_engine`` (GPU production path, ``XSEngine``): the WHOLE epoch runs in
  the native engine of each rank -- towers, loss passes, tower backward, BPTT, clip + Adam, the
  evaluations and the bookkeeping -- and the engine calls back at each cross-sectional coupling
  so the rank-local sums are all-reduced on the engine stream, one collective per coupling.
  Phases 1 / 3 use the Gram-form losses, so a training epoch exchanges only the period sums
  ([T] + [3T] per split) and one packed gradient vector; the Gram matrices are all-reduced once
  per moment refresh.
* ``train_3phase_xsection`` (any device): the CPU trainer's loop over ``XSectionGAN``, whose local
  towers run on the native engine (``EngineTowers``) or as PyTorch ops, with the cross-sectional
  remainder (zero mean, P_t, E, losses: [T]- and [N_r, K]-sized tensors) in torch around the
  all-reduces. Autograd enters the engine at two points -- the raw SDF weights w[t, i] and the
  moment sums E[k, i] = Σ_t h q / T_i -- and leaves through ``Engine.xs_backward``, which
  recomputes the rank's forward and runs the engine's tower backward from the external dL/dw or
  (dL/dE, global SDF_t). On CPU (or ``engine=False``) the towers are PyTorch ops.
"""
from __future__ import annotations

import argparse
import contextlib
import io
import json
import time
from typing import Dict, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as tdist

from ..models import losses as L
from ..models.gan import AssetPricingGAN
from ..train.metrics import compute_max_drawdown, compute_sharpe
from . import comm

SPLITS = ("train", "valid", "test")


class _AllReduceSum(torch.autograd.Function):
    """y = Σ_ranks x on every rank; backward: dx = Σ_ranks dy (every rank's loss uses y)."""

    @staticmethod
    def forward(ctx, x):
        y = x.clone()
        tdist.all_reduce(y)
        return y

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous().clone()
        tdist.all_reduce(g)
        return g


def all_reduce_sum(x: torch.Tensor, d: comm.Dist) -> torch.Tensor:
    if not d.active:
        return x
    return _AllReduceSum.apply(x)


def shard_bounds(n: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous stock range [a, b) of ``rank`` (sizes differ by at most one)."""
    q, r = divmod(n, world)
    a = rank * q + min(rank, r)
    return a, a + q + (1 if rank < r else 0)


def shard_batch(batch: Dict, rank: int, world: int) -> Dict:
    """The rank's stocks of a split dict ([T, N, ...] tensors sliced on N; macro replicated)."""
    n = batch["returns"].shape[1]
    a, b = shard_bounds(n, rank, world)
    out = {k: (v if k == "macro_features" or v is None else v[:, a:b].contiguous()) for k, v in batch.items()}
    out["n_total"] = n
    return out


def _mkey(t: torch.Tensor):
    return (t.data_ptr(), tuple(t.shape), t._version)


class EngineTowers:
    """The rank's local towers on the native engine (one model, the rank's shards of the
    train / valid / test splits). Reference modules: `SDFNetwork` / `MomentNetwork` /
    `MacroLSTM` (`/root/reference/src/model.py:21-279`)."""

    def __init__(self, model: AssetPricingGAN, shards: Sequence[Optional[Dict]], device,
                 seed: int = 0, precision: str = "bf16", tower_salt: int = 0):
        from ..engine.runner import GANEngine
        self.device = torch.device(device)
        self.spec = model.spec
        self.eng = GANEngine(model.spec, 1, max_epochs=8, precision=precision)
        dev = [None if b is None else {k: (v.to(self.device) if isinstance(v, torch.Tensor) else v)
                                       for k, v in b.items() if k != "n_total"} for b in shards]
        self.eng.set_data(*dev)
        # the same seed on every rank: the replicated LSTM draws identical inter-layer masks; the
        # towers' dropout is salted per rank so local stock i of two shards gets independent masks
        # (the reference draws an independent Bernoulli mask for every (t, stock))
        self.eng.eng.set_seed(0, int(seed) & 0xFFFFFFFF)
        self.eng.eng.set_tower_salt(0, int(tower_salt) & 0xFFFFFFFF)
        self.masks = {}
        for s, b in enumerate(dev):
            if b is not None:
                m = b["mask"].bool()
                self.masks[s] = m
        self.keys = {}
        self.param_key = None
        self.step = 0
        self._flat = None
        self._h = {}

    def register(self, s: int, mask: torch.Tensor):
        self.keys[_mkey(mask)] = s

    def split_of(self, mask: torch.Tensor) -> int:
        s = self.keys.get(_mkey(mask))
        if s is None:
            for k, m in self.masks.items():      # same tensor values as a registered split
                if m.shape == mask.shape and bool(torch.equal(m, mask.bool())):
                    self.keys[_mkey(mask)] = s = k
                    break
        if s is None:
            raise KeyError("EngineTowers: this shard is not one of the engine's splits")
        return s

    def _ts(self) -> int:
        return torch.cuda.current_stream(self.device).cuda_stream

    def sync_params(self, params: Sequence[torch.Tensor], training: bool):
        from ..ops.fused import _ParamKey, _flat_params
        params = list(params)
        fresh = self.param_key is None or not self.param_key.matches(params)
        if fresh:
            self._flat = _flat_params(params, self.device).contiguous()
        ts = self._ts()
        self.eng.eng.join_from(ts)
        if fresh:
            self.eng.eng.set_params_dev(0, self._flat.data_ptr())
            self.param_key = _ParamKey(params)
        if training:
            self.step += 1
            self.eng.eng.set_drop_step(0, self.step)
        return ts

    def forward(self, s: int, training: bool, do_mom: bool):
        """Raw SDF weights [T, N_r] (zero where masked) and moments [K, T, N_r] of split s."""
        ts = self._ts()
        self.eng.eng.forward_split(s, bool(training), bool(do_mom), False)
        m = self.masks[s]
        R = int(self.eng.eng.split_rows(s))
        wc = torch.empty(max(R, 1), dtype=torch.float32, device=self.device)
        self.eng.eng.copy_ws(0, s, "w", wc.data_ptr())
        h = None
        if do_mom:
            T, N = m.shape
            h = torch.empty(T * N * self.spec.num_moments, dtype=torch.float32, device=self.device)
            self.eng.eng.copy_ws(0, s, "h", h.data_ptr())
        self.eng.eng.join_to(ts)
        w = torch.zeros(m.shape, dtype=torch.float32, device=self.device)
        w[m] = wc[:R]
        if h is not None:
            h = h.reshape(m.shape[0], m.shape[1], -1).permute(2, 0, 1)
        return w, h

    def backward(self, phase: int, dw: Optional[torch.Tensor] = None, dE: Optional[torch.Tensor] = None,
                 sdf: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Flat parameter gradient of the train split from external dL/dw [T, N_r] (phases 1 / 3)
        or dL/dE [K, N_r] with the global SDF_t (phase 2)."""
        P = sum(int(n) for n in self.spec.param_counts())
        out = torch.empty(P, dtype=torch.float32, device=self.device)
        ts = self._ts()
        if phase == 2:
            dEc = dE.detach().t().contiguous().float()          # engine layout [N][K]
            sdfc = sdf.detach().contiguous().float()
            self.eng.eng.join_from(ts)
            self.eng.eng.xs_backward(2, 0, dEc.data_ptr(), sdfc.data_ptr())
        else:
            dwc = dw.detach()[self.masks[0]].contiguous().float()
            if dwc.numel() == 0:
                dwc = torch.zeros(1, device=self.device)
            self.eng.eng.join_from(ts)
            self.eng.eng.xs_backward(phase, dwc.data_ptr(), 0, 0)
        self.eng.eng.copy_grads(0, out.data_ptr())
        self.eng.eng.join_to(ts)
        return out


class _TowerSDF(torch.autograd.Function):
    """w_raw [T, N_r] (computed by the engine, passed in as ``w``) as a function of the SDF-side
    parameters (``params``, flat-layout order); backward: ``Engine.xs_backward`` phase 1."""

    @staticmethod
    def forward(ctx, et, s, w, *params):
        ctx.et, ctx.s = et, s
        ctx.shapes = [p.shape for p in params]
        return w.clone()

    @staticmethod
    def backward(ctx, g):
        if ctx.s != 0:
            raise RuntimeError("engine towers: gradients only for the train split")
        flat = ctx.et.backward(1, dw=g)
        P_sdf = ctx.et.spec.param_counts()[0]
        return (None, None, None, *_split_like(flat[:P_sdf], ctx.shapes))


class _TowerE(torch.autograd.Function):
    """E [K, N_r] = Σ_t h q / T_i with q = R m SDF_t and h the engine's moments (``h``, computed
    outside); differentiable w.r.t. SDF_t (in torch) and the moment parameters (``params``,
    through ``Engine.xs_backward`` phase 2 when ``want`` is set)."""

    @staticmethod
    def forward(ctx, et, want, h, r, m, t_i, sdf, *params):
        ctx.et, ctx.want = et, want
        ctx.shapes = [p.shape for p in params]
        ctx.save_for_backward(h, r, m, t_i, sdf)
        q = r * m * sdf[:, None]
        return (h * q[None]).sum(1) / t_i

    @staticmethod
    def backward(ctx, de):
        h, r, m, t_i, sdf = ctx.saved_tensors
        g = de / t_i                                            # [K, N_r]
        dsdf = (torch.einsum("ki,kti->ti", g, h) * r * m).sum(1)
        grads = [None] * len(ctx.shapes)
        if ctx.want:
            flat = ctx.et.backward(2, dE=de, sdf=sdf)
            P_sdf = ctx.et.spec.param_counts()[0]
            grads = _split_like(flat[P_sdf:], ctx.shapes)
        return (None, None, None, None, None, None, dsdf, *grads)


def _split_like(flat: torch.Tensor, shapes):
    out, off = [], 0
    for shp in shapes:
        n = int(np.prod(shp)) if len(shp) else 1
        out.append(flat[off:off + n].reshape(shp))
        off += n
    return out


class XSectionGAN(AssetPricingGAN):
    """``AssetPricingGAN`` whose forward / get_weights take the rank's stock shard and return
    the GLOBAL losses, portfolio returns and Sharpe (weights and moments stay local).
    State-dict keys and initialisation equal ``AssetPricingGAN`` (it is a subclass)."""

    def __init__(self, config: Dict, dist: comm.Dist, lstm_seed: int = 0):
        super().__init__(config)
        self.dist = dist
        self.lstm_seed = int(lstm_seed)
        self._lstm_calls = 0
        self.et: Optional[EngineTowers] = None

    def attach_engine(self, shards: Sequence[Optional[Dict]], device, precision: str = "bf16") -> "XSectionGAN":
        """Run the local towers on the native engine (``shards``: this rank's train / valid /
        test dicts, as passed to train_epoch / evaluate)."""
        self.et = EngineTowers(self, shards, device, seed=self.lstm_seed, precision=precision,
                               tower_salt=self.dist.rank + 1 if self.dist.active else 0)
        return self

    def _engine_pass(self, mask, want_mom: bool):
        from ..ops.fused import _ordered_params
        et = self.et
        s = et.split_of(mask)
        params = _ordered_params(self)
        n_sdf = sum(1 for k, _ in self.spec.param_layout() if k.startswith("sdf_net."))
        et.sync_params(params, self.training)
        w, h = et.forward(s, self.training, want_mom)
        if torch.is_grad_enabled() and s == 0:
            w = _TowerSDF.apply(et, s, w, *params[:n_sdf])
        return s, w, h, params[n_sdf:]

    def _global_n(self, returns) -> int:
        """Total stocks over all ranks for a local width N_r: one all-reduce (and host read) per
        distinct local width, cached -- a training loop's forwards issue no host sync for it."""
        n_loc = int(returns.shape[1])
        if not self.dist.active:
            return n_loc
        cache = self.__dict__.setdefault("_n_total", {})
        if n_loc not in cache:
            cache[n_loc] = int(all_reduce_sum(torch.tensor([float(n_loc)], device=returns.device),
                                              self.dist).item())
        return cache[n_loc]

    def _normalize(self, w_raw, mask):
        m = mask.float()
        w = w_raw * m
        if not self.sdf_net.normalize_weights:
            return w
        s = all_reduce_sum(torch.stack([(w * m).sum(1), m.sum(1)]), self.dist)
        mu = s[0] / s[1].clamp(min=1)
        return (w - mu[:, None]) * m

    # -- local pieces --------------------------------------------------------------------------
    def _macro_state(self, macro):
        lstm = self.sdf_net.macro_lstm
        if macro is None or lstm is None:
            return macro
        if self.training and lstm.num_layers > 1 and lstm.lstm.dropout > 0:
            # inter-layer LSTM dropout must draw the same mask on every rank
            self._lstm_calls += 1
            devs = [macro.device] if macro.is_cuda else []
            with torch.random.fork_rng(devices=devs):
                torch.manual_seed(self.lstm_seed * 1000003 + self._lstm_calls)
                return lstm(macro)[0]
        return lstm(macro)[0]

    def raw_weights(self, macro, x):
        T, n, _ = x.shape
        state = self._macro_state(macro)
        inp = x if state is None else torch.cat([x, state[:, None, :].expand(T, n, state.shape[-1])], -1)
        return self.sdf_net.output_proj(self.sdf_net.fc_layers(inp.reshape(T * n, -1))).reshape(T, n)

    def shard_weights(self, macro, x, mask):
        """Zero-mean (over ALL ranks' valid stocks) weights of the local stocks."""
        if self.et is not None:
            return self._normalize(self._engine_pass(mask, False)[1], mask)
        return self._normalize(self.raw_weights(macro, x), mask)

    # -- global losses -------------------------------------------------------------------------
    def _portfolio(self, w, r, m):
        s = all_reduce_sum(torch.stack([(w * r * m).sum(1), m.sum(1)]), self.dist)
        if not self.weighted_loss:
            return s[0]
        n_t = s[1].clamp(min=1)
        return s[0] / n_t * n_t.mean()

    def _moment_loss(self, h, r, m, sdf, n_total, engine=None):
        t_i = m.sum(0).clamp(min=1)
        if engine is not None:        # (et, want moment-parameter gradients, moment params)
            et, want, mparams = engine
            e = _TowerE.apply(et, want, h, r, m, t_i, sdf, *mparams)
        else:
            q = r * m * sdf[:, None]
            e = (q.sum(0) / t_i)[None] if h is None else (h * q[None]).sum(1) / t_i     # [K, N_r]
        return all_reduce_sum((e ** 2).sum(1), self.dist).mean() / n_total

    def _residual(self, w, r, m):
        s = all_reduce_sum(torch.stack([m.sum(1), (w * w * m).sum(1), (r * w * m).sum(1),
                                        (r * r * m).sum(1)]), self.dist)
        n, ww, rw, rr = s
        use = n >= 2
        has = use & (ww > 1e-8)
        beta = torch.where(has, rw / torch.where(has, ww, torch.ones_like(ww)), torch.zeros_like(ww))
        nc = n.clamp(min=1)
        resid = (rr - 2 * beta * rw + beta * beta * ww) / nc
        rsq = rr / nc
        # (no host sync: without a usable period both masked numerators are 0 -> loss 0)
        resid_mean = (resid * has.float()).sum() / has.float().sum().clamp(min=1)
        rsq_mean = (rsq * use.float()).sum() / use.float().sum().clamp(min=1)
        return resid_mean / rsq_mean.clamp(min=1e-8)

    def forward(self, macro_features, individual_features, returns, mask, hidden=None,
                phase: str = "conditional", n_total: Optional[int] = None) -> Dict[str, torch.Tensor]:
        """Same dict as ``AssetPricingGAN.forward`` (`model.py:485-563`): loss, losses, sharpe
        and portfolio returns are global; weights [T, N_r] and moments [K, T, N_r] local."""
        if n_total is None:
            n_total = self._global_n(returns)
        m = mask.float()
        eng = None
        if self.et is not None:
            # engine towers; the moment network's output only enters the losses through E
            s_, w_raw, moments, mparams = self._engine_pass(mask, phase != "unconditional")
            w = self._normalize(w_raw, mask)
            if moments is not None:
                eng = (self.et, torch.is_grad_enabled() and s_ == 0 and phase == "moment", mparams)
        else:
            w = self.shard_weights(macro_features, individual_features, mask)
            moments = self.moment_net(self._moment_input(macro_features, individual_features))
        p = self._portfolio(w, returns, m)
        zero = torch.zeros((), device=w.device)
        if phase == "unconditional":
            loss_unc = self._moment_loss(None, returns, m, p + 1.0, n_total)
            loss_cond, total = zero, loss_unc
        elif phase == "moment":
            loss_cond = self._moment_loss(moments, returns, m, p + 1.0, n_total, eng)
            loss_unc, total = zero, -loss_cond
        else:
            loss_cond = self._moment_loss(moments, returns, m, p + 1.0, n_total, eng)
            loss_unc = self._moment_loss(None, returns, m, p + 1.0, n_total)
            total = loss_cond
        loss_res = zero
        if self.residual_loss_factor > 0:
            loss_res = self._residual(w, returns, m)
            total = total + self.residual_loss_factor * loss_res
        return {"weights": w, "loss": total, "loss_unconditional": loss_unc,
                "loss_conditional": loss_cond, "loss_residual": loss_res,
                "sharpe": L.sharpe_monitor(p), "portfolio_returns": p, "hidden": None,
                "moments": moments}

    def get_weights(self, macro_features, individual_features, mask, hidden=None,
                    normalized: bool = False):
        w = self.shard_weights(macro_features, individual_features, mask)
        if normalized:
            s = all_reduce_sum((w.abs() * mask.float()).sum(1), self.dist).clamp(min=1e-8)
            w = w / s[:, None]
        return w, None


class _Bundle:
    """Device scalars of one epoch read back to the host in ONE transfer. ``train_epoch`` and
    ``evaluate`` register their results (valid / test evaluations follow the step without a host
    read in between) and return ``_Deferred`` mappings; the first key access of any of them copies
    every pending tensor at once (the step and the two evaluations used to
    cost a device-to-host read each)."""
    pending: list = []

    @classmethod
    def add(cls, vec: torch.Tensor, post) -> "_Deferred":
        d = _Deferred(vec.detach().float().reshape(-1), post)
        cls.pending.append(d)
        return d

    @classmethod
    def flush(cls):
        todo, cls.pending = cls.pending, []
        live = [d for d in todo if d._vals is None]
        if not live:
            return
        host = torch.cat([d._vec for d in live]).cpu().numpy()
        off = 0
        for d in live:
            n = d._vec.numel()
            d._vals = d._post(host[off:off + n])
            d._vec = None
            off += n


class _Deferred(dict):
    """A result dict whose scalar entries arrive with the epoch's bundle read; device tensors
    (``weights``) are available at once."""

    def __init__(self, vec, post, **eager):
        super().__init__(**eager)
        self._vec, self._post, self._vals = vec, post, None

    def _ready(self):
        if self._vals is None:
            _Bundle.flush()
        if self._vals is not None and not self._merged:
            super().update(self._vals)
            self._merged = True

    _merged = False

    def __getitem__(self, k):
        if not dict.__contains__(self, k):
            self._ready()
        return super().__getitem__(k)

    def get(self, k, default=None):
        try:
            return self[k]
        except KeyError:
            return default

    def __contains__(self, k):
        self._ready()
        return super().__contains__(k)

    def keys(self):
        self._ready()
        return super().keys()

    def items(self):
        self._ready()
        return super().items()

    def values(self):
        self._ready()
        return super().values()

    def __iter__(self):            # (also keeps {**d} / dict(d) off the raw-storage fast path)
        self._ready()
        return super().__iter__()

    def __len__(self):
        self._ready()
        return super().__len__()

    def __repr__(self):
        self._ready()
        return super().__repr__()


def _args(data: Dict, device):
    macro = data.get("macro_features")
    return (None if macro is None else macro.to(device), data["individual_features"].to(device),
            data["returns"].to(device), data["mask"].to(device))


def train_epoch(model: XSectionGAN, optimizer, data: Dict, device, phase: str = "conditional",
                grad_clip: float = 1.0, scope: str = "all") -> Dict:
    """One full-batch step over the sharded panel (`/root/reference/src/train.py:45-103`)."""
    d = model.dist
    model.train()
    macro, x, r, m = _args(data, device)
    optimizer.zero_grad()
    out = model(macro, x, r, m, phase=phase, n_total=data.get("n_total"))
    (out["loss"] / d.world).backward()
    params = list({"sdf": model.sdf_net.parameters, "moment": model.moment_net.parameters}.get(
        scope, model.parameters)())
    grads = [p.grad for p in params if p.grad is not None]
    if d.active and grads:
        flat = torch.cat([g.reshape(-1) for g in grads])          # one collective for all params
        tdist.all_reduce(flat)
        off = 0
        for g in grads:
            g.copy_(flat[off:off + g.numel()].view_as(g))
            off += g.numel()
    gn = torch.nn.utils.clip_grad_norm_(params, max_norm=grad_clip)
    optimizer.step()
    # the six scalars stay on the device until the epoch's bundle is read (no host sync here;
    # the reference: six .item() syncs per step)
    dev = out["loss"].device
    p = out["portfolio_returns"].detach().float()
    sd = p.std()
    sharpe = torch.where(sd < 1e-8, torch.zeros_like(sd), p.mean() / sd)
    v = torch.stack([out["loss"].detach().float().reshape(()), out["loss_unconditional"].detach().float().reshape(()),
                     out["loss_conditional"].detach().float().reshape(()),
                     out["loss_residual"].detach().float().reshape(()), sharpe,
                     torch.as_tensor(gn, device=dev).detach().float().reshape(())])
    keys = ("loss", "loss_unc", "loss_cond", "loss_residual", "sharpe", "grad_norm")
    return _Bundle.add(v, lambda h: {k: float(x) for k, x in zip(keys, h)})


@torch.no_grad()
def evaluate(model: XSectionGAN, data: Dict, device, normalized: bool = True) -> Dict:
    """Global evaluation metrics from the rank's shard (`/root/reference/src/train.py:106-153`);
    ``weights`` are the rank's stocks."""
    model.eval()
    macro, x, r, m = _args(data, device)
    w, _ = model.get_weights(macro, x, m, normalized=normalized)
    pr = all_reduce_sum((w * r * m.float()).sum(1), model.dist)
    out = model(macro, x, r, m, phase="conditional", n_total=data.get("n_total"))
    # portfolio returns and the three losses join the epoch's bundle read (train_epoch)
    v = torch.cat([pr.float(), torch.stack([out["loss"].float().reshape(()),
                                            out["loss_unconditional"].float().reshape(()),
                                            out["loss_conditional"].float().reshape(())])])

    def post(h):
        port = np.asarray(h[:-3], dtype=np.float32)
        return {"loss": float(h[-3]), "loss_unc": float(h[-2]), "loss_cond": float(h[-1]),
                "sharpe": compute_sharpe(torch.from_numpy(port)), "max_drawdown": compute_max_drawdown(port),
                "mean_return": port.mean(), "std_return": port.std()}
    d = _Bundle.add(v, post)
    dict.__setitem__(d, "weights", w)                    # (the rank's stocks, on its device)
    return d


def train_3phase_xsection(config: Dict, train_data: Dict, valid_data: Dict, test_data: Optional[Dict],
                          dist: comm.Dist, device=None, num_epochs_unc: int = 256,
                          num_epochs_moment: int = 64, num_epochs: int = 1024, lr: float = 1e-3,
                          print_freq: int = 128, save_dir: Optional[str] = None, ignore_epoch: int = 64,
                          seed: int = 42, selection_sign: float = 1.0, verbose: bool = True,
                          nan_policy: str = "warn", engine: Optional[bool] = None, precision: str = "bf16"):
    """``train_3phase`` over stock shards (``*_data``: FULL split dicts or already-sharded ones
    carrying ``n_total``). Same schedule, trackers and checkpoints as the CPU trainer; rank 0
    writes the checkpoints. Returns ``(model, history)`` on every rank.
    ``engine`` (default: on a GPU) runs the local towers on the native engine."""
    from ..train.trainer import _train_3phase_cpu
    device = torch.device(device or dist.device)
    sh = [None if b is None else (b if "n_total" in b else shard_batch(b, dist.rank, dist.world))
          for b in (train_data, valid_data, test_data)]
    use_engine = device.type == "cuda" if engine is None else bool(engine)
    if use_engine:       # shards resident on the device once (the engine keys its splits by them)
        sh = [None if b is None else {k: (v.to(device) if isinstance(v, torch.Tensor) else v) for k, v in b.items()}
              for b in sh]
    torch.manual_seed(seed)                      # identical initial parameters on every rank
    model = XSectionGAN(config, dist, lstm_seed=seed).to(device)
    if use_engine:
        model.attach_engine(sh, device, precision=precision)
        for s_, b in enumerate(sh):
            if b is not None:
                model.et.register(s_, b["mask"])
    torch.manual_seed(seed + 7919 * (dist.rank + 1))   # per-rank dropout streams of the local rows
    main = dist.rank == 0
    # every rank runs the same (collective) evaluations, including the verbose final report;
    # only rank 0's output is shown
    quiet = contextlib.redirect_stdout(io.StringIO()) if not main else contextlib.nullcontext()
    with quiet:
        return _train_3phase_cpu(config, sh[0], sh[1], sh[2], device, num_epochs_unc, num_epochs_moment,
                                 num_epochs, lr, print_freq, save_dir if main else None, ignore_epoch,
                                 selection_sign, verbose, nan_policy=nan_policy,
                                 model=model, train_fn=train_epoch, eval_fn=evaluate)


class _DevView:
    """A typed 1-D view of engine device memory (``torch.as_tensor`` reads the interface)."""

    def __init__(self, ptr: int, n: int, typestr: str):
        self.__cuda_array_interface__ = {"shape": (int(n),), "typestr": typestr, "data": (int(ptr), False),
                                         "version": 2}


class XSEngine:
    """Cross-sectional sharding INSIDE the native epoch engine: every rank's ``Engine`` holds the
    rank's stocks of the three splits and runs the whole epoch itself (towers, losses, backward,
    BPTT, Adam); at each cross-sectional coupling it calls back (``Engine.set_xs``) and the
    rank-local sums are all-reduced on the engine stream, one collective per coupling:

      sums1  [T]  Σ w of every period (the zero mean),             per split, before the P pass
      sums2  [3T] Σ w'R, Σ |w'|, Σ w'^2 (P_t, the L1 portfolio, the residual loss)
      gram   [2T²] fp64 Gram matrices (once per moment refresh: the phase-1/3 losses and dL/dSDF_t
             are quadratic forms of them, so a training epoch needs NO loss all-reduce)
      loss   [2]  the dense asset passes' loss sums (phase 2, dense evaluations)
      grads  [P + T Dm (+ 64 T)] the flat gradient and the per-period input gradients of the
             replicated LSTM, after the tower backward -- the only backward collective.

    Reference math: `/root/reference/src/model.py:271-279` (zero mean), `:346-433` (losses);
    the per-period constants N_t, mean R, Σ R², N̄ and the loss normaliser N are the global ones
    (``Engine.xs_set_globals``). Replicated parameters stay bit-identical (every rank applies the
    same summed gradient). With one rank the callbacks return at once."""

    def __init__(self, eng, shards: Sequence[Optional[Dict]], dist: comm.Dist):
        self.ge, self.d = eng, dist
        self.dev = torch.device("cuda", torch.cuda.current_device())
        self.T = {s: int(b["returns"].shape[0]) for s, b in enumerate(shards) if b is not None}
        self._views: Dict = {}
        self._streams: Dict[int, torch.cuda.ExternalStream] = {}
        self.n_calls = 0
        if self.d.active:
            for s, b in enumerate(shards):
                if b is not None:
                    self._set_globals(s, b)
        self.ge.eng.set_xs(self._hook)

    def _set_globals(self, s: int, b: Dict):
        m = b["mask"].to(self.dev).bool()
        r = torch.where(m, b["returns"].to(self.dev, torch.float64), torch.zeros((), dtype=torch.float64,
                                                                                 device=self.dev))
        st = torch.stack([m.sum(1).double(), r.sum(1), (r * r).sum(1)])        # [3, T]
        tdist.all_reduce(st)
        nc = st[0].clamp_min(1.0)
        Nt, invNt = st[0].float().contiguous(), (1.0 / nc).float().contiguous()
        meanR, RR = (st[1] / nc).float().contiguous(), st[2].float().contiguous()
        nbar = float(nc.mean()) if nc.numel() else 1.0
        n_total = int(b["n_total"]) if "n_total" in b else self._sum_int(m.shape[1])
        ts = torch.cuda.current_stream(self.dev).cuda_stream
        self.ge.eng.join_from(ts)
        self.ge.eng.xs_set_globals(s, Nt.data_ptr(), invNt.data_ptr(), meanR.data_ptr(), RR.data_ptr(),
                                   nbar, float(n_total))
        self.ge.eng.sync()                          # (the temporaries are read)

    def _sum_int(self, v: int) -> int:
        t = torch.tensor([float(v)], dtype=torch.float64, device=self.dev)
        tdist.all_reduce(t)
        return int(t.item())

    def _view(self, key, ptr: int, n: int, typestr: str) -> torch.Tensor:
        v = self._views.get(key)
        if v is None or v[0] != ptr:
            v = (ptr, torch.as_tensor(_DevView(ptr, n, typestr), device=self.dev))
            self._views[key] = v
        return v[1]

    def _ws(self, s: int, name: str, typestr: str = "<f4") -> torch.Tensor:
        ptr, n = self.ge.eng.ws_ptr(0, s, name)
        return self._view((s, name), ptr, n, typestr)

    def _bufs(self, what: str, which: int) -> list:
        splits = [s for s in sorted(self.T) if which & (1 << s)]
        if what == "grads":
            ptr, n = self.ge.eng.grads_ptr(0)
            out = [self._view("grads", ptr, n, "<f4"), self._ws(0, "dpp")]
            if which == 2:
                out.append(self._ws(0, "dab"))
            return out
        if what == "gram":
            return [self._ws(s, "gram", "<f8") for s in splits]
        rows = {"sums1": (0, 1), "sums2": (1, 4)}
        out = []
        for s in splits:
            T, xs = self.T[s], self._ws(s, "xs")
            if what == "loss":
                out.append(xs[4 * T:4 * T + 2])
            else:
                a, b = rows[what]
                out.append(xs[a * T:b * T])
        return out

    def _hook(self, what: str, which: int, stream: int):
        self.n_calls += 1
        if not self.d.active:
            return
        bufs = [b for b in self._bufs(what, which) if b.numel()]
        st = self._streams.get(stream)
        if st is None:
            st = self._streams[stream] = torch.cuda.ExternalStream(stream, device=self.dev)
        with torch.cuda.stream(st):
            if len(bufs) == 1:
                tdist.all_reduce(bufs[0])
                return
            flat = torch.cat([b.reshape(-1) for b in bufs])      # one collective per coupling
            tdist.all_reduce(flat)
            o = 0
            for b in bufs:
                b.copy_(flat[o:o + b.numel()])
                o += b.numel()


def train_3phase_xsection_engine(config: Dict, train_data: Dict, valid_data: Dict, test_data: Optional[Dict],
                                 dist: comm.Dist, device=None, seed: int = 42, verbose: bool = True,
                                 save_dir: Optional[str] = None, **kw):
    """``train_3phase`` over stock shards with the whole epoch on the native engine (``XSEngine``).
    ``*_data``: FULL split dicts or this rank's shards (carrying ``n_total``). Returns
    ``(model, history)`` on every rank; ``model.engine_final_eval[s]`` holds the GLOBAL metrics
    (the weights are the rank's stocks). ``kw``: the schedule / optimiser arguments of
    ``engine.runner.train_3phase_gpu``."""
    from ..engine.runner import train_3phase_gpu
    device = torch.device(device or dist.device)
    sh = [None if b is None else (b if "n_total" in b else shard_batch(b, dist.rank, dist.world))
          for b in (train_data, valid_data, test_data)]
    sh = [None if b is None else {k: (v.to(device) if isinstance(v, torch.Tensor) else v) for k, v in b.items()}
          for b in sh]
    torch.manual_seed(seed)                      # identical initial parameters on every rank
    model = AssetPricingGAN(config)
    salt = dist.rank + 1 if dist.active else 0
    holder = {}

    def setup(eng):
        eng.eng.set_tower_salt(0, salt)          # independent tower dropout masks per rank
        holder["xs"] = XSEngine(eng, sh, dist)

    main = dist.rank == 0
    quiet = contextlib.redirect_stdout(io.StringIO()) if not main else contextlib.nullcontext()
    with quiet:
        out = train_3phase_gpu(config, *[None if b is None else {k: v for k, v in b.items() if k != "n_total"}
                                         for b in sh],
                               device=device, seed=seed, models=[model], seeds=[seed], verbose=verbose and main,
                               save_dir=save_dir if main else None, engine_setup=setup, **kw)
    train_3phase_xsection_engine.last_xs = holder.get("xs")
    return out


def load_shards(args, d: comm.Dist) -> Dict[str, Dict]:
    """Each rank's stocks of every split: from ``--data_dir`` (each rank reads the files and keeps
    its slice) or a ``--synthetic`` panel generated identically on every rank."""
    from .ensemble import _load_batches
    full = _load_batches(args)
    return {k: shard_batch(full[k], d.rank, d.world) for k in SPLITS}


def main(argv: Optional[Sequence[str]] = None):
    from ..config import default_cli_config
    ap = argparse.ArgumentParser(description="Cross-sectionally sharded GAN training (torchrun, one rank per GPU)")
    ap.add_argument("--data_dir", default=None)
    ap.add_argument("--synthetic", type=int, nargs=6, default=None, metavar=("T_TR", "T_VA", "T_TE", "N", "F", "M"))
    ap.add_argument("--data_seed", type=int, default=0)
    ap.add_argument("--epochs", type=int, nargs=3, default=[256, 64, 1024])
    ap.add_argument("--ignore_epoch", type=int, default=64)
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--print_freq", type=int, default=128)
    ap.add_argument("--save_dir", default=None)
    ap.add_argument("--cpu", action="store_true")
    ap.add_argument("--torch_towers", action="store_true", help="local towers as PyTorch ops instead of the engine")
    ap.add_argument("--mode", choices=("engine", "towers"), default="engine",
                    help="engine: the whole epoch on the native engine with all-reduce callbacks (GPU); "
                         "towers: engine (or --torch_towers) towers under eager torch losses")
    ap.add_argument("--out", default=None)
    args = ap.parse_args(argv)
    d = comm.init(use_gpu=False if args.cpu else None)
    b = load_shards(args, d)
    tr = b["train"]
    cfg = default_cli_config(tr["macro_features"].shape[1] if tr.get("macro_features") is not None else 0,
                             tr["individual_features"].shape[2])
    t0 = time.time()
    if args.mode == "engine" and d.device.type == "cuda" and not args.torch_towers:
        model, hist = train_3phase_xsection_engine(cfg, b["train"], b["valid"], b["test"], d,
                                                   num_epochs_unc=args.epochs[0], num_epochs_moment=args.epochs[1],
                                                   num_epochs=args.epochs[2], lr=args.lr,
                                                   print_freq=args.print_freq, save_dir=args.save_dir,
                                                   ignore_epoch=args.ignore_epoch, seed=args.seed)
        ev = {k: model.engine_final_eval[i] for i, k in enumerate(SPLITS)}
    else:
        model, hist = train_3phase_xsection(cfg, b["train"], b["valid"], b["test"], d, num_epochs_unc=args.epochs[0],
                                            num_epochs_moment=args.epochs[1], num_epochs=args.epochs[2], lr=args.lr,
                                            print_freq=args.print_freq, save_dir=args.save_dir,
                                            ignore_epoch=args.ignore_epoch, seed=args.seed,
                                            engine=False if args.torch_towers else None)
        ev = {k: evaluate(model, b[k], d.device) for k in SPLITS}
    wall = time.time() - t0
    n_ep = sum(args.epochs)
    res = {"world_size": d.world, "n_stocks": tr["n_total"], "wall_s": wall, "epochs": n_ep,
           "ms_per_epoch": 1e3 * wall / max(n_ep, 1),        # incl. the valid / test evaluations
           **{f"{k}_sharpe": float(ev[k]["sharpe"]) for k in SPLITS}}
    if d.is_main:
        print(json.dumps(res))
        if args.out:
            with open(args.out, "w") as f:
                json.dump(res, f)
    comm.shutdown(d)
    return res


if __name__ == "__main__":
    main()
