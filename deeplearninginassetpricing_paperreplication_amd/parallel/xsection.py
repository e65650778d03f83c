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
flat gradient all-reduce (~12k floats) — all latency-bound, a few µs each over xGMI. The local
towers run as PyTorch ops on the rank's device (hipBLASLt GEMMs on a GPU): this mode trades the
fused single-GPU engine for capacity.
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


class XSectionGAN(AssetPricingGAN):
    """``AssetPricingGAN`` whose forward / get_weights take the rank's stock shard and return
    the GLOBAL losses, portfolio returns and Sharpe (weights and moments stay local).
    State-dict keys and initialisation equal ``AssetPricingGAN`` (it is a subclass)."""

    def __init__(self, config: Dict, dist: comm.Dist, lstm_seed: int = 0):
        super().__init__(config)
        self.dist = dist
        self.lstm_seed = int(lstm_seed)
        self._lstm_calls = 0

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
        m = mask.float()
        w = self.raw_weights(macro, x) * m
        if not self.sdf_net.normalize_weights:
            return w
        s = all_reduce_sum(torch.stack([(w * m).sum(1), m.sum(1)]), self.dist)
        mu = s[0] / s[1].clamp(min=1)
        return (w - mu[:, None]) * m

    # -- global losses -------------------------------------------------------------------------
    def _portfolio(self, w, r, m):
        s = all_reduce_sum(torch.stack([(w * r * m).sum(1), m.sum(1)]), self.dist)
        if not self.weighted_loss:
            return s[0]
        n_t = s[1].clamp(min=1)
        return s[0] / n_t * n_t.mean()

    def _moment_loss(self, h, r, m, sdf, n_total):
        t_i = m.sum(0).clamp(min=1)
        q = r * m * sdf[:, None]
        e = (q.sum(0) / t_i)[None] if h is None else (h * q[None]).sum(1) / t_i     # [K, N_r]
        return all_reduce_sum((e ** 2).sum(1), self.dist).mean() / n_total

    def _residual(self, w, r, m):
        s = all_reduce_sum(torch.stack([m.sum(1), (w * w * m).sum(1), (r * w * m).sum(1),
                                        (r * r * m).sum(1)]), self.dist)
        n, ww, rw, rr = s
        use = n >= 2
        has = use & (ww > 1e-8)
        if not bool(use.any()) or not bool(has.any()):
            return torch.zeros((), device=w.device)
        beta = torch.where(has, rw / torch.where(has, ww, torch.ones_like(ww)), torch.zeros_like(ww))
        nc = n.clamp(min=1)
        resid = (rr - 2 * beta * rw + beta * beta * ww) / nc
        rsq = rr / nc
        resid_mean = (resid * has.float()).sum() / has.float().sum()
        rsq_mean = (rsq * use.float()).sum() / use.float().sum()
        return resid_mean / rsq_mean.clamp(min=1e-8)

    def forward(self, macro_features, individual_features, returns, mask, hidden=None,
                phase: str = "conditional", n_total: Optional[int] = None) -> Dict[str, torch.Tensor]:
        """Same dict as ``AssetPricingGAN.forward`` (`model.py:485-563`): loss, losses, sharpe
        and portfolio returns are global; weights [T, N_r] and moments [K, T, N_r] local."""
        if n_total is None:
            n_total = int(all_reduce_sum(torch.tensor([float(returns.shape[1])], device=returns.device),
                                         self.dist).item()) if self.dist.active else returns.shape[1]
        m = mask.float()
        w = self.shard_weights(macro_features, individual_features, mask)
        moments = self.moment_net(self._moment_input(macro_features, individual_features))
        p = self._portfolio(w, returns, m)
        zero = torch.zeros((), device=w.device)
        if phase == "unconditional":
            loss_unc = self._moment_loss(None, returns, m, p + 1.0, n_total)
            loss_cond, total = zero, loss_unc
        elif phase == "moment":
            loss_cond = self._moment_loss(moments, returns, m, p + 1.0, n_total)
            loss_unc, total = zero, -loss_cond
        else:
            loss_cond = self._moment_loss(moments, returns, m, p + 1.0, n_total)
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
    return {"loss": out["loss"].item(), "loss_unc": out["loss_unconditional"].item(),
            "loss_cond": out["loss_conditional"].item(), "loss_residual": out["loss_residual"].item(),
            "sharpe": compute_sharpe(out["portfolio_returns"].detach()),
            "grad_norm": gn.item() if isinstance(gn, torch.Tensor) else gn}


@torch.no_grad()
def evaluate(model: XSectionGAN, data: Dict, device, normalized: bool = True) -> Dict:
    """Global evaluation metrics from the rank's shard (`/root/reference/src/train.py:106-153`);
    ``weights`` are the rank's stocks."""
    model.eval()
    macro, x, r, m = _args(data, device)
    w, _ = model.get_weights(macro, x, m, normalized=normalized)
    pr = all_reduce_sum((w * r * m.float()).sum(1), model.dist)
    port = pr.cpu().numpy()
    out = model(macro, x, r, m, phase="conditional", n_total=data.get("n_total"))
    return {"loss": out["loss"].item(), "loss_unc": out["loss_unconditional"].item(),
            "loss_cond": out["loss_conditional"].item(), "sharpe": compute_sharpe(pr.cpu()),
            "max_drawdown": compute_max_drawdown(port), "mean_return": port.mean(),
            "std_return": port.std(), "weights": w.cpu()}


def train_3phase_xsection(config: Dict, train_data: Dict, valid_data: Dict, test_data: Optional[Dict],
                          dist: comm.Dist, device=None, num_epochs_unc: int = 256,
                          num_epochs_moment: int = 64, num_epochs: int = 1024, lr: float = 1e-3,
                          print_freq: int = 128, save_dir: Optional[str] = None, ignore_epoch: int = 64,
                          seed: int = 42, selection_sign: float = 1.0, verbose: bool = True,
                          nan_policy: str = "warn"):
    """``train_3phase`` over stock shards (``*_data``: FULL split dicts or already-sharded ones
    carrying ``n_total``). Same schedule, trackers and checkpoints as the CPU trainer; rank 0
    writes the checkpoints. Returns ``(model, history)`` on every rank."""
    from ..train.trainer import _train_3phase_cpu
    device = torch.device(device or dist.device)
    sh = [None if b is None else (b if "n_total" in b else shard_batch(b, dist.rank, dist.world))
          for b in (train_data, valid_data, test_data)]
    torch.manual_seed(seed)                      # identical initial parameters on every rank
    model = XSectionGAN(config, dist, lstm_seed=seed).to(device)
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
    ap.add_argument("--out", default=None)
    args = ap.parse_args(argv)
    d = comm.init(use_gpu=False if args.cpu else None)
    b = load_shards(args, d)
    tr = b["train"]
    cfg = default_cli_config(tr["macro_features"].shape[1] if tr.get("macro_features") is not None else 0,
                             tr["individual_features"].shape[2])
    t0 = time.time()
    model, hist = train_3phase_xsection(cfg, b["train"], b["valid"], b["test"], d, num_epochs_unc=args.epochs[0],
                                        num_epochs_moment=args.epochs[1], num_epochs=args.epochs[2], lr=args.lr,
                                        print_freq=args.print_freq, save_dir=args.save_dir,
                                        ignore_epoch=args.ignore_epoch, seed=args.seed)
    ev = {k: evaluate(model, b[k], d.device) for k in SPLITS}
    res = {"world_size": d.world, "n_stocks": tr["n_total"], "wall_s": time.time() - t0,
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
