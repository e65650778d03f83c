"""Stage-by-stage numerics check of the native engine against the fp32 PyTorch semantics.

Run on a GPU box:  python tools/gpu_check.py [--F 46 --M 8 --hidden 64 64 ...]
Prints max abs / relative errors for forward outputs, the three phases' gradients and a
short training run. Exit status 1 if any check exceeds its bf16 tolerance.
"""
import argparse
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from deeplearninginassetpricing_paperreplication_amd.config import default_cli_config  # noqa: E402
from deeplearninginassetpricing_paperreplication_amd.data.synthetic import generate_panel_fast  # noqa: E402
from deeplearninginassetpricing_paperreplication_amd.engine.runner import GANEngine, flatten_state, unflatten_state  # noqa: E402
from deeplearninginassetpricing_paperreplication_amd.models.gan import AssetPricingGAN  # noqa: E402

FAIL = []


def rel(a, b):
    a = np.asarray(a, np.float64); b = np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / (np.abs(b).max() + 1e-30))


def check(name, got, ref, tol):
    r = rel(got, ref)
    cos = float(np.dot(np.ravel(got), np.ravel(ref)) / (np.linalg.norm(got) * np.linalg.norm(ref) + 1e-30))
    ok = r < tol
    print(f"  {'ok ' if ok else 'BAD'} {name:34s} rel_max={r:.3e} cos={cos:.6f}")
    if not ok:
        FAIL.append(name)


def batch_from(ret, feats, mask, mac):
    return {"returns": ret, "individual_features": feats, "mask": mask, "macro_features": mac}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=48)
    ap.add_argument("--N", type=int, default=300)
    ap.add_argument("--F", type=int, default=46)
    ap.add_argument("--M", type=int, default=8)
    ap.add_argument("--hidden", type=int, nargs="+", default=[64, 64])
    ap.add_argument("--rnn", type=int, nargs="+", default=[4])
    ap.add_argument("--hm", type=int, nargs="*", default=[])
    ap.add_argument("--K", type=int, default=8)
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args()
    print(f"config: T={a.T} N={a.N} F={a.F} M={a.M} hidden={a.hidden} rnn={a.rnn} hm={a.hm} K={a.K}")
    ret, feats, mask, mac = generate_panel_fast(a.T, a.N, a.F, a.M, seed=a.seed)
    mac = (mac - mac.mean(0)) / (mac.std(0, unbiased=False) + 1e-8)
    cfg = default_cli_config(a.M, a.F, hidden_dim=a.hidden, rnn_dim=a.rnn, num_moments=a.K,
                             dropout=0.0, hidden_dim_moment=a.hm)
    torch.manual_seed(a.seed)
    model = AssetPricingGAN(cfg)
    # make the moment net less trivial (default init gives small h)
    b = batch_from(ret, feats, mask, mac)
    eng = GANEngine(model.spec, 1, max_epochs=64)
    eng.set_data(b, b, b)
    eng.set_model(0, model, 1234)
    # ---------------- forward ----------------
    with torch.no_grad():
        out = model(mac, feats, ret, mask, phase="conditional")
    eng.eng.forward_split(0, False, True)
    T, N = a.T, a.N
    wn = eng.eng.read_ws(0, 0, "wn").reshape(T, N)
    h = eng.eng.read_ws(0, 0, "h").reshape(T, N, a.K)
    P = eng.eng.read_ws(0, 0, "P")
    sc = eng.eng.read_ws(0, 0, "scal")
    m = mask.numpy()
    print("forward:")
    if model.sdf_net.macro_lstm is not None:
        with torch.no_grad():
            lh, _ = model.sdf_net.macro_lstm(mac)
        check("lstm output", eng.eng.read_ws(0, 0, "pp").reshape(T, -1), lh.numpy(), 1e-4)
    check("weights w'", wn, out["weights"].numpy(), 3e-2)
    check("moments h (valid)", h[m], out["moments"].permute(1, 2, 0).numpy()[m], 3e-2)
    check("portfolio P", P, out["portfolio_returns"].numpy(), 3e-2)
    check("loss_cond", sc[0], out["loss_conditional"].item(), 3e-2)
    check("loss_unc", sc[1], out["loss_unconditional"].item(), 3e-2)
    # ---------------- gradients ----------------
    for phase, pname in ((1, "unconditional"), (3, "conditional"), (2, "moment")):
        model.zero_grad()
        o = model(mac, feats, ret, mask, phase=pname)
        o["loss"].backward()
        ref = flatten_state({k: (p.grad if p.grad is not None else torch.zeros_like(p))
                             for k, p in model.named_parameters()}, model.spec)
        eng.eng.backward_only(phase)
        got = eng.eng.get_grads(0)
        P_sdf = model.spec.param_counts()[0]
        sl = slice(0, P_sdf) if phase != 2 else slice(P_sdf, None)
        print(f"phase {phase} gradients:")
        lay = model.spec.param_layout()
        o_ = 0
        scale = np.linalg.norm(ref[sl])
        for k, shp in lay:
            n = int(np.prod(shp))
            if (phase != 2 and k.startswith("sdf")) or (phase == 2 and k.startswith("moment")):
                g_, r_ = got[o_:o_ + n], ref[o_:o_ + n]
                err = np.linalg.norm(g_ - r_) / max(np.linalg.norm(r_), 1e-3 * scale)
                ok = err < 0.08
                print(f"  {'ok ' if ok else 'BAD'} {k:44s} rel_l2={err:.3e} |g|={np.linalg.norm(r_):.3e}")
                if not ok:
                    FAIL.append(k)
            o_ += n
    # ---------------- short training vs CPU ----------------
    from deeplearninginassetpricing_paperreplication_amd.train.trainer import train_3phase
    torch.manual_seed(a.seed)
    m_cpu, h_cpu = train_3phase(cfg, b, b, b, device="cpu", num_epochs_unc=6, num_epochs_moment=3,
                                num_epochs=6, print_freq=100, ignore_epoch=1, verbose=False)
    torch.manual_seed(a.seed)
    t0 = time.time()
    m_gpu, h_gpu = train_3phase(cfg, b, b, b, device="cuda", num_epochs_unc=6, num_epochs_moment=3,
                                num_epochs=6, print_freq=100, ignore_epoch=1, verbose=False, seed=5)
    print(f"train_3phase gpu wall {time.time() - t0:.2f}s")
    print("history (gpu vs cpu):")
    for k in ("train_loss", "valid_loss", "valid_sharpe", "train_sharpe"):
        check(k, np.array(h_gpu[k]), np.array(h_cpu[k]), 0.15)
    print("FAILED:" if FAIL else "ALL OK", FAIL)
    return 1 if FAIL else 0


if __name__ == "__main__":
    sys.exit(main())
