"""Statistical parity of the bf16 GPU engine with the fp32 CPU trainer.

Dropout streams cannot match bitwise (a counter hash on the GPU, torch's ``bernoulli_`` on the
CPU), so the two executors are compared as distributions over seeds: the paper-sign test Sharpe
of every seed's selected model and the epoch the reference's selection rule picks in phases 1 and
3 (`/root/reference/src/train.py:268,378`: strict improvement of the un-negated validation Sharpe
after ``ignore_epoch``). ``tools/cpu_parity_record.py`` records the CPU side once
(``tests/fixtures/cpu_parity_record.json``); ``tests/test_parity_gpu.py`` trains the same seeds on
the GPU and checks that the means agree within their standard errors.
"""
from __future__ import annotations

from typing import Dict, Sequence

import numpy as np

SEEDS = (42, 123, 456, 789, 1000, 2000, 3000, 4000, 5000)   # `notebooks/demo_full.ipynb:1221`
SCHEDULE = (256, 64, 1024)
IGNORE_EPOCH = 64


def best_epochs(history: Dict, n_unc: int, ignore_epoch: int = IGNORE_EPOCH, sel: float = 1.0):
    """(phase-1 best epoch, phase-3 best epoch) the reference's rule selects from a history dict
    (``valid_sharpe`` over phases 1 then 3; -1 when no epoch qualifies)."""
    vs = np.asarray(history["valid_sharpe"], np.float64)
    out = []
    for lo, hi in ((0, n_unc), (n_unc, len(vs))):
        best, arg = -np.inf, -1
        for e in range(hi - lo):
            v = sel * vs[lo + e]
            if e > ignore_epoch and v > best:
                best, arg = v, e
        out.append(arg)
    return tuple(out)


def summarize(test_sharpes: Sequence[float], best: Sequence[Sequence[int]]) -> Dict:
    ts = np.asarray(test_sharpes, np.float64)
    b = np.asarray(best, np.float64)
    n = len(ts)
    return {"n": n,
            "test_sharpe_mean": float(ts.mean()), "test_sharpe_sd": float(ts.std(ddof=1)) if n > 1 else 0.0,
            "best_p1_mean": float(b[:, 0].mean()), "best_p1_sd": float(b[:, 0].std(ddof=1)) if n > 1 else 0.0,
            "best_p3_mean": float(b[:, 1].mean()), "best_p3_sd": float(b[:, 1].std(ddof=1)) if n > 1 else 0.0}


def within_se(a: Dict, b: Dict, key: str, z: float = 3.0) -> bool:
    """|mean_a - mean_b| <= z * SE of the difference of two independent means."""
    se = np.sqrt(a[key + "_sd"] ** 2 / a["n"] + b[key + "_sd"] ** 2 / b["n"])
    return bool(abs(a[key + "_mean"] - b[key + "_mean"]) <= z * max(se, 1e-12))
