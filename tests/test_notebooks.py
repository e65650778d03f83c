"""The shipped notebooks stay runnable: execute the synthetic demo's code cells on the CPU with
a shortened schedule and a smaller panel (the plotting cell is skipped when matplotlib is absent)."""
import json
import os

import pytest

NB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "notebooks")


def _cells(name):
    with open(os.path.join(NB, name)) as fh:
        nb = json.load(fh)
    return ["".join(c["source"]) for c in nb["cells"] if c["cell_type"] == "code"]


@pytest.mark.parametrize("name", ["demo_synthetic.ipynb", "demo.ipynb", "demo_full.ipynb"])
def test_notebooks_are_valid_json_with_code(name):
    cells = _cells(name)
    assert cells and all(compile(c, name, "exec") for c in cells)


def test_demo_synthetic_runs_shortened(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    (tmp_path / "nb").mkdir()
    monkeypatch.chdir(tmp_path / "nb")
    subs = {"n_stocks=500": "n_stocks=80", "num_epochs_unc=256": "num_epochs_unc=3",
            "num_epochs_moment=64": "num_epochs_moment=2", "num_epochs=1024": "num_epochs=3",
            "ignore_epoch=64": "ignore_epoch=0", "device=device": "device=torch.device('cpu')",
            "sys.path.insert(0, os.path.abspath('..'))":
                f"sys.path.insert(0, {os.path.dirname(NB)!r})"}
    env = {}
    for src in _cells("demo_synthetic.ipynb"):
        if "matplotlib" in src:
            pytest.importorskip("matplotlib")
            continue
        for a, b in subs.items():
            src = src.replace(a, b)
        exec(compile(src, "demo_synthetic", "exec"), env)
    assert len(env["history"]["train_loss"]) == 6
