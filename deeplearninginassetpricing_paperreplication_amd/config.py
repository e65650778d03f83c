"""Model configuration: the config-dict contract of the reference and the derived layout.

The reference model reads exactly 13 keys from its config dict with ``.get`` defaults
(`/root/reference/src/model.py:298-344`); every other key (``num_layers``,
``cell_type_rnn`` ...) is accepted and ignored.  ``ModelSpec`` freezes that contract into
an immutable description shared by the PyTorch modules, the native engine
(``csrc/engine.cpp`` mirrors ``param_layout``) and the ensemble/sweep drivers.

Quirks preserved on purpose:
  * the macro LSTM has ``len(num_units_rnn)`` layers, *all* of width ``num_units_rnn[-1]``
    (`model.py:39-45`);
  * ``num_units_rnn_moment`` / ``use_rnn_moment`` are parsed but have no effect
    (`model.py:309-311,337-338`);
  * the moment network input is ``[raw macro ; individual]`` while the SDF input is
    ``[individual ; lstm(macro)]`` (`model.py:253-255,513-516`).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Tuple

# Keys the model reads and their defaults (model.py:304-344).
MODEL_KEY_DEFAULTS = {
    "num_units_rnn": [4],
    "num_units_rnn_moment": [32],
    "dropout": 0.05,
    "macro_feature_dim": 0,
    "hidden_dim": [64, 64],
    "use_rnn": True,
    "normalize_w": True,
    "hidden_dim_moment": [],
    "num_condition_moment": 8,
    "use_rnn_moment": True,
    "residual_loss_factor": 0.0,
    "weighted_loss": True,
}
# 'individual_feature_dim' is required (KeyError if missing, model.py:319).


def _as_list(v) -> List[int]:
    if isinstance(v, int):
        return [v]
    return [int(x) for x in v]


@dataclass(frozen=True)
class ModelSpec:
    macro_dim: int
    individual_dim: int
    hidden: Tuple[int, ...]
    rnn_layers: int          # number of LSTM layers (0 = no LSTM)
    rnn_hidden: int          # width of every LSTM layer
    moment_hidden: Tuple[int, ...]
    num_moments: int
    dropout: float
    normalize_w: bool
    weighted_loss: bool
    residual_loss_factor: float
    raw: Dict = field(default_factory=dict, compare=False, hash=False)

    @staticmethod
    def from_config(config: Dict) -> "ModelSpec":
        g = lambda k: config.get(k, MODEL_KEY_DEFAULTS[k])
        rnn = _as_list(g("num_units_rnn"))
        use_rnn = bool(g("use_rnn"))
        macro_dim = int(g("macro_feature_dim"))
        has_lstm = use_rnn and len(rnn) > 0 and macro_dim > 0
        return ModelSpec(
            macro_dim=macro_dim,
            individual_dim=int(config["individual_feature_dim"]),
            hidden=tuple(_as_list(g("hidden_dim"))),
            rnn_layers=len(rnn) if has_lstm else 0,
            rnn_hidden=rnn[-1] if has_lstm else 0,
            moment_hidden=tuple(_as_list(g("hidden_dim_moment"))),
            num_moments=int(g("num_condition_moment")),
            dropout=float(g("dropout")),
            normalize_w=bool(g("normalize_w")),
            weighted_loss=bool(g("weighted_loss")),
            residual_loss_factor=float(g("residual_loss_factor")),
            raw=dict(config),
        )

    # ---- derived dimensions -------------------------------------------------------
    @property
    def sdf_macro_dim(self) -> int:
        """Width of the macro block appended to the individual features in the SDF input."""
        return self.rnn_hidden if self.rnn_layers > 0 else self.macro_dim

    @property
    def sdf_in(self) -> int:
        return self.individual_dim + self.sdf_macro_dim

    @property
    def moment_in(self) -> int:
        return self.macro_dim + self.individual_dim

    def param_layout(self) -> List[Tuple[str, Tuple[int, ...]]]:
        """(state_dict key, shape) in ``state_dict()`` order of the reference module."""
        out: List[Tuple[str, Tuple[int, ...]]] = []
        H = self.rnn_hidden
        for l in range(self.rnn_layers):
            inp = self.macro_dim if l == 0 else H
            p = "sdf_net.macro_lstm.lstm."
            out += [(f"{p}weight_ih_l{l}", (4 * H, inp)), (f"{p}weight_hh_l{l}", (4 * H, H)),
                    (f"{p}bias_ih_l{l}", (4 * H,)), (f"{p}bias_hh_l{l}", (4 * H,))]
        prev = self.sdf_in
        for j, h in enumerate(self.hidden):
            out += [(f"sdf_net.fc_layers.{3 * j}.weight", (h, prev)),
                    (f"sdf_net.fc_layers.{3 * j}.bias", (h,))]
            prev = h
        out += [("sdf_net.output_proj.weight", (1, prev)), ("sdf_net.output_proj.bias", (1,))]
        prev = self.moment_in
        for j, h in enumerate(self.moment_hidden):
            out += [(f"moment_net.fc_layers.{3 * j}.weight", (h, prev)),
                    (f"moment_net.fc_layers.{3 * j}.bias", (h,))]
            prev = h
        out += [("moment_net.output_proj.weight", (self.num_moments, prev)),
                ("moment_net.output_proj.bias", (self.num_moments,))]
        return out

    def param_counts(self) -> Tuple[int, int]:
        """(#SDF params, #moment params)."""
        sdf = mom = 0
        for k, shp in self.param_layout():
            n = 1
            for s in shp:
                n *= s
            if k.startswith("sdf_net."):
                sdf += n
            else:
                mom += n
        return sdf, mom


def default_cli_config(macro_dim: int, individual_dim: int, hidden_dim=(64, 64), use_lstm=True,
                       rnn_dim=(4,), num_moments=8, dropout=0.05, hidden_dim_moment=(),
                       rnn_dim_moment=(32,)) -> Dict:
    """The 17-key dict the CLI writes to ``config.json`` (`/root/reference/src/train.py:530-561`)."""
    hidden_dim, rnn_dim = list(hidden_dim), list(rnn_dim)
    hidden_dim_moment, rnn_dim_moment = list(hidden_dim_moment), list(rnn_dim_moment)
    return {
        "macro_feature_dim": macro_dim,
        "individual_feature_dim": individual_dim,
        "hidden_dim": hidden_dim,
        "num_layers": len(hidden_dim),
        "use_rnn": use_lstm,
        "num_units_rnn": rnn_dim,
        "num_layers_rnn": len(rnn_dim),
        "cell_type_rnn": "lstm",
        "hidden_dim_moment": hidden_dim_moment,
        "num_layers_moment": len(hidden_dim_moment),
        "num_condition_moment": num_moments,
        "use_rnn_moment": True,
        "num_units_rnn_moment": rnn_dim_moment,
        "num_layers_rnn_moment": len(rnn_dim_moment),
        "cell_type_rnn_moment": "lstm",
        "dropout": dropout,
        "normalize_w": True,
        "weighted_loss": True,
        "residual_loss_factor": 0.0,
    }
