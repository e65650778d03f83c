"""``.npz`` panel loading with the reference's masking / standardisation semantics.

Contract (`/root/reference/src/data_loader.py:11-237`):
  * ``data[:, :, 0]`` are returns, ``data[:, :, 1:]`` firm characteristics (float32);
  * an entry is valid iff return > −98.99, return is not NaN and *every* characteristic
    > −98.99 (missing sentinel −99.99); invalid entries are zero-filled;
  * macro series are z-scored with the *train* mean / std (numpy ddof=0, std + 1e-8);
    valid / test receive the train statistics;
  * ``get_full_batch`` hands out zero-copy CPU tensors.

Host memory: the reference keeps the raw array plus full copies of returns, features and
their zero-filled versions (~4 panel copies). Here an uncompressed (``np.savez``) member is
memory-mapped straight out of the archive (``_npz_member``: no read into RAM at all), and the
mask / zero-fill run over period chunks into the one output array, so the resident cost is one
float32 panel (plus the decompressed raw array for ``savez_compressed`` files, which cannot be
mapped).
"""
from __future__ import annotations

from typing import Optional, Sequence

import zipfile

import numpy as np
import torch

MISSING_VALUE = -99.99
_CHUNK_BYTES = 256 << 20          # period chunk of the masking pass


def _npz_member(path: str, name: str):
    """Array ``name`` of the ``.npz`` at ``path``: a read-only ``np.memmap`` into the archive when
    the member is stored uncompressed (``np.savez``), else the decompressed array."""
    with zipfile.ZipFile(path) as zf:
        info = zf.getinfo(name + ".npy")
        if info.compress_type == zipfile.ZIP_STORED:
            with zf.open(info) as f:
                version = np.lib.format.read_magic(f)
                if version == (1, 0):
                    shape, fortran, dtype = np.lib.format.read_array_header_1_0(f)
                else:
                    shape, fortran, dtype = np.lib.format.read_array_header_2_0(f)
                header = f.tell()
            if not dtype.hasobject:
                with open(path, "rb") as fh:          # data offset = local header + npy header
                    fh.seek(info.header_offset + 26)
                    ln = int.from_bytes(fh.read(2), "little") + int.from_bytes(fh.read(2), "little")
                start = info.header_offset + 30 + ln + header
                return np.memmap(path, dtype=dtype, mode="r", offset=start, shape=shape,
                                 order="F" if fortran else "C")
    with np.load(path) as z:
        return z[name]


class AssetPricingDataset(torch.utils.data.Dataset):
    def __init__(self, path_individual_feature: str, path_macro_feature: Optional[str] = None,
                 macro_idx: Optional[Sequence[int]] = None, mean_macro: Optional[np.ndarray] = None,
                 std_macro: Optional[np.ndarray] = None, normalize_macro: bool = True):
        with np.load(path_individual_feature) as z:
            files = set(z.files)
            self.dates = z["date"] if "date" in files else None
            self.variable_names = z["variable"] if "variable" in files else None
        raw = _npz_member(path_individual_feature, "data")
        T, N, C = raw.shape
        if self.dates is None:
            self.dates = np.arange(T)
        thr = np.float32(MISSING_VALUE + 1)
        self.mask = np.empty((T, N), dtype=bool)
        self.returns = np.empty((T, N), dtype=np.float32)
        self.individual_features = np.empty((T, N, C - 1), dtype=np.float32)
        step = max(1, _CHUNK_BYTES // max(1, N * C * 4))
        for t0 in range(0, T, step):       # one period chunk in flight: mask, zero-fill, copy out
            blk = np.asarray(raw[t0:t0 + step], dtype=np.float32)
            ret, feat = blk[:, :, 0], blk[:, :, 1:]
            m = (ret > thr) & ~np.isnan(ret)
            m &= np.all(feat > thr, axis=2)
            self.mask[t0:t0 + step] = m
            self.returns[t0:t0 + step] = np.where(m, ret, np.float32(0.0))
            out = self.individual_features[t0:t0 + step]
            out[...] = feat
            out[~m] = 0.0
        del raw

        self.mean_macro = self.std_macro = None
        self.macro_features = None
        if path_macro_feature is not None:
            mac = np.load(path_macro_feature)["data"].astype(np.float32)
            if macro_idx is not None:
                mac = mac[:, list(macro_idx)]
            if normalize_macro:
                if mean_macro is None:
                    self.mean_macro = mac.mean(axis=0, keepdims=True)
                    self.std_macro = mac.std(axis=0, keepdims=True) + 1e-8
                else:
                    self.mean_macro, self.std_macro = mean_macro, std_macro
                mac = (mac - self.mean_macro) / self.std_macro
            self.macro_features = mac

        self.T, self.N = self.returns.shape
        self.individual_feature_dim = self.individual_features.shape[2]
        self.macro_feature_dim = 0 if self.macro_features is None else self.macro_features.shape[1]

    @classmethod
    def from_arrays(cls, returns: np.ndarray, features: np.ndarray, mask: np.ndarray,
                    macro: Optional[np.ndarray] = None) -> "AssetPricingDataset":
        """Build directly from in-memory (already masked, zero-filled) arrays."""
        self = cls.__new__(cls)
        self.mask = mask.astype(bool)
        self.returns = np.where(self.mask, returns, 0).astype(np.float32)
        self.individual_features = np.where(self.mask[:, :, None], features, 0).astype(np.float32)
        self.dates = np.arange(returns.shape[0])
        self.variable_names = None
        self.macro_features = None if macro is None else macro.astype(np.float32)
        self.mean_macro = self.std_macro = None
        self.T, self.N = self.returns.shape
        self.individual_feature_dim = self.individual_features.shape[2]
        self.macro_feature_dim = 0 if macro is None else macro.shape[1]
        return self

    def __len__(self) -> int:
        return self.T

    def __getitem__(self, idx):
        item = {"individual_features": torch.from_numpy(self.individual_features[idx]),
                "returns": torch.from_numpy(self.returns[idx]),
                "mask": torch.from_numpy(self.mask[idx])}
        if self.macro_features is not None:
            item["macro_features"] = torch.from_numpy(self.macro_features[idx])
        return item

    def get_full_batch(self):
        b = {"individual_features": torch.from_numpy(self.individual_features),
             "returns": torch.from_numpy(self.returns),
             "mask": torch.from_numpy(self.mask)}
        if self.macro_features is not None:
            b["macro_features"] = torch.from_numpy(self.macro_features)
        return b

    def get_macro_stats(self):
        return self.mean_macro, self.std_macro

    def get_date_count_list(self) -> np.ndarray:
        return self.mask.sum(axis=1).astype(np.float32)


def create_data_loaders(train_individual_path: str, train_macro_path: str,
                        valid_individual_path: str, valid_macro_path: str,
                        test_individual_path: str = None, test_macro_path: str = None,
                        macro_idx=None, batch_size=None):
    """Train / valid / (test) datasets sharing the train macro statistics."""
    tr = AssetPricingDataset(train_individual_path, train_macro_path, macro_idx=macro_idx)
    mu, sd = tr.get_macro_stats()
    va = AssetPricingDataset(valid_individual_path, valid_macro_path, macro_idx=macro_idx,
                             mean_macro=mu, std_macro=sd)
    te = None
    if test_individual_path is not None:
        te = AssetPricingDataset(test_individual_path, test_macro_path, macro_idx=macro_idx,
                                 mean_macro=mu, std_macro=sd)
    return tr, va, te


def create_small_sample(dataset: AssetPricingDataset, n_periods: int = 50, n_stocks: int = 100):
    """First ``n_periods`` periods and the ``n_stocks`` stocks with the most valid months.

    Stock order follows ``np.argsort(counts)[-N:]`` (ascending count), as in the reference.
    """
    T = min(n_periods, dataset.T)
    N = min(n_stocks, dataset.N)
    keep = np.argsort(dataset.mask.sum(axis=0))[-N:]
    out = {"individual_features": torch.from_numpy(dataset.individual_features[:T, keep, :]),
           "returns": torch.from_numpy(dataset.returns[:T, keep]),
           "mask": torch.from_numpy(dataset.mask[:T, keep])}
    if dataset.macro_features is not None:
        out["macro_features"] = torch.from_numpy(dataset.macro_features[:T])
    return out


def load_splits(data_dir: str, macro_idx=None):
    """The three datasets of a ``data_dir`` laid out as ``char/Char_{split}.npz`` +
    ``macro/macro_{split}.npz`` (macro optional)."""
    import os
    out = []
    stats = (None, None)
    for s in ("train", "valid", "test"):
        c = os.path.join(data_dir, "char", f"Char_{s}.npz")
        m = os.path.join(data_dir, "macro", f"macro_{s}.npz")
        ds = AssetPricingDataset(c, m if os.path.exists(m) else None, macro_idx=macro_idx,
                                 mean_macro=stats[0], std_macro=stats[1])
        if s == "train":
            stats = ds.get_macro_stats()
        out.append(ds)
    return tuple(out)
