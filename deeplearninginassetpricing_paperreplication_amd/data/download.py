"""Fetch the paper's real dataset (Google Drive) into ``<output_dir>/{char,macro}``.

Behaviour of `/root/reference/src/download_data.py`: same public functions
(``download_all_data``, ``check_data_exists``, ``download_datasets_zip``,
``download_from_folder``, ``print_data_info``), same CLI flags
(``--output_dir/-o --force/-f --quiet/-q --info/-i --check --method/-m {zip,folder}``) and exit
codes. Difference: ``gdown`` is imported only when a download actually starts, so ``--check``
and ``--info`` work without it (the reference exits at import time); a missing ``gdown`` or
network makes the download return False with a message instead.
"""
from __future__ import annotations

import argparse
import shutil
import sys
import tempfile
import zipfile
from pathlib import Path
from typing import Dict, List

DATASETS_ZIP_ID = "1h9O7YwPLaRBbghtF50Cr-JmIq0aHHi4Y"
GDRIVE_FOLDER_ID = "1TrYzMUA_xLID5-gXOy_as8sH2ahLwz-l"

_KB, _MB = 1024, 1024 * 1024
EXPECTED_SIZES = {"Char_train.npz": 317 * _MB, "Char_valid.npz": 72 * _MB, "Char_test.npz": 768 * _MB,
                  "macro_train.npz": 351 * _KB, "macro_valid.npz": 96 * _KB, "macro_test.npz": 436 * _KB}
REQUIRED = [("char", f"Char_{s}.npz") for s in ("train", "valid", "test")] + \
           [("macro", f"macro_{s}.npz") for s in ("train", "valid", "test")]


def check_data_exists(data_dir: str) -> Dict:
    root = Path(data_dir)
    files = [root / sub / name for sub, name in REQUIRED]
    have = [f for f in files if f.exists()]
    miss = [f for f in files if not f.exists()]
    return {"existing": have, "missing": miss, "complete": not miss}


def _gdown(quiet: bool):
    try:
        import gdown  # noqa: F401
        return gdown
    except ImportError:
        if not quiet:
            print("Error: 'gdown' package is required for downloading data.")
            print("Install it with: pip install gdown")
        return None


def _install_tree(src_root: Path, output_dir: Path) -> List[Path]:
    """Move every ``*/char/*.npz`` and ``*/macro/*.npz`` under src_root into output_dir."""
    moved = []
    for sub in ("char", "macro"):
        (output_dir / sub).mkdir(parents=True, exist_ok=True)
        for f in src_root.rglob(f"{sub}/*.npz"):
            if "__MACOSX" in f.parts:
                continue
            dst = output_dir / sub / f.name
            shutil.move(str(f), str(dst))
            moved.append(dst)
    return moved


def download_datasets_zip(output_dir: str, quiet: bool = False) -> bool:
    gd = _gdown(quiet)
    if gd is None:
        return False
    out = Path(output_dir)
    out.mkdir(parents=True, exist_ok=True)
    try:
        with tempfile.TemporaryDirectory(dir=out) as tmp:
            zpath = Path(tmp) / "datasets.zip"
            if not quiet:
                print(f"Downloading datasets.zip (id {DATASETS_ZIP_ID}) ...")
            got = gd.download(id=DATASETS_ZIP_ID, output=str(zpath), quiet=quiet)
            if not got or not zpath.exists():
                if not quiet:
                    print("Download failed.")
                return False
            with zipfile.ZipFile(zpath) as z:
                z.extractall(tmp)
            moved = _install_tree(Path(tmp), out)
        if not quiet:
            print(f"Installed {len(moved)} files into {out.absolute()}")
        return check_data_exists(output_dir)["complete"]
    except Exception as e:  # network / archive errors: report, do not raise
        if not quiet:
            print(f"Error during download: {e}")
        return False


def download_from_folder(output_dir: str, quiet: bool = False) -> bool:
    gd = _gdown(quiet)
    if gd is None:
        return False
    out = Path(output_dir)
    out.mkdir(parents=True, exist_ok=True)
    try:
        with tempfile.TemporaryDirectory(dir=out) as tmp:
            url = f"https://drive.google.com/drive/folders/{GDRIVE_FOLDER_ID}"
            if not quiet:
                print(f"Downloading folder {url} ...")
            gd.download_folder(url=url, output=tmp, quiet=quiet)
            moved = _install_tree(Path(tmp), out)
        if not quiet:
            print(f"Installed {len(moved)} files into {out.absolute()}")
        return check_data_exists(output_dir)["complete"]
    except Exception as e:
        if not quiet:
            print(f"Error during download: {e}")
        return False


def download_all_data(output_dir: str = "./data", force: bool = False, quiet: bool = False,
                      method: str = "zip") -> bool:
    if not force:
        st = check_data_exists(output_dir)
        if st["complete"]:
            if not quiet:
                print("All data files already exist!")
                print(f"Location: {Path(output_dir).absolute()}")
                print("\nUse --force to re-download.")
            return True
        if st["existing"] and not quiet:
            print(f"Found {len(st['existing'])} existing files.")
            print(f"Missing {len(st['missing'])} files:")
            for f in st["missing"]:
                print(f"  - {f}")
    order = ["zip", "folder"] if method == "zip" else ["folder", "zip"]
    for m in order:
        ok = download_datasets_zip(output_dir, quiet) if m == "zip" else download_from_folder(output_dir, quiet)
        if ok:
            return True
        if not quiet:
            print(f"Method '{m}' failed" + (", trying the other one..." if m == order[0] else "."))
    if not quiet:
        print("\nManual download:")
        print(f"  https://drive.google.com/drive/folders/{GDRIVE_FOLDER_ID}")
    return False


def print_data_info():
    print("Deep Learning in Asset Pricing - data files")
    print("=" * 50)
    for sub, name in REQUIRED:
        sz = EXPECTED_SIZES[name]
        print(f"  {sub}/{name:18s} ~{sz / _MB:8.1f} MB" if sz >= _MB else f"  {sub}/{name:18s} ~{sz / _KB:8.1f} KB")
    print("\nchar/Char_{split}.npz : data [T, N, 47] (returns + 46 characteristics), date, variable")
    print("macro/macro_{split}.npz: data [T, 178] macro series")
    print(f"Source: https://drive.google.com/drive/folders/{GDRIVE_FOLDER_ID}")


def main(argv=None):
    p = argparse.ArgumentParser(description="Download data for Deep Learning in Asset Pricing")
    p.add_argument("--output_dir", "-o", type=str, default="./data",
                   help="Directory to save data files (default: ./data)")
    p.add_argument("--force", "-f", action="store_true", help="Force re-download even if files exist")
    p.add_argument("--quiet", "-q", action="store_true", help="Suppress progress output")
    p.add_argument("--info", "-i", action="store_true", help="Print information about data files and exit")
    p.add_argument("--check", action="store_true", help="Check if data files exist and exit")
    p.add_argument("--method", "-m", type=str, choices=["zip", "folder"], default="zip",
                   help="Download method: 'zip' (faster, recommended) or 'folder' (default: zip)")
    a = p.parse_args(argv)
    if a.info:
        print_data_info()
        return 0
    if a.check:
        st = check_data_exists(a.output_dir)
        if st["complete"]:
            print("All data files found!")
            for f in st["existing"]:
                print(f"  {f} ({f.stat().st_size / _MB:.1f} MB)")
            sys.exit(0)
        print("Missing data files:")
        for f in st["missing"]:
            print(f"  {f}")
        sys.exit(1)
    sys.exit(0 if download_all_data(a.output_dir, a.force, a.quiet, a.method) else 1)


if __name__ == "__main__":
    main()
