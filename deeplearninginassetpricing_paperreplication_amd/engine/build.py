"""Build the native HIP extension ``_dlap_hip`` in-tree with hipcc (gfx950 only).

Every ``csrc/*.hip`` kernel file and the C++ runtime ``csrc/engine.cpp`` are compiled as
separate objects (in parallel, cached by source hash) and linked into
``deeplearninginassetpricing_paperreplication_amd/_dlap_hip*.so``. No torch headers are
involved: the runtime talks to Python through pybind11 and to the GPU through HIP directly.
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import os
import subprocess
import sys
import sysconfig
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
CSRC = ROOT / "csrc"
PKG = ROOT / "deeplearninginassetpricing_paperreplication_amd"
BUILD = ROOT / "build" / "native"
ARCH = os.environ.get("DLAP_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def ext_path() -> Path:
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return PKG / f"_dlap_hip{suffix}"


def _includes():
    import pybind11
    return [f"-I{CSRC}", f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}"]


def _hash(files) -> str:
    h = hashlib.sha256()
    for f in sorted(files):
        h.update(f.name.encode())
        h.update(f.read_bytes())
    h.update(ARCH.encode())
    return h.hexdigest()[:16]


def _compile(src: Path, obj: Path, flags):
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", *flags, "-c", str(src), "-o", str(obj)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src.name}:\n{r.stderr[-4000:]}")
    return obj


# Host-side undefined-behaviour checks in trap mode (no sanitizer runtime to preload into the
# Python process; any UB in the C++ runtime or the launchers stops the process with SIGILL).
# GPU sanitizers are not available on the MI355X pool, the device code is unchanged.
UBSAN_FLAGS = ["-Xarch_host", "-fsanitize=undefined", "-Xarch_host", "-fsanitize-trap=undefined",
               "-Xarch_host", "-fno-sanitize=vptr"]


# Device-side bounds assertions (DLAP_ASSERT in csrc/common.h) for fault hunting: a kernel index
# that leaves its allocation aborts with the failing condition printed.
DEBUG_FLAGS = ["-DDLAP_DEBUG=1"]


def variant_path(variant: str) -> Path:
    """Where a non-default build lives (``PKG/<variant>/_dlap_hip*.so``); ``ops.native.load``
    imports it instead of the production module when ``DLAP_NATIVE=<variant>``."""
    return PKG / variant / ext_path().name


# Per-source extra flags of the production build (none). Measured alternative, kept for A/B
# runs: k_mlp.hip with "-mllvm -amdgpu-mfma-vgpr-form" (MFMA results in VGPRs instead of the
# accumulator file: half the v_accvgpr_read moves in the tower backward) ran within noise of
# the default (3954/3999 vs 3990/3972 model-epochs/s, profiles/README.md).
# k_tbwd.hip: the builtin MFMAs in VGPR form (the forward / chain layer results feed VALU work
# without accumulator-file moves); its long-lived weight-gradient sums are pinned to AGPRs by asm.
FILE_FLAGS: dict = {"k_tbwd.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form"]}


def build(force: bool = False, jobs: int = 8, verbose: bool = True, ubsan: bool = False,
          debug: bool = False, variant: str | None = None, file_flags: dict | None = None) -> Path:
    """Build the extension; ``variant`` + ``file_flags`` build a named side artefact (loaded with
    ``DLAP_NATIVE=<variant>``) whose per-file flags replace FILE_FLAGS, for A/B measurements."""
    srcs = sorted(CSRC.glob("*.hip")) + [CSRC / "engine.cpp"]
    headers = sorted(CSRC.glob("*.h"))
    out = ext_path()
    build_dir = BUILD
    ff = FILE_FLAGS if file_flags is None else file_flags
    variant = "ubsan" if ubsan else ("debug" if debug else variant)
    if variant:     # a separate artefact next to the production one (selected by DLAP_NATIVE)
        out = variant_path(variant)
        out.parent.mkdir(exist_ok=True)
        build_dir = BUILD / variant
    stamp = build_dir / "stamp"
    key = _hash(srcs + headers) + repr(sorted(ff.items()))
    if not force and out.exists() and stamp.exists() and stamp.read_text() == key:
        if verbose:
            print(f"[dlap] native extension up to date: {out.name}")
        return out
    build_dir.mkdir(parents=True, exist_ok=True)
    flags = _includes() + ["-Wno-unused-result"] + (UBSAN_FLAGS if ubsan else []) + (DEBUG_FLAGS if debug else [])
    objs = []
    hkey = _hash(headers)
    todo = []
    for s in srcs:      # per-object cache: source + every header + its flags
        obj = build_dir / (s.stem + ".o")
        okey = build_dir / (s.stem + ".key")
        k = _hash([s]) + hkey + repr(flags + ff.get(s.name, []))
        if not force and obj.exists() and okey.exists() and okey.read_text() == k:
            objs.append(obj)
        else:
            todo.append((s, obj, okey, k))
    with cf.ThreadPoolExecutor(max_workers=max(1, min(jobs, len(todo) or 1))) as ex:
        futs = {ex.submit(_compile, s, obj, flags + ff.get(s.name, [])): (s, okey, k) for s, obj, okey, k in todo}
        for f in cf.as_completed(futs):
            objs.append(f.result())
            s, okey, k = futs[f]
            okey.write_text(k)
            if verbose:
                print(f"[dlap] compiled {s.name}")
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *(UBSAN_FLAGS if ubsan else []),
           *map(str, sorted(objs)), "-o", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr[-4000:]}")
    stamp.write_text(key)
    if verbose:
        print(f"[dlap] built {out}")
    return out


# Host AddressSanitizer harness: the runtime + the host side of every kernel file,
# instrumented, linked into an executable that embeds Python (csrc/host/asan_main.cpp). The ASan
# runtime is part of the executable, so nothing has to be preloaded into a Python process.
# Device code is not instrumented (GPU sanitizers are not available on the MI355X pool).
ASAN_FLAGS = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fno-omit-frame-pointer"]


def asan_harness_path() -> Path:
    # in-tree next to the package (travels to the GPU box with the snapshot; git-ignored)
    return PKG / "asan" / "dlap_asan_python"


def build_asan_harness(force: bool = False, jobs: int = 8, verbose: bool = True) -> Path:
    srcs = sorted(CSRC.glob("*.hip")) + [CSRC / "engine.cpp", CSRC / "host" / "asan_main.cpp"]
    headers = sorted(CSRC.glob("*.h"))
    bdir = BUILD / "asan"
    out = asan_harness_path()
    stamp = bdir / "stamp"
    key = _hash(srcs + headers) + "asan"
    if not force and out.exists() and stamp.exists() and stamp.read_text() == key:
        return out
    bdir.mkdir(parents=True, exist_ok=True)
    out.parent.mkdir(exist_ok=True)
    flags = _includes() + ["-Wno-unused-result", "-DDLAP_EMBED=1"] + ASAN_FLAGS
    with cf.ThreadPoolExecutor(max_workers=max(1, min(jobs, len(srcs)))) as ex:
        futs = {ex.submit(_compile, s, bdir / (s.stem + ".o"), flags): s for s in srcs}
        objs = [f.result() for f in cf.as_completed(futs)]
    libdir = sysconfig.get_config_var("LIBDIR")
    pyver = sysconfig.get_config_var("LDVERSION") or sysconfig.get_python_version()
    import importlib.util
    spec = importlib.util.find_spec("torch")
    # torch dlopens some of its own libraries by bare name (e.g. libcaffe2_nvrtc): the harness
    # executable carries torch/lib in its rpath, as the python binary's loader setup does
    rp = [f"-Wl,-rpath,{libdir}"] + ([f"-Wl,-rpath,{Path(spec.origin).parent / 'lib'}"] if spec else [])
    cmd = [HIPCC, f"--offload-arch={ARCH}", *ASAN_FLAGS, *map(str, sorted(objs)), f"-L{libdir}",
           f"-lpython{pyver}", *rp, "-o", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"asan harness link failed:\n{r.stderr[-4000:]}")
    stamp.write_text(key)
    if verbose:
        print(f"[dlap] built {out}")
    return out


if __name__ == "__main__":
    # --variant NAME [--file-flags FILE=FLAG,FLAG ...]: a named side build for A/B runs
    argv = sys.argv[1:]
    var, ffl = None, None
    if "--variant" in argv:
        var = argv[argv.index("--variant") + 1]
        ffl = {}
        for a in argv:
            if "=" in a and a.split("=", 1)[0].endswith((".hip", ".cpp")):
                f, fl = a.split("=", 1)
                ffl[f] = [x for x in fl.split(",") if x]
    if "--asan-harness" in argv:
        build_asan_harness(force="--force" in argv)
    else:
        build(force="--force" in argv, ubsan="--ubsan" in argv, debug="--debug" in argv, variant=var, file_flags=ffl)
