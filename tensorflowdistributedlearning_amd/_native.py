"""Loader for the in-tree native extension (HIP kernels + C++ runtime).

The extension ``_C*.so`` is built by ``build_ext.py`` (``hipcc --offload-arch=gfx950``) and lives
next to this file, so it travels with the repository snapshot to the GPU box.

Dispatch rule used by every op in :mod:`tensorflowdistributedlearning_amd.ops`:

* tensor on a HIP device  -> the hand-written gfx950 kernel in ``_C`` (no silent fallback: if the
  extension is missing the op raises);
* tensor on the CPU       -> the plain PyTorch fp32 reference of the same op (the numerics oracle,
  also used by the CPU plumbing configuration).

The reference's runtime is TF 1.x's C++ executor/cuDNN/NCCL; this
module is the single entry point to our MI355X-native replacement of those.
"""
from __future__ import annotations

import glob
import importlib.util
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
_EXT = None
_EXT_ERR = None


def _find_so(name):
    cands = sorted(glob.glob(os.path.join(_HERE, name + "*.so")))
    return cands[0] if cands else None


def load():
    """Import and return the native extension module (cached). Raises if unavailable."""
    global _EXT, _EXT_ERR
    if _EXT is not None:
        return _EXT
    if _EXT_ERR is not None:
        raise _EXT_ERR
    # TDL_EXT_SO: load another build of the same extension (same-box A/B of kernel changes,
    # dev/scripts/ab_build.sh); the module name stays tensorflowdistributedlearning_amd._C
    so = os.environ.get("TDL_EXT_SO") or _find_so("_C")
    if so is None:
        _EXT_ERR = ImportError(
            "native extension _C.so not built; run `python build_ext.py` (hipcc --offload-arch=gfx950)")
        raise _EXT_ERR
    import torch  # noqa: F401  (libtorch must be loaded before the extension)
    spec = importlib.util.spec_from_file_location("tensorflowdistributedlearning_amd._C", so)
    mod = importlib.util.module_from_spec(spec)
    try:
        spec.loader.exec_module(mod)
    except Exception as e:  # pragma: no cover - depends on the build
        _EXT_ERR = ImportError(f"failed to load native extension {so}: {e}")
        raise _EXT_ERR
    _EXT = mod
    return mod


def available() -> bool:
    try:
        load()
        return True
    except ImportError:
        return False


def ext():
    """Alias of :func:`load` used inside ops (reads better at call sites)."""
    return _EXT if _EXT is not None else load()


def so_path():
    return _find_so("_C")
