"""Loader for the native runtime extension ``_cek``.

The extension is built in-tree (``python -m cekirdekler_amd.build_native``).
PyTorch, when importable, is imported first so the process has exactly one HIP
runtime (torch ships ``libamdhip64.so.7``, the same SONAME the extension links
against): RCCL, hiprtc and torch tensors then share one device context.
There is no silent fallback: if the extension is missing the import fails
loudly with the build command to run.
"""
from __future__ import annotations

import importlib
import os

try:  # one HIP runtime per process: let torch load it first
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is optional for the runtime
    torch = None

_mod = None


def _load():
    global _mod
    if _mod is not None:
        return _mod
    try:
        _mod = importlib.import_module("cekirdekler_amd._cek")
    except ImportError as e:
        if os.environ.get("CEK_AUTOBUILD", "1") != "0":
            from . import build_native

            build_native.build_extension()
            _mod = importlib.import_module("cekirdekler_amd._cek")
        else:
            raise ImportError(
                "cekirdekler_amd native extension _cek is not built; run "
                "`python -m cekirdekler_amd.build_native`") from e
    return _mod


cek = _load()
CekError = cek.CekError


def kernel_dir() -> str:
    return os.path.join(os.path.dirname(os.path.abspath(__file__)), "kernels")


def gpu_available() -> bool:
    return cek.gpu_count() > 0
