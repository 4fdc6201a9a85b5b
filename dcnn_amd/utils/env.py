"""``.env`` loading and typed environment lookup (reference include/utils/env.hpp:41-137).

Parsing is done by the native runtime (``_native.load_env_file``); ``get_env`` mirrors the
reference's ``get_env<T>(key, default)``: the default's type decides the conversion, bools
accept 1/0/true/false/yes/no/on/off.
"""
from __future__ import annotations

import os
from typing import Any

from ..ops._ext import native


def load_env_file(path: str = "./.env", overwrite: bool = False) -> int:
    """Load KEY=VALUE pairs into ``os.environ``; returns the number of keys set (-1: no file)."""
    if not os.path.exists(path):
        return -1
    n = 0
    for k, v in native().parse_env_text(open(path).read()).items():
        if overwrite or k not in os.environ:
            os.environ[k] = v
            n += 1
    return n


_TRUE = {"1", "true", "yes", "on"}
_FALSE = {"0", "false", "no", "off"}


def get_env(key: str, default: Any = None, typ: type = None) -> Any:
    raw = os.environ.get(key)
    if raw is None:
        return default
    t = typ or (type(default) if default is not None else str)
    try:
        if t is bool:
            s = raw.strip().lower()
            if s in _TRUE:
                return True
            if s in _FALSE:
                return False
            return default
        if t is int:
            return int(float(raw))
        if t is float:
            return float(raw)
        return t(raw)
    except (TypeError, ValueError):
        return default
