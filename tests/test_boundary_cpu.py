"""C-ABI boundary checks that need no GPU: the library loads, exports exactly what
include/tw_hip.h declares, and the ctypes signatures agree with the header arity."""
import os
import re

import pytest

from conftest import REPO


def header_decls():
    src = open(os.path.join(REPO, "include", "tw_hip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    decls = {}
    for m in re.finditer(r"\bint\s+(tw_\w+)\s*\(([^;]*?)\)\s*;", src, flags=re.S):
        args = [a for a in m.group(2).split(",") if a.strip()]
        decls[m.group(1)] = len(args)
    return decls


def test_library_exports_every_header_symbol():
    from tw import _native
    lib = _native.lib()
    decls = header_decls()
    assert len(decls) >= 18
    for name in decls:
        assert hasattr(lib, name), name


def test_ctypes_signatures_match_header():
    from tw import _native
    decls = header_decls()
    assert set(decls) == set(_native.SIGNATURES)
    for name, n in decls.items():
        assert len(_native.SIGNATURES[name]) == n, name


def test_missing_library_fails_loudly(monkeypatch):
    from tw import _native
    monkeypatch.setattr(_native, "_lib", None)
    monkeypatch.setattr(_native, "LIB_PATH", "/nonexistent/libtw_hip.so")
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        _native.lib()
