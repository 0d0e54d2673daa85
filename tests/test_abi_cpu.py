"""The C-ABI library loads on a host without a GPU and exports exactly what
include/reth_hip.h declares; the ctypes binding matches the header.  No compute calls."""
import ctypes
import os
import re

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "reth_hip.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[\w\s\*]+?\b(rth_\w+)\s*\(", text, flags=re.M)
    return sorted(set(names))


def test_header_parses():
    names = declared_functions()
    assert "rth_sumtree_update" in names and "rth_td_huber" in names and len(names) >= 30


def test_library_exports_every_declared_symbol():
    from reth_amd import _lib

    lib = _lib.lib()  # loads libreth_hip.so (libamdhip64 resolves without a device)
    for name in declared_functions():
        assert hasattr(lib, name), f"{name} declared in reth_hip.h but not exported"
    assert lib.rth_version() == 100


def test_library_built_from_this_tree():
    """the compiled-in source id equals the tree's (build() rebuilds on any difference)"""
    from reth_amd import _lib

    assert _lib.lib().rth_build_id().decode() == _lib.source_build_id()
    assert _lib.library_build_id() == _lib.source_build_id()


def test_binding_covers_header():
    from reth_amd import _lib

    assert sorted(_lib.SIGNATURES) == declared_functions()


def test_binding_arg_counts_match_header():
    from reth_amd import _lib

    text = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    for name, (_, args) in _lib.SIGNATURES.items():
        m = re.search(rf"\b{name}\s*\((.*?)\)\s*;", text, flags=re.S)
        assert m, name
        params = [p for p in m.group(1).split(",") if p.strip() and p.strip() != "void"]
        assert len(params) == len(args), f"{name}: header {len(params)} args, binding {len(args)}"


def test_struct_layouts():
    from reth_amd._lib import ColDesc, Src

    assert ctypes.sizeof(ColDesc) == 24
    assert ctypes.sizeof(Src) == 32


def test_no_cpu_fallback_when_library_missing(monkeypatch, tmp_path):
    from reth_amd import _lib

    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "missing.so"))
    monkeypatch.setattr(_lib, "_lib", None)
    import pytest

    with pytest.raises(_lib.HipExtensionMissing):
        _lib.lib()
