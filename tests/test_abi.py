"""CPU: the C-ABI library builds for gfx950, loads, and exports every symbol
include/dssgpu.h declares; without a device it fails loudly (no fallback)."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "dss_amd", "libdss_amd.so")


def declared_symbols():
    text = open(os.path.join(ROOT, "include", "dssgpu.h")).read()
    return sorted(set(re.findall(r"\b(dssg_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_entry_points():
    syms = declared_symbols()
    for s in ("dssg_create", "dssg_cover_batch", "dssg_cover_batch_device", "dssg_area_to_cell_ids",
              "dssg_index_build", "dssg_search", "dssg_search_operations", "dssg_search_isas",
              "dssg_search_subscriptions"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    if not os.path.exists(LIB):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "dss_amd", "csrc")])
    out = subprocess.check_output(["nm", "-D", "--defined-only", LIB]).decode()
    exported = set(re.findall(r"\bT (dssg_[a-z0-9_]+)", out))
    missing = [s for s in declared_symbols() if s not in exported]
    assert not missing, missing


def test_library_has_gfx950_code_object():
    out = subprocess.check_output(["strings", LIB]).decode()
    assert "amdgcn-amd-amdhsa--gfx950" in out


def test_no_device_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    from dss_amd import _lib
    with pytest.raises(_lib.DssgError):
        _lib.Context(0)
