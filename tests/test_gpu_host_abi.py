"""The C ABI called from plain C the way the cgo binding (go/pkg/gpu) calls
it -- host buffers, no ctypes (tests/host/abi_test.c, built by
__graft_entry__.build()).  Its known answers: the reference covering KAT
(pkg/models/geo_test.go:10-55), the covering error statuses, and
hand-checked search / store answers."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_host_abi():
    exe = os.path.join(ROOT, "tests", "host", "abi_test")
    assert os.path.exists(exe), "tests/host/abi_test not built (run __graft_entry__.build())"
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "abi_test ok" in r.stdout
