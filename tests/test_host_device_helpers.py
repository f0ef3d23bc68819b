"""CPU: the device S2 helpers (dss_amd/csrc/*.cuh, compiled as host code by
hipcc) agree with the oracle -- catches labelling bugs without a GPU."""
import ctypes as C
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def ids_output(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("host") / "ids_check")
    subprocess.check_call(["/opt/rocm/bin/hipcc", "-std=c++17", "-O2", "-ffp-contract=off", "-o", exe,
                           os.path.join(ROOT, "tests", "host", "ids_check.cpp")])
    return subprocess.check_output([exe]).decode().split("\n")


def test_cell_ids_and_orientation(oracle, ids_output):
    L = oracle.lib()
    n = 0
    for line in ids_output:
        if not line.strip():
            continue
        face, i, j, level, cid, o = (int(x) for x in line.split())
        oo = C.c_int()
        ref = L.orc_cellid_from_face_ij_level(face, i, j, level, C.byref(oo))
        assert cid == ref, (face, i, j, level)
        assert o == oo.value, (face, i, j, level)
        n += 1
    assert n == 2000
