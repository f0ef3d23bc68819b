"""CPU: the oracle reproduces the committed golden fixtures bit for bit
(guards the checker itself against drift)."""
import numpy as np


def test_covering_golden(oracle, golden_covering):
    g = golden_covering
    offs, cells, status, area = oracle.cover_batch(g["kind"], g["voff"], g["lat"], g["lng"], g["radius_m"])
    assert np.array_equal(status, g["status"])
    assert np.array_equal(offs, g["offs"])
    assert np.array_equal(cells, g["cells"])
    assert np.array_equal(area.view(np.uint64), g["area_km2"].view(np.uint64))


def test_coverings_sorted_unique_level13(golden_covering):
    g = golden_covering
    cells = g["cells"]
    lsb = cells & (~cells + np.uint64(1))
    assert np.all(lsb == np.uint64(1 << 34))
    for i in range(len(g["kind"])):
        c = cells[g["offs"][i]:g["offs"][i + 1]]
        assert np.all(np.diff(c.astype(object)) > 0) if len(c) > 1 else True


def test_search_golden(oracle, golden_search):
    g = golden_search
    tlo = np.maximum(g["q_start"], g["now"])
    rq, re = oracle.search(g["e_offs"], g["e_cells"], g["e_alt_lo"], g["e_alt_hi"], g["e_t0"], g["e_t1"],
                           g["e_owner"], g["q_offs"], g["q_cells"], g["q_alt_lo"], g["q_alt_hi"], tlo, g["q_end"])
    assert np.array_equal(rq, g["pairs_q"]) and np.array_equal(re, g["pairs_e"])
