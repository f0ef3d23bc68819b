"""GPU: the hand-written LSD radix sort (radix.hip) through the C ABI
(`dssg_radix_sort_device`) equals a stable sort on the low `bits` bits --
the ordering the index build relies on for `scd_cells_operations`'s
(cell_id, operation_id) primary key (pkg/scd/store/cockroach/store.go:140-147)
and the join's key grouping.  Bit-exact: keys and carried values."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def gpu_sort(keys, vals, bits, key_bytes):
    import torch

    from dss_amd import _lib
    ctx = _lib.context()
    n = len(keys)
    kt = np.int64 if key_bytes == 8 else np.int32
    dk = torch.from_numpy(np.ascontiguousarray(keys).view(kt).copy()).cuda()
    dko = torch.empty_like(dk)
    dv = dvo = None
    if vals is not None:
        dv = torch.from_numpy(np.ascontiguousarray(vals).view(np.int32).copy()).cuda()
        dvo = torch.empty_like(dv)
    torch.cuda.synchronize()
    ms = C.c_double(0)
    p = lambda t: C.c_void_p(t.data_ptr()) if t is not None and n else None  # noqa: E731
    ctx.check(ctx.L.dssg_radix_sort_device(ctx.h, key_bytes, n, bits, p(dk), p(dko), p(dv), p(dvo), None,
                                           C.byref(ms)))
    ko = dko.cpu().numpy().view(np.uint64 if key_bytes == 8 else np.uint32)
    vo = dvo.cpu().numpy().view(np.uint32) if dvo is not None else None
    return ko, vo, ms.value


def ref_sort(keys, vals, bits):
    mask = (1 << bits) - 1 if bits < 64 else (1 << 64) - 1
    order = np.argsort(keys & keys.dtype.type(mask), kind="stable")
    return keys[order], (vals[order] if vals is not None else None)


CASES = [  # (n, bits, key_bytes, with values)
    (0, 64, 8, True), (1, 64, 8, True), (100, 7, 8, True), (4096, 64, 8, True), (4097, 13, 8, True),
    (250_000, 64, 8, True), (1_000_003, 29, 8, False), (300_000, 64, 8, False), (5, 0, 8, True),
    (1_234_567, 18, 4, True), (77_777, 32, 4, True), (4096 * 3 + 17, 1, 4, True), (65_536, 9, 4, True),
]


@pytest.mark.parametrize("n,bits,key_bytes,with_vals", CASES)
def test_radix_sort_matches_stable_sort(n, bits, key_bytes, with_vals):
    rng = np.random.default_rng(n * 131 + bits)
    dt = np.uint64 if key_bytes == 8 else np.uint32
    keys = rng.integers(0, np.iinfo(dt).max, size=n, dtype=dt, endpoint=True)
    if n > 1000:  # heavy duplication + sorted runs, as group ids and cell ids have
        keys[: n // 3] = keys[: n // 3] % dt(97)
        keys[n // 3: n // 2] = np.sort(keys[n // 3: n // 2])
    vals = np.arange(n, dtype=np.uint32) if with_vals else None
    ko, vo, _ = gpu_sort(keys, vals, bits, key_bytes)
    rk, rv = ref_sort(keys, vals, bits)
    assert np.array_equal(ko, rk)
    if with_vals:
        assert np.array_equal(vo, rv)


def test_radix_sort_level13_cells():
    """Level-13 cell ids of one metro (face 4, high bits shared) with entity ids:
    the index build's 64-bit (cell, entity) sort."""
    from dss_amd import workload as W
    from oracle import oracle as O
    O.build()
    _, _, _, it, _, _ = W.config(0, scale=0.05)
    offs, cells = O.cover_batch(it.kind, it.voff, it.lat, it.lng, it.radius_m)[:2]
    ent = np.repeat(np.arange(len(offs) - 1, dtype=np.uint32), np.diff(offs))
    ko, vo, _ = gpu_sort(cells.astype(np.uint64), ent, 64, 8)
    rk, rv = ref_sort(cells.astype(np.uint64), ent, 64)
    assert np.array_equal(ko, rk) and np.array_equal(vo, rv)


PACKED = [  # (name, n, bits, key high bits, key low constant, key shift, value max): 8-B keys with values
    ("level-13 ids, packed", 300_000, 64, 29, (1 << 34), 35, 2**32 - 1),
    ("one pass, packed", 100_000, 64, 6, 0x123, 40, 2**32 - 1),
    ("bits < 64, unsorted high bits kept", 200_000, 50, 10, 0x28, 38, 2**30),
    ("values too wide: plain sort", 150_000, 64, 30, 0x7, 20, 2**31),
    ("values fit the low bits", 150_000, 64, 30, 0x0, 20, 2**16),
]


@pytest.mark.parametrize("name,n,bits,hb,low,sh,vmax", PACKED)
def test_radix_sort_packed_words(name, n, bits, hb, low, sh, vmax):
    """The packed 8-B path (key bits below the lowest varying one constant and
    wide enough for every value) and its fallback both equal the stable sort:
    keys restored with their constant low bits and any unsorted high bits,
    values carried."""
    rng = np.random.default_rng(n + hb)
    k = (rng.integers(0, 1 << hb, n, dtype=np.uint64) << np.uint64(sh)) | np.uint64(low)
    k[: n // 4] = k[: n // 4] % np.uint64(1 << (sh + 3)) | np.uint64(low)  # duplicates
    if bits < 64:  # random bits above the sorted ones ride along unsorted
        k |= rng.integers(0, 1 << (64 - bits), n, dtype=np.uint64) << np.uint64(bits)
    vals = rng.integers(0, vmax, n, dtype=np.uint64, endpoint=True).astype(np.uint32)
    ko, vo, _ = gpu_sort(k, vals, bits, 8)
    rk, rv = ref_sort(k, vals, bits)
    assert np.array_equal(ko, rk), name
    assert np.array_equal(vo, rv), name


def test_radix_sort_rejects_aliasing():
    from dss_amd import _lib
    ctx = _lib.context()
    import torch
    d = torch.zeros(16, dtype=torch.int64, device="cuda")
    rc = ctx.L.dssg_radix_sort_device(ctx.h, 8, 16, 64, C.c_void_p(d.data_ptr()), C.c_void_p(d.data_ptr()), None, None,
                                      None, None)
    assert rc == _lib.DSSG_ERR_INVALID


@pytest.mark.parametrize("key_bytes", [8, 4])
def test_radix_sort_constant_and_high_bit_keys(key_bytes):
    """Keys equal on every sorted bit (stable = identity) and keys that differ
    only in their top bits (the varying-span shortcut skips the low passes)."""
    dt = np.uint64 if key_bytes == 8 else np.uint32
    top = 8 * key_bytes
    n = 70_001
    vals = np.arange(n, dtype=np.uint32)[::-1].copy()
    same = np.full(n, dt(0xABCD1234), dtype=dt)
    ko, vo, _ = gpu_sort(same, vals, top, key_bytes)
    assert np.array_equal(ko, same) and np.array_equal(vo, vals)
    rng = np.random.default_rng(11)
    high = (rng.integers(0, 8, n).astype(dt) << dt(top - 3)) | dt(5)
    ko, vo, _ = gpu_sort(high, vals, top, key_bytes)
    rk, rv = ref_sort(high, vals, top)
    assert np.array_equal(ko, rk) and np.array_equal(vo, rv)
    ko, vo, _ = gpu_sort(high, vals, top - 3, key_bytes)  # varying bits outside the sorted range
    assert np.array_equal(ko, high) and np.array_equal(vo, vals)


@pytest.mark.parametrize("n,shift", [(0, 0), (1, 0), (2047, 1), (2048, 0), (2049, 1), (4096 * 7 + 3, 0),
                                     (1_000_003, 1), (1_000_003, 0), (6_700_001, 3)])
def test_exclusive_scan_matches_cumsum(n, shift):
    """The hand-written int64 exclusive scan (scan.hip) behind every CSR
    offset array: out[0] = 0, out[k + 1] = sum(in[:k + 1]), aligned and
    8-byte-misaligned inputs, single and multi-tile sizes."""
    from dss_amd import _lib
    ctx = _lib.context()
    rng = np.random.default_rng(n + shift)
    x = rng.integers(0, 1 << 20, size=n, dtype=np.int64)
    out = np.full(n + 1, -1, dtype=np.int64)
    P = lambda a: a.ctypes.data_as(C.POINTER(C.c_int64))  # noqa: E731
    ctx.check(ctx.L.dssg_selftest_scan(ctx.h, n, shift, P(x) if n else None, P(out)))
    ref = np.concatenate([[0], np.cumsum(x)]).astype(np.int64)
    assert np.array_equal(out, ref)
