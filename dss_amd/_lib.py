"""ctypes binding of libdss_amd.so (include/dssgpu.h).

The product path has no CPU fallback: if the gfx950 library is missing or no
gfx950 device is visible, every entry point raises.  The library lives in the
package directory (built in-tree by ``__graft_entry__.build()``).
"""
from __future__ import annotations

import ctypes as C
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
# DSS_AMD_LIB: load a differently-tuned build of the same library (kernel
# tuning experiments, tools/variants.sh); default: the in-tree build.
LIB_PATH = os.environ.get("DSS_AMD_LIB") or os.path.join(_HERE, "libdss_amd.so")

DSSG_OK = 0
DSSG_ERR_INVALID = 1
DSSG_ERR_CAPACITY = 2
DSSG_ERR_DEVICE = 3
DSSG_ERR_NOMEM = 4
DSSG_ERR_NO_DEVICE = 5

ST_OK = 0
ST_BAD_COORD_SET = 1
ST_NOT_ENOUGH_POINTS = 2
ST_ODD_COORDS = 3
ST_RADIUS = 4
ST_AREA_TOO_LARGE = 5

KIND_POLYGON = 0
KIND_CIRCLE = 1
KIND_POINTS = 2

TIME_NULL_START = -(2**63)
TIME_NULL_END = -(2**63)
TIME_NULL_END_Q = 2**63 - 1


class DssgError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"dssg error {code}: {msg}")
        self.code = code


class Cells(C.Structure):
    _fields_ = [("n", C.c_int64), ("offs", C.c_void_p), ("cells", C.c_void_p), ("status", C.c_void_p),
                ("area_km2", C.c_void_p), ("total_cells", C.c_int64)]


class Pairs(C.Structure):
    _fields_ = [("q", C.c_void_p), ("e", C.c_void_p), ("n", C.c_int64), ("n_tagged", C.c_int64)]


MAX_PARTS = 64
ROUTE_ROW_BYTES = 32
COMM_ID_BYTES = 128


class Volumes(C.Structure):
    """dssg_volumes: UnionVolumes4D results (device)."""
    _fields_ = [("n", C.c_int64), ("offs", C.c_void_p), ("cells", C.c_void_p), ("status", C.c_void_p),
                ("area_km2", C.c_void_p), ("alt_lo", C.c_void_p), ("alt_hi", C.c_void_p), ("t0", C.c_void_p),
                ("t1", C.c_void_p), ("has_footprint", C.c_void_p), ("total_cells", C.c_int64)]


class Batch(C.Structure):
    """dssg_batch: a received (unpacked) query batch."""
    _fields_ = [("n", C.c_int64), ("offs", C.c_void_p), ("cells", C.c_void_p), ("alt_lo", C.c_void_p),
                ("alt_hi", C.c_void_p), ("tlo", C.c_void_p), ("thi", C.c_void_p), ("home", C.c_void_p),
                ("qid", C.c_void_p)]


_lib = None
_lock = threading.Lock()


def load():
    """Load the HIP library; raises if it was not built."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise DssgError(DSSG_ERR_NO_DEVICE,
                            f"{LIB_PATH} missing: build it with __graft_entry__.build() (no CPU fallback exists)")
        # One HIP runtime per process: the torch wheel bundles its own
        # libamdhip64.so.7 (same SONAME as /opt/rocm's).  If torch is
        # importable, load it first so this library binds to the same runtime
        # torch's device buffers come from (torch is plumbing only).
        try:
            import torch  # noqa: F401
        except Exception:
            pass
        L = C.CDLL(LIB_PATH)
        P, vp = C.POINTER, C.c_void_p
        i32, i64, d, f = C.c_int32, C.c_int64, C.c_double, C.c_float
        u32, u64 = C.c_uint32, C.c_uint64
        L.dssg_create.argtypes = [C.c_int, P(vp)]
        L.dssg_destroy.argtypes = [vp]
        L.dssg_destroy.restype = None
        L.dssg_strerror.argtypes = [C.c_int]
        L.dssg_strerror.restype = C.c_char_p
        L.dssg_last_error.argtypes = [vp]
        L.dssg_last_error.restype = C.c_char_p
        L.dssg_cover_batch.argtypes = [vp, i64, P(i32), P(i64), P(d), P(d), P(f), P(i64), P(u64), i64, P(i64),
                                       P(i32), P(d)]
        L.dssg_cover_batch_device.argtypes = [vp, i64, vp, vp, vp, vp, vp, vp, P(Cells)]
        L.dssg_area_to_cell_ids.argtypes = [vp, C.c_char_p, P(u64), i64, P(i64), P(i32), P(d)]
        L.dssg_index_build.argtypes = [vp, i64, P(i64), P(u64), P(f), P(f), P(i64), P(i64), P(i32), P(vp)]
        L.dssg_index_build_device.argtypes = [vp, i64, vp, vp, vp, vp, vp, vp, vp, vp, P(vp)]
        L.dssg_index_build_range.argtypes = [vp, i64, P(i64), P(u64), P(f), P(f), P(i64), P(i64), P(i32), u64, u64,
                                             P(vp)]
        L.dssg_index_build_range_device.argtypes = [vp, i64, vp, vp, vp, vp, vp, vp, vp, u64, u64, vp, P(vp)]
        L.dssg_index_free.argtypes = [vp]
        L.dssg_index_free.restype = None
        L.dssg_index_num_postings.argtypes = [vp]
        L.dssg_index_num_postings.restype = i64
        L.dssg_index_num_cells.argtypes = [vp]
        L.dssg_index_num_cells.restype = i64
        L.dssg_index_grain.argtypes = [vp]
        L.dssg_index_grain.restype = C.c_int32
        L.dssg_search_device.argtypes = [vp, vp, i64, vp, vp, vp, vp, vp, vp, vp, vp, P(Pairs)]
        L.dssg_search.argtypes = [vp, vp, i64, P(i64), P(u64), P(f), P(f), P(i64), P(i64), P(i32), P(u32), P(u32),
                                  i64, P(i64)]
        L.dssg_search_operations.argtypes = [vp, vp, i64, P(i64), P(u64), P(f), P(f), P(i64), P(i64), i64, P(u32),
                                             P(u32), i64, P(i64)]
        L.dssg_search_isas.argtypes = [vp, vp, i64, P(i64), P(u64), P(i64), P(i64), P(u32), P(u32), i64, P(i64)]
        L.dssg_search_subscriptions.argtypes = [vp, vp, i64, P(i64), P(u64), P(i32), i64, P(u32), P(u32), i64,
                                                P(i64)]
        L.dssg_union_volumes_device.argtypes = [vp, i64, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, P(Volumes)]
        L.dssg_store_create.argtypes = [vp, i32, P(vp)]
        L.dssg_store_free.argtypes = [vp]
        L.dssg_store_free.restype = None
        L.dssg_store_upsert.argtypes = [vp, vp, i64, P(u32), P(i64), P(u64), P(f), P(f), P(i64), P(i64), P(i32)]
        L.dssg_store_delete.argtypes = [vp, vp, i64, P(u32), P(i32)]
        L.dssg_store_compact.argtypes = [vp, vp]
        L.dssg_store_stats.argtypes = [vp, P(i64), P(i64), P(i64), P(i64)]
        L.dssg_store_search.argtypes = [vp, vp, i64, P(i64), P(u64), P(f), P(f), P(i64), P(i64), P(i32), P(u32),
                                        P(u32), i64, P(i64)]
        L.dssg_store_max_subscription_count.argtypes = [vp, vp, i64, P(i64), P(u64), P(i32), i64, P(i64)]
        L.dssg_index_set_notification_index.argtypes = [vp, vp, P(i64)]
        L.dssg_index_get_notification_index.argtypes = [vp, vp, P(i64)]
        L.dssg_notify_subscriptions.argtypes = [vp, vp, i64, P(i64), P(u64), i64, P(u32), P(u32), P(i64), i64, P(i64)]
        L.dssg_owner_subscriptions.argtypes = [vp, vp, i64, P(i32), i64, P(u32), P(u32), i64, P(i64)]
        L.dssg_max_subscription_count.argtypes = [vp, vp, i64, P(i64), P(u64), P(i32), i64, P(i64)]
        L.dssg_route_plan_device.argtypes = [vp, i64, vp, vp, i32, vp, vp, P(i64), P(i64), P(i64)]
        L.dssg_route_fill_device.argtypes = [vp, i64, vp, vp, vp, vp, vp, vp, vp, vp]
        L.dssg_unpack_queries_device.argtypes = [vp, vp, i32, P(i64), P(i64), vp, P(Batch)]
        L.dssg_route_pairs_plan_device.argtypes = [vp, P(Batch), P(Pairs), i32, i32, vp, P(i64)]
        L.dssg_route_pairs_fill_device.argtypes = [vp, P(Batch), P(Pairs), vp, vp, vp, vp]
        L.dssg_unpack_pairs_device.argtypes = [vp, i64, vp, vp, vp, vp]
        L.dssg_phase_times.argtypes = [vp, P(d), P(d), P(d)]
        L.dssg_set_timing.argtypes = [vp, C.c_int]
        L.dssg_set_timing.restype = None
        L.dssg_set_tuning.argtypes = [vp, C.c_char_p, C.c_int64]
        L.dssg_join_events.argtypes = [vp, P(i64), P(i64), P(i64), P(i64)]
        L.dssg_join_longs.argtypes = [vp, P(i64), P(i64)]
        L.dssg_join_profile.argtypes = [vp, P(i64), C.c_int, P(C.c_int)]
        L.dssg_join_profile_name.argtypes = [C.c_int]
        L.dssg_join_profile_name.restype = C.c_char_p
        L.dssg_search_counters.argtypes = [vp, P(i64), P(i64), P(i64), P(i64), P(i64)]
        L.dssg_search_stats_device.argtypes = [vp, vp, i64, vp, vp, vp, P(i64), P(i64)]
        L.dssg_search_touched_device.argtypes = [vp, vp, i64, vp, vp, vp, P(i64)]
        L.dssg_index_info.argtypes = [vp, P(i64), P(i64), P(i64), P(i64), P(i64), P(i64)]
        L.dssg_copy_to_host.argtypes = [vp, vp, vp, C.c_size_t]
        L.dssg_copy_device.argtypes = [vp, vp, vp, C.c_size_t, vp]
        L.dssg_comm_unique_id.argtypes = [vp]
        L.dssg_comm_init.argtypes = [vp, C.c_int32, C.c_int32, vp, P(vp)]
        L.dssg_comm_free.argtypes = [vp]
        L.dssg_comm_free.restype = None
        L.dssg_comm_alltoallv_device.argtypes = [vp, vp, vp, vp, vp, vp, vp]
        L.dssg_batcher_create.argtypes = [C.c_int, vp, C.c_int32, C.c_int32, P(vp)]
        L.dssg_batcher_free.argtypes = [vp]
        L.dssg_batcher_free.restype = None
        L.dssg_batcher_search_operations.argtypes = [vp, C.c_int32, C.c_int64, vp, vp, C.c_float, C.c_float, C.c_float,
                                                      C.c_int64, C.c_int64, C.c_int64, vp, C.c_int64, P(C.c_int64),
                                                      P(C.c_int32), P(C.c_double)]
        L.dssg_batcher_stats.argtypes = [vp, P(C.c_int64), P(C.c_int64)]
        L.dssg_sharded_search_device.argtypes = [vp, vp, vp, vp, C.c_int64, vp, vp, vp, vp, vp, vp, vp, P(Pairs)]
        L.dssg_sharded_search_async_device.argtypes = [vp, vp, vp, vp, vp, C.c_int64, vp, vp, vp, vp, vp, vp, vp, vp,
                                                       P(Pairs)]
        L.dssg_sharded_stats.argtypes = [vp, P(d), P(i64)]
        L.dssg_radix_sort_device.argtypes = [vp, C.c_int, i64, C.c_int, vp, vp, vp, vp, vp, P(d)]
        L.dssg_selftest_scan.argtypes = [vp, i64, C.c_int, P(i64), P(i64)]
        L.dssg_selftest_math.argtypes = [vp, C.c_int, i64, P(d), P(d), P(d)]
        _lib = L
        return L


class Context:
    """One engine context (device, stream, scratch) -- `dssg_ctx`."""

    def __init__(self, device: int = 0):
        L = load()
        h = C.c_void_p()
        rc = L.dssg_create(device, C.byref(h))
        if rc != DSSG_OK:
            raise DssgError(rc, L.dssg_strerror(rc).decode())
        self.h = h
        self.L = L
        self.device = device

    def check(self, rc: int):
        if rc not in (DSSG_OK,):
            raise DssgError(rc, self.L.dssg_last_error(self.h).decode() or self.L.dssg_strerror(rc).decode())

    def set_tuning(self, key: str, value: int):
        """dssg_set_tuning (e.g. "tag_bucket_avg")."""
        self.check(self.L.dssg_set_tuning(self.h, key.encode(), int(value)))

    def join_profile(self) -> dict | None:
        """dssg_join_profile: the counting build's per-predicate sums since
        the last call ({name: count}); None from the shipped library."""
        buf = (C.c_int64 * 64)()
        n = C.c_int()
        self.check(self.L.dssg_join_profile(self.h, buf, 64, C.byref(n)))
        if n.value == 0:
            return None
        return {self.L.dssg_join_profile_name(i).decode(): int(buf[i]) for i in range(n.value)}

    def close(self):
        if getattr(self, "h", None):
            self.L.dssg_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_ctx = {}
_ctx_lock = threading.Lock()  # not _lock: Context() -> load() takes that one


def context(device: int = 0) -> Context:
    """The process's shared context for `device` (created once, under a lock,
    so concurrent first callers get the same one)."""
    with _ctx_lock:
        c = _ctx.get(device)
        if c is None:
            c = Context(device)
            _ctx[device] = c
        return c
