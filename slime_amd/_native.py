"""ctypes binding of libslime_rs.so (the C-ABI in include/slime_rs.h).

The library is built in-tree (``make`` / ``__graft_entry__.build()``) at
slime_amd/lib/libslime_rs.so.  There is no fallback: if it is missing, every
import of this module raises.

HIP runtime ownership: PyTorch-ROCm ships its own libamdhip64 with the same
soname (libamdhip64.so.7) as /opt/rocm's.  If torch is importable it is
imported FIRST, so the dynamic loader binds our library to torch's already
loaded runtime and device pointers/streams from torch tensors are valid here.
"""
from __future__ import annotations

import contextlib
import ctypes
import os

try:  # noqa: SIM105 - see module docstring
    import torch  # noqa: F401
except ImportError:  # pragma: no cover - torch is part of the image
    torch = None

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "libslime_rs.so")

if not os.path.exists(LIB_PATH):
    raise ImportError(f"{LIB_PATH} is not built; run `make` at the repo root or __graft_entry__.build()")

lib = ctypes.CDLL(LIB_PATH)

c_u32p = ctypes.POINTER(ctypes.c_uint32)
c_u64p = ctypes.POINTER(ctypes.c_uint64)
c_intp = ctypes.POINTER(ctypes.c_int)
c_u8p = ctypes.POINTER(ctypes.c_uint8)


class Call(ctypes.Structure):
    """slime_rs_call_t: per-call device and failure-detail buffer (the *_ex forms)."""
    _fields_ = [("device", ctypes.c_int), ("detail", ctypes.c_char_p), ("detail_cap", ctypes.c_size_t)]


class CacheStats(ctypes.Structure):
    """slime_rs_cache_stats_t."""
    _fields_ = [("live", ctypes.c_uint64), ("capacity", ctypes.c_uint64), ("hits", ctypes.c_uint64),
                ("misses", ctypes.c_uint64), ("evictions", ctypes.c_uint64), ("device_tables", ctypes.c_uint64)]


ANY_DEVICE = -1


class HostStats(ctypes.Structure):
    """slime_rs_host_stats_t."""
    _fields_ = [(f, ctypes.c_uint64) for f in ("calls", "windows", "copy_in_us", "enqueue_us", "wait_us",
                                                "copy_out_us", "total_us")]


class AllocInfo(ctypes.Structure):
    """slime_rs_alloc_info_t: how slime_rs_device_alloc placed a buffer."""
    _fields_ = [("kind", ctypes.c_int), ("probes", ctypes.c_int), ("chosen", ctypes.c_int),
                ("chunk_bytes", ctypes.c_uint64), ("probe_gbs", ctypes.c_double * 4),
                ("probe_chunk", ctypes.c_uint64 * 4)]


class Layout(ctypes.Structure):
    """slime_rs_layout_t: shard s of object o at base + o*obj_stride + s*shard_stride."""
    _fields_ = [("obj_stride", ctypes.c_uint64), ("shard_stride", ctypes.c_uint64)]


# (name, restype, argtypes) for every symbol include/slime_rs.h declares.
SIGNATURES = [
    ("slime_rs_status_string", ctypes.c_char_p, [ctypes.c_int]),
    ("slime_rs_last_error", ctypes.c_char_p, []),
    ("slime_rs_version", ctypes.c_char_p, []),
    ("slime_rs_device_count", ctypes.c_int, []),
    ("slime_rs_select_device", ctypes.c_int, [ctypes.c_int]),
    ("slime_rs_selected_device", ctypes.c_int, []),
    ("slime_rs_kernel_pipeline", ctypes.c_int, [ctypes.c_int]),
    ("slime_rs_kernel_schedule", ctypes.c_int, [ctypes.c_int]),
    ("slime_rs_kernel_matrix_cores", ctypes.c_int, [ctypes.c_int]),
    ("slime_rs_switch_bits", ctypes.c_int, [ctypes.c_int]),
    ("slime_rs_device_alloc", ctypes.c_int, [ctypes.c_int, ctypes.c_uint64, ctypes.POINTER(ctypes.c_void_p)]),
    ("slime_rs_device_free", ctypes.c_int, [ctypes.c_void_p]),
    ("slime_rs_device_alloc_info", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(AllocInfo)]),
    ("slime_rs_probe_placement", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.POINTER(ctypes.c_double)]),
    ("slime_rs_placement_threshold", ctypes.c_double, []),
    ("slime_gf_max_val", ctypes.c_uint32, []),
    ("slime_gf_minverse", ctypes.c_uint32, [ctypes.c_uint32]),
    ("slime_gf_raise", ctypes.c_uint32, [ctypes.c_uint32, ctypes.c_uint32]),
    ("slime_gf_map_to_gf", ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, c_u32p, ctypes.c_void_p]),
    ("slime_gf_map_to_gf_with", ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p]),
    ("slime_gf_map_from_gf", ctypes.c_int, [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]),
    ("slime_gf_seed", None, [ctypes.c_uint64]),
    ("slime_gf_codec_placement", ctypes.c_int, [ctypes.c_int]),
    ("slime_gf_codec_info", ctypes.c_int, [ctypes.POINTER(ctypes.c_char_p), c_intp]),
    ("slime_rs_vandermonde_matrix", ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_void_p]),
    ("slime_rs_parity_matrix", ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_void_p]),
    ("slime_rs_parity_matrix_cached", ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.POINTER(c_u32p)]),
    ("slime_rs_solve_sub_identity", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]),
    ("slime_rs_invert_matrix", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]),
    ("slime_rs_create_parity", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]),
    ("slime_rs_create_parities", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]),
    ("slime_rs_recover_data", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]),
    ("slime_rs_plan_encode", ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    ("slime_rs_plan_reconstruct", ctypes.c_int,
     [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
      ctypes.POINTER(ctypes.c_void_p)]),
    ("slime_rs_plan_matrix", ctypes.c_int,
     [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p)]),
    ("slime_rs_plan_execute", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_void_p, Layout, ctypes.c_void_p, Layout, ctypes.c_uint64, ctypes.c_uint64,
      ctypes.c_void_p]),
    ("slime_rs_plan_set_outputs", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    ("slime_rs_plan_shape", ctypes.c_int, [ctypes.c_void_p, c_intp, c_intp]),
    ("slime_rs_plan_coefficients", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    ("slime_rs_plan_destroy", ctypes.c_int, [ctypes.c_void_p]),
    ("slime_rs_encode_objects", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p,
      ctypes.c_void_p, ctypes.c_void_p]),
    ("slime_rs_resolve_fallbacks", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p,
      ctypes.c_void_p, ctypes.c_void_p, c_intp]),
    ("slime_rs_decode_objects", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p,
      ctypes.c_void_p]),
    ("slime_rs_encode_objects_chunked", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    ("slime_rs_encode_objects_phased", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    ("slime_rs_resolve_fallbacks_chunked", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, c_intp]),
    ("slime_rs_decode_objects_chunked", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
      ctypes.c_void_p, ctypes.c_void_p]),
    ("slime_rs_chunk_size", ctypes.c_uint64, [ctypes.c_uint64, ctypes.c_int]),
    ("slime_rs_write_chunks", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, c_u32p]),
    ("slime_rs_reconstruct", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64,
      ctypes.c_void_p]),
    ("slime_gf_pack_device", ctypes.c_int,
     [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
      ctypes.c_void_p]),
    ("slime_gf_unpack_device", ctypes.c_int,
     [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]),
    ("slime_rs_fill_symbols", ctypes.c_int,
     [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p]),
    # *_ex forms (per-call context)
    ("slime_rs_create_parity_ex", ctypes.c_int,
     [ctypes.POINTER(Call), ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]),
    ("slime_rs_create_parities_ex", ctypes.c_int,
     [ctypes.POINTER(Call), ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]),
    ("slime_rs_recover_data_ex", ctypes.c_int,
     [ctypes.POINTER(Call), ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
      ctypes.c_void_p]),
    ("slime_rs_write_chunks_ex", ctypes.c_int,
     [ctypes.POINTER(Call), ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, c_u32p]),
    ("slime_rs_reconstruct_ex", ctypes.c_int,
     [ctypes.POINTER(Call), ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint32,
      ctypes.c_uint64, ctypes.c_void_p]),
    ("slime_gf_map_to_gf_ex", ctypes.c_int,
     [ctypes.POINTER(Call), ctypes.c_void_p, ctypes.c_uint64, c_u32p, ctypes.c_void_p]),
    ("slime_gf_map_to_gf_with_ex", ctypes.c_int,
     [ctypes.POINTER(Call), ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p]),
    ("slime_gf_map_from_gf_ex", ctypes.c_int,
     [ctypes.POINTER(Call), ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]),
    ("slime_rs_parity_matrix_ex", ctypes.c_int, [ctypes.POINTER(Call), ctypes.c_int, ctypes.c_int, ctypes.c_void_p]),
    ("slime_rs_vandermonde_matrix_ex", ctypes.c_int,
     [ctypes.POINTER(Call), ctypes.c_int, ctypes.c_int, ctypes.c_void_p]),
    ("slime_rs_solve_sub_identity_ex", ctypes.c_int,
     [ctypes.POINTER(Call), ctypes.c_void_p, ctypes.c_int, ctypes.c_int]),
    ("slime_rs_invert_matrix_ex", ctypes.c_int, [ctypes.POINTER(Call), ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]),
    # plan cache / device pool
    ("slime_rs_plan_cache_stats", ctypes.c_int, [ctypes.POINTER(CacheStats)]),
    ("slime_rs_plan_cache_capacity", ctypes.c_int, [ctypes.c_uint64]),
    ("slime_rs_pool_calls", ctypes.c_int, [ctypes.c_int, c_u64p, c_intp]),
    ("slime_rs_host_call_slots", ctypes.c_int, []),
    ("slime_rs_ticket_sets", ctypes.c_int, [ctypes.c_int, c_u64p, c_u64p]),
    ("slime_rs_schedule_counts", ctypes.c_int, [ctypes.c_int, c_u64p, c_u64p]),
    ("slime_rs_host_stats", ctypes.c_int, [ctypes.POINTER(HostStats), ctypes.c_int]),
    # chunk and object digests (host)
    ("slime_rs_sha256", ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]),
    ("slime_rs_chunk_digests", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]),
    ("slime_rs_write_chunks_digest", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, c_u32p, ctypes.c_void_p,
      ctypes.c_void_p]),
    ("slime_rs_reconstruct_verify", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64,
      ctypes.c_void_p, ctypes.c_void_p]),
    ("slime_rs_digest_info", ctypes.c_int, [c_intp, c_intp]),
    ("slime_rs_write_chunks_digest_ex", ctypes.c_int,
     [ctypes.POINTER(Call), ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, c_u32p,
      ctypes.c_void_p, ctypes.c_void_p]),
    ("slime_rs_reconstruct_verify_ex", ctypes.c_int,
     [ctypes.POINTER(Call), ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint32,
      ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]),
]

for _name, _res, _args in SIGNATURES:
    _fn = getattr(lib, _name)
    _fn.restype = _res
    _fn.argtypes = _args

# Status codes (enum slime_rs_status).
OK = 0
ERR_VARYING_LENGTH = 1
ERR_LEN_MISMATCH = 2
ERR_EMPTY = 3
ERR_NO_INDICES = 4
ERR_SINGULAR_NONZERO = 5
ERR_SINGULAR_ONE = 6
ERR_SINGULAR_ZERO = 7
ERR_INDEX_RANGE = 8
ERR_INVALID_ARG = 9
ERR_NO_DEVICE = 10
ERR_HIP = 11
ERR_MAPPING_FALLBACK = 12
ERR_BAD_HASH = 13

PANIC_CODES = range(1, 9)


class Panic(Exception):
    """Raised where the reference panics; str(e) is the reference's panic text."""

    def __init__(self, code: int, message: str, detail: str = ""):
        super().__init__(message)
        self.code = code
        self.detail = detail


class NativeError(RuntimeError):
    """A non-panic failure of the native library (no device, HIP error, misuse)."""

    def __init__(self, code: int, detail: str):
        super().__init__(f"slime_rs error {code}: {detail}")
        self.code = code


class BadHash(NativeError):
    """reconstruct's ErrBadHash: "bad checksum after reconstruction" (multi_store.go:26,244-249)."""


def check(rc: int) -> None:
    """Turn a C-ABI status into the reference's behaviour (panic) or an error."""
    if rc == OK:
        return
    detail = lib.slime_rs_last_error().decode()
    if rc in PANIC_CODES:
        msg = lib.slime_rs_status_string(rc).decode()
        if rc == ERR_INDEX_RANGE and detail:
            msg = detail  # Go's runtime panic text carries the index
        raise Panic(rc, msg, detail)
    if rc == ERR_BAD_HASH:
        raise BadHash(rc, detail)
    raise NativeError(rc, detail)


def device_count() -> int:
    return int(lib.slime_rs_device_count())


def plan_cache_stats() -> dict:
    st = CacheStats()
    check(lib.slime_rs_plan_cache_stats(ctypes.byref(st)))
    return {f: int(getattr(st, f)) for f, _ in CacheStats._fields_}


def set_plan_cache_capacity(cap: int) -> None:
    check(lib.slime_rs_plan_cache_capacity(cap))


def host_stats(reset: bool = False) -> dict:
    """Split of the host pipeline's wall time (microseconds) since start / last reset."""
    st = HostStats()
    check(lib.slime_rs_host_stats(ctypes.byref(st), int(reset)))
    return {f: int(getattr(st, f)) for f, _ in HostStats._fields_}


def digest_info() -> tuple[bool, int]:
    """(SHA-256 runs on the CPU's SHA extensions, digest threads besides the caller)."""
    e, t = ctypes.c_int(), ctypes.c_int()
    check(lib.slime_rs_digest_info(ctypes.byref(e), ctypes.byref(t)))
    return bool(e.value), int(t.value)


def codec_info() -> dict:
    """The host codec's instruction set and the threads its passes run on (the copy pool + the caller)."""
    isa, th = ctypes.c_char_p(), ctypes.c_int()
    check(lib.slime_gf_codec_info(ctypes.byref(isa), ctypes.byref(th)))
    return {"isa": isa.value.decode(), "threads": int(th.value)}


def alloc_info(ptr: int) -> dict:
    """Placement of a slime_rs_device_alloc buffer (its base): probed rates and the one kept."""
    st = AllocInfo()
    check(lib.slime_rs_device_alloc_info(ctypes.c_void_p(ptr), ctypes.byref(st)))
    n = st.probes
    kinds = ["hipMalloc" if st.probe_chunk[i] == 0 else f"{st.probe_chunk[i] >> 20} MiB chunks" for i in range(n)]
    return {"kept": ("hipMalloc" if st.kind == 1 else f"{st.chunk_bytes >> 20} MiB chunks"),
            "probes": [{"placement": kinds[i], "probe_gbs": round(st.probe_gbs[i], 1)} for i in range(n)],
            "retries": max(0, n - 1), "chosen": st.chosen if n else None}


def ticket_sets(device: int) -> tuple[int, int]:
    """(ticket-counter sets allocated on `device`, sets held by unfinished launches or captured graphs)."""
    s, h = ctypes.c_uint64(), ctypes.c_uint64()
    check(lib.slime_rs_ticket_sets(device, ctypes.byref(s), ctypes.byref(h)))
    return int(s.value), int(h.value)


def schedule_counts(device: int) -> tuple[int, int]:
    """(launches that ran the dynamic schedule on a counter set, launches that asked for one and got none)."""
    d, f = ctypes.c_uint64(), ctypes.c_uint64()
    check(lib.slime_rs_schedule_counts(device, ctypes.byref(d), ctypes.byref(f)))
    return int(d.value), int(f.value)


@contextlib.contextmanager
def on_device(device: int | None):
    """Route the calling thread's host entry points (rs.*, gf.*, objects.*) to
    `device` for the block (slime_rs_select_device); None leaves the routing as
    it is (the device pool picks).  A rank that owns one GPU wraps its host
    calls in this, so they never spread onto other ranks' devices.  On exit
    the thread's previous selection is restored -- whether it came from an
    enclosing block or a direct slime_rs_select_device call."""
    if device is None:
        yield
        return
    prev = int(lib.slime_rs_selected_device())
    check(lib.slime_rs_select_device(int(device)))
    try:
        yield
    finally:
        check(lib.slime_rs_select_device(prev))


def pool_calls(device: int) -> tuple[int, int]:
    """(host calls routed to `device` by the device pool so far, calls in flight there)."""
    c, f = ctypes.c_uint64(), ctypes.c_int()
    check(lib.slime_rs_pool_calls(device, ctypes.byref(c), ctypes.byref(f)))
    return int(c.value), int(f.value)
