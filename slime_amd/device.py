"""Device-resident batch API (the hot path) over torch tensors in HBM.

Objects are laid out ``[object][shard][L]`` uint32 symbols (torch has no
general uint32 arithmetic, so buffers are ``torch.int32`` tensors holding the
same bits).  A plan carries the coefficient rows on the device; executing it
launches the gfx950 kernel on the given (default: current) torch stream.
PyTorch here is plumbing only: memory, streams, events.
"""
from __future__ import annotations

import ctypes
import logging
from typing import Optional, Sequence

import numpy as np
import torch

from . import _native as N

lib = N.lib


def _stream_handle(device: int, stream) -> ctypes.c_void_p:
    """A torch stream (default: the device's current one), or a raw hipStream_t
    handle given as an int (e.g. 2 = hipStreamPerThread)."""
    if isinstance(stream, int):
        return ctypes.c_void_p(stream)
    s = stream if stream is not None else torch.cuda.current_stream(device)
    return ctypes.c_void_p(s.cuda_stream)


def _dev_index(t: torch.Tensor) -> int:
    if t.device.type != "cuda":
        raise ValueError("slime_amd.device needs tensors on a HIP device (torch 'cuda')")
    return t.device.index if t.device.index is not None else torch.cuda.current_device()


_TYPESTR = {torch.int32: "<i4", torch.uint8: "|u1", torch.int64: "<i8", torch.uint32: "<u4"}


_deferred_frees: list = []  # buffers dropped while a graph capture was running
_log = logging.getLogger("slime_amd")
# Storage bases whose placement is known: slime_rs_device_alloc buffers (probed
# and re-placed when created) and caller buffers probed by probe_placement.
_known_placement: set = set()
_warned_placement: set = set()
PLACEMENT_WARN_BYTES = 16 << 30
# probe_placement's slow mode: below this fraction of the allocator's
# threshold (5300-5700 GB/s vs fast placements at 5950-6370 on this
# project's boxes, profiles/r06/s34_placement_aim).
SLOW_PLACEMENT = 0.92


def _capturing() -> bool:
    try:
        return bool(torch.cuda.is_current_stream_capturing())
    except Exception:  # pragma: no cover - no device / interpreter shutdown
        return False


def release_deferred() -> None:
    """Free the device buffers whose last tensor died during a graph capture
    (called on the next allocation or drop outside a capture)."""
    while _deferred_frees and not _capturing():
        lib.slime_rs_device_free(ctypes.c_void_p(_deferred_frees.pop()))


class _DeviceBuffer:
    """A slime_rs_device_alloc buffer exposed through __cuda_array_interface__;
    freed when the last tensor viewing it is gone (torch.as_tensor keeps its
    source object alive for the tensor's lifetime).  The free waits for the
    device (hipDeviceSynchronize: work queued on any stream may still touch
    the range), which a graph capture forbids: a buffer dropped during a
    capture on this thread's current stream is freed at the next allocation
    or drop outside one (release_deferred)."""

    def __init__(self, device: int, numel: int, dtype: torch.dtype):
        release_deferred()
        itemsize = torch.empty((), dtype=dtype).element_size()
        p = ctypes.c_void_p()
        N.check(lib.slime_rs_device_alloc(device, max(1, numel * itemsize), ctypes.byref(p)))
        self.ptr = p.value
        _known_placement.add(self.ptr)
        self.__cuda_array_interface__ = {"shape": (numel,), "typestr": _TYPESTR[dtype], "data": (self.ptr, False),
                                         "strides": None, "version": 3, "stream": None}

    def __del__(self):
        if getattr(self, "ptr", None):
            try:
                if _capturing():
                    _deferred_frees.append(self.ptr)
                else:
                    _known_placement.discard(self.ptr)
                    lib.slime_rs_device_free(ctypes.c_void_p(self.ptr))  # waits for the device, then unmaps
                    release_deferred()
            except Exception:  # pragma: no cover - interpreter shutdown
                pass
            self.ptr = None


def device_empty(numel: int, dtype: torch.dtype = torch.int32, device: int = 0) -> torch.Tensor:
    """An uninitialised 1-D tensor on `device` backed by slime_rs_device_alloc:
    physical chunks mapped into one virtual range, the batch-buffer placement
    the apply kernels stream well from (include/slime_rs.h, DESIGN.md
    "Placement modes").  Use it for large device-resident batches."""
    if dtype not in _TYPESTR:
        raise TypeError(f"device_empty: unsupported dtype {dtype}")
    with torch.cuda.device(device):
        t = torch.as_tensor(_DeviceBuffer(device, numel, dtype), device=f"cuda:{device}")
    if t.data_ptr() == 0 or t.numel() != numel:
        raise RuntimeError("device_empty: torch did not wrap the device buffer")
    return t


def placement(t: torch.Tensor) -> dict:
    """How device_empty placed t's buffer (slime_rs_device_alloc_info): the
    placements probed, their probe rates and the one kept."""
    return N.alloc_info(t.data_ptr())


def probe_placement(t: torch.Tensor) -> float:
    """The library's placement probe over a caller's FRESH buffer t (it
    overwrites t): GB/s of the C3-shaped read/write walk over its storage, 0
    if too small to measure (slime_rs_probe_placement).  Logs a warning when
    the rate is in the slow mode (below SLOW_PLACEMENT x the allocator's
    threshold): such a buffer runs the kernels about 10% slower for its whole
    life -- re-allocate it, or use device_empty(), which probes and re-places
    by itself."""
    dev = _dev_index(t)
    base = t.untyped_storage().data_ptr()
    nbytes = t.untyped_storage().nbytes()
    gbs = ctypes.c_double()
    N.check(lib.slime_rs_probe_placement(ctypes.c_void_p(base), nbytes, dev, ctypes.byref(gbs)))
    _known_placement.add(base)
    slow = SLOW_PLACEMENT * float(lib.slime_rs_placement_threshold())
    if 0 < gbs.value < slow:
        _log.warning("slime_amd: buffer at 0x%x (%.1f GiB) probes %.0f GB/s, the slow placement (< %.0f): "
                     "the kernels will stream ~10%% slower on it; allocate batches with "
                     "slime_amd.device.device_empty (slime_rs_device_alloc)", base, nbytes / 2**30, gbs.value, slow)
    return gbs.value


def _note_unprobed(t: torch.Tensor) -> None:
    """Once per storage: a >= 16 GiB caller buffer whose placement nobody probed
    (not from device_empty, never passed to probe_placement)."""
    st = t.untyped_storage()
    base = st.data_ptr()
    if st.nbytes() < PLACEMENT_WARN_BYTES or base in _known_placement or base in _warned_placement:
        return
    _warned_placement.add(base)
    _log.warning("slime_amd: %.1f GiB batch buffer at 0x%x has an unprobed physical placement; about 40%% of large "
                 "hipMalloc buffers land in the slow mode (~10%% slower kernels for the buffer's life).  Allocate "
                 "with slime_amd.device.device_empty, or call probe_placement() on the fresh buffer "
                 "(DESIGN.md §4)", st.nbytes() / 2**30, base)


def layout_of(nshards: int, L: int, shard_stride: Optional[int] = None) -> N.Layout:
    ss = L if shard_stride is None else shard_stride
    return N.Layout(obj_stride=ss * nshards, shard_stride=ss)


class Plan:
    """A compiled coefficient matrix on one device (slime_rs_plan_t)."""

    def __init__(self, handle: ctypes.c_void_p, device: int, in_max: int):
        self._h = handle
        self.device = device
        self.in_max = in_max  # highest source shard index a launch reads
        self.out_max = None   # highest destination shard index (None: rows - 1)
        rows, k = ctypes.c_int(), ctypes.c_int()
        N.check(lib.slime_rs_plan_shape(self._h, ctypes.byref(rows), ctypes.byref(k)))
        self.rows, self.k = rows.value, k.value

    @classmethod
    def encode(cls, need: int, total: int, device: int = 0) -> "Plan":
        h = ctypes.c_void_p()
        N.check(lib.slime_rs_plan_encode(device, need, total, ctypes.byref(h)))
        return cls(h, device, need - 1)

    @classmethod
    def reconstruct(cls, need: int, total: int, have: Sequence[int], want: Sequence[int], device: int = 0) -> "Plan":
        # The C entry point reads exactly `need` survivor indices.
        if len(have) != need:
            raise ValueError(f"reconstruct needs exactly need={need} surviving shard indices, got {len(have)}")
        if not want:
            raise ValueError("reconstruct needs at least one output row")
        h = ctypes.c_void_p()
        hv = (ctypes.c_int * len(have))(*have)
        wv = (ctypes.c_int * len(want))(*want)
        N.check(lib.slime_rs_plan_reconstruct(device, need, total, hv, wv, len(want), ctypes.byref(h)))
        return cls(h, device, max(have))

    @classmethod
    def matrix(cls, coeff: np.ndarray, in_shards: Sequence[int], device: int = 0) -> "Plan":
        c = np.ascontiguousarray(coeff, dtype=np.uint32)
        h = ctypes.c_void_p()
        sv = (ctypes.c_int * len(in_shards))(*in_shards)
        N.check(lib.slime_rs_plan_matrix(device, c.ctypes.data, c.shape[0], c.shape[1], sv, ctypes.byref(h)))
        return cls(h, device, max(in_shards))

    def set_outputs(self, out_shards: Sequence[int]) -> "Plan":
        """Write output row i to destination shard out_shards[i] (e.g. repair in place)."""
        if len(out_shards) != self.rows:
            raise ValueError("need one destination shard per output row")
        sv = (ctypes.c_int * len(out_shards))(*out_shards)
        N.check(lib.slime_rs_plan_set_outputs(self._h, sv))
        self.out_max = max(out_shards)
        return self

    def coefficients(self) -> np.ndarray:
        out = np.zeros((self.rows, self.k), dtype=np.uint32)
        N.check(lib.slime_rs_plan_coefficients(self._h, out.ctypes.data))
        return out

    def __call__(self, src: torch.Tensor, src_layout: N.Layout, dst: torch.Tensor, dst_layout: N.Layout, L: int,
                 nobj: int, stream: Optional[torch.cuda.Stream] = None, src_offset: int = 0,
                 dst_offset: int = 0) -> None:
        """Launch over nobj objects; offsets are in uint32 elements from the tensors' starts."""
        for t in (src, dst):
            if t.dtype not in (torch.int32, torch.uint32) or not t.is_contiguous():
                raise TypeError("plan buffers must be contiguous int32/uint32 tensors")
            if _dev_index(t) != self.device:
                raise ValueError("tensor is not on the plan's device")
        self._check_extent(src, src_offset, src_layout, L, nobj, self.in_max)
        self._check_extent(dst, dst_offset, dst_layout, L, nobj,
                           self.rows - 1 if self.out_max is None else self.out_max)
        _note_unprobed(src)
        if dst.data_ptr() != src.data_ptr():
            _note_unprobed(dst)
        N.check(lib.slime_rs_plan_execute(self._h, ctypes.c_void_p(src.data_ptr() + 4 * src_offset), src_layout,
                                          ctypes.c_void_p(dst.data_ptr() + 4 * dst_offset), dst_layout, L, nobj,
                                          _stream_handle(self.device, stream)))

    @staticmethod
    def _check_extent(t: torch.Tensor, off: int, lay: N.Layout, L: int, nobj: int, max_shard: int) -> None:
        # Host-side bounds check before launching a hand-written kernel.
        if nobj == 0 or L == 0:
            return
        last = off + (nobj - 1) * lay.obj_stride + max_shard * lay.shard_stride + L
        if off < 0 or last > t.numel():
            raise ValueError(f"layout addresses element {last} of a {t.numel()}-element tensor")

    def close(self) -> None:
        if self._h:
            lib.slime_rs_plan_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # pragma: no cover - interpreter shutdown
            pass


def fill_symbols(t: torch.Tensor, seed: int, stream: Optional[torch.cuda.Stream] = None) -> None:
    """Deterministic synthetic symbols in [0, p) — word g is a function of (seed, g)."""
    dev = _dev_index(t)
    N.check(lib.slime_rs_fill_symbols(dev, ctypes.c_void_p(t.data_ptr()), t.numel(), seed & (2**64 - 1),
                                      _stream_handle(dev, stream)))


def pack_bytes(src: torch.Tensor, mapping: int, words: torch.Tensor, flags: Optional[torch.Tensor] = None,
               stream: Optional[torch.cuda.Stream] = None) -> None:
    """Device MapToGFWith: uint8 tensor -> int32 word tensor (big-endian, XOR mapping)."""
    dev = _dev_index(src)
    if words.numel() < (src.numel() + 3) // 4:
        raise ValueError("words tensor too small")
    fp = ctypes.c_void_p(flags.data_ptr()) if flags is not None else None
    if _dev_index(words) != dev or (flags is not None and _dev_index(flags) != dev):
        raise ValueError("pack_bytes: tensors on different devices")
    N.check(lib.slime_gf_pack_device(dev, ctypes.c_void_p(src.data_ptr()), src.numel(), mapping & 0xFFFFFFFF,
                                     ctypes.c_void_p(words.data_ptr()), fp, _stream_handle(dev, stream)))


def unpack_words(words: torch.Tensor, mapping: int, dst: torch.Tensor,
                 stream: Optional[torch.cuda.Stream] = None) -> None:
    """Device MapFromGF: int32 word tensor -> uint8 tensor of 4x the length."""
    dev = _dev_index(words)
    if dst.numel() < 4 * words.numel():
        raise ValueError("byte tensor too small")
    if _dev_index(dst) != dev:
        raise ValueError("unpack_words: tensors on different devices")
    N.check(lib.slime_gf_unpack_device(dev, ctypes.c_void_p(words.data_ptr()), words.numel(), mapping & 0xFFFFFFFF,
                                       ctypes.c_void_p(dst.data_ptr()), _stream_handle(dev, stream)))


# ---- fused byte-domain object pipeline (writeChunks / reconstruct on device) ----

def slot_geometry(object_size: int, need: int, total: int, chunk_align: int = 1) -> tuple[int, int, int]:
    """(L symbols per chunk, chunk stride in bytes, minimal slot bytes) for objects of
    object_size bytes.  chunk_align 1 is the wire layout (chunk stride 4L, the object's
    bytes contiguous at the slot start); e.g. 256 puts every chunk on a line boundary."""
    L = -(-(-(-object_size // 4)) // need)
    if chunk_align < 1 or chunk_align % 4 and chunk_align != 1:
        raise ValueError("chunk_align must be 1 or a positive multiple of 4")
    cs = -(-4 * L // chunk_align) * chunk_align
    return L, cs, cs * total


def _check_slots(slots: torch.Tensor, slot_stride: int, nobj: int, slot_bytes: int) -> int:
    if slots.dtype != torch.uint8 or not slots.is_contiguous():
        raise TypeError("slots must be a contiguous uint8 tensor")
    if nobj and (slot_stride < slot_bytes or (nobj - 1) * slot_stride + slot_bytes > slots.numel()):
        raise ValueError("slot layout exceeds the slots tensor")
    return _dev_index(slots)


def _chunk_stride(L: int, chunk_stride: int) -> int:
    cs = chunk_stride or 4 * L
    if cs < 4 * L or cs % 4:
        raise ValueError("chunk_stride must be 0 or a multiple of 4 that is >= 4L")
    return cs


def encode_objects(plan: Plan, slots: torch.Tensor, slot_stride: int, object_size: int, nobj: int,
                   mapping: torch.Tensor, status: torch.Tensor, stream: Optional[torch.cuda.Stream] = None,
                   chunk_stride: int = 0, phase_event: Optional[torch.cuda.Event] = None) -> None:
    """Device writeChunks: chunks of every object slot, gf.MapToGF's mapping per object.
    Chunk c of a slot is at slot + c*chunk_stride (0: 4L, the object's bytes in place).
    phase_event (a recorded torch.cuda.Event) is recorded again on the stream
    between the speculative pass and the 1<<31 re-encode."""
    L, _, _ = slot_geometry(object_size, plan.k, plan.k + plan.rows)
    dev = _check_slots(slots, slot_stride, nobj, _chunk_stride(L, chunk_stride) * (plan.k + plan.rows))
    for t in (mapping, status):
        if t.numel() < nobj or t.dtype not in (torch.int32, torch.uint32) or _dev_index(t) != dev:
            raise ValueError("mapping/status need nobj int32 words on the slots' device")
    ev = None
    if phase_event is not None:
        if not phase_event.cuda_event:
            raise ValueError("phase_event must have been recorded once (torch creates events lazily)")
        ev = ctypes.c_void_p(phase_event.cuda_event)
    N.check(lib.slime_rs_encode_objects_phased(plan._h, ctypes.c_void_p(slots.data_ptr()), slot_stride,
                                               chunk_stride, object_size, nobj,
                                               ctypes.c_void_p(mapping.data_ptr()),
                                               ctypes.c_void_p(status.data_ptr()), _stream_handle(dev, stream), ev))


def resolve_fallbacks(plan: Plan, slots: torch.Tensor, slot_stride: int, object_size: int, nobj: int,
                      mapping: torch.Tensor, status: torch.Tensor,
                      stream: Optional[torch.cuda.Stream] = None, chunk_stride: int = 0) -> int:
    """Finish objects that need MapToGF's random mapping; returns how many were fixed."""
    L, _, _ = slot_geometry(object_size, plan.k, plan.k + plan.rows)
    dev = _check_slots(slots, slot_stride, nobj, _chunk_stride(L, chunk_stride) * (plan.k + plan.rows))
    n = ctypes.c_int(0)
    N.check(lib.slime_rs_resolve_fallbacks_chunked(plan._h, ctypes.c_void_p(slots.data_ptr()), slot_stride,
                                                   chunk_stride, object_size, nobj,
                                                   ctypes.c_void_p(mapping.data_ptr()),
                                                   ctypes.c_void_p(status.data_ptr()), _stream_handle(dev, stream),
                                                   ctypes.byref(n)))
    return n.value


def decode_objects(plan: Plan, slots: torch.Tensor, slot_stride: int, L: int, nobj: int, mapping: torch.Tensor,
                   stream: Optional[torch.cuda.Stream] = None, chunk_stride: int = 0) -> None:
    """Device reconstruct: rebuild the plan's output chunks from its input chunks in every slot."""
    hi = max(plan.in_max, plan.rows - 1 if plan.out_max is None else plan.out_max)
    dev = _check_slots(slots, slot_stride, nobj, _chunk_stride(L, chunk_stride) * (hi + 1))
    if mapping.numel() < nobj or mapping.dtype not in (torch.int32, torch.uint32) or _dev_index(mapping) != dev:
        raise ValueError("mapping needs nobj int32 words on the slots' device")
    N.check(lib.slime_rs_decode_objects_chunked(plan._h, ctypes.c_void_p(slots.data_ptr()), slot_stride,
                                                chunk_stride, L, nobj, ctypes.c_void_p(mapping.data_ptr()),
                                                _stream_handle(dev, stream)))
