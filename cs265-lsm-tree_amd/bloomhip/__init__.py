"""bloomhip — Python view of the MI355X Bloom-filter engine's C ABI.

Thin ctypes binding of ``include/bloomhip.h`` (``lib/libbloomhip.so``).  It
mirrors the reference's filter surface (jackdent/cs265-lsm-tree
src/bloom_filter.h:6-15) so tests read like the reference's own usage:

    f = BloomFilter(m_bits)         # BloomFilter(long length)   bloom_filter.h:12
    f.set(key)                      # void set(KEY_t)            bloom_filter.cpp:49-53
    f.is_set(key)                   # bool is_set(KEY_t) const   bloom_filter.cpp:55-59

plus the batch calls the GPU needs (``set_batch`` / ``test_batch``) and
``m_bits(max_size, bits_per_entry)`` for Run::Run's sizing (src/run.cpp:13-15).

There is no CPU fallback: if the HIP library is missing this module raises on
import, and every compute call goes through the gfx950 kernels.
"""
from __future__ import annotations

import ctypes
import os
from typing import Sequence

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(os.path.dirname(PKG_DIR), "lib")
# BLOOMHIP_LIB: another build of the same library (tools/ab.sh times two
# builds of the engine against each other in one GPU session).
LIB_PATH = os.environ.get("BLOOMHIP_LIB") or os.path.join(LIB_DIR, "libbloomhip.so")

OK = 0
EIO = -5
ENOMEM = -12
ENODEV = -19
EINVAL = -22
ERANGE = -34

BUILD_AUTO = 0
BUILD_ATOMIC = 1
BUILD_LDS = 2
BUILD_PARTITION = 3
PROBE_AUTO = 0
PROBE_GATHER = 1
PROBE_PARTITION = 2
PROBE_LDS = 3
PROBE_STACKED = 4
STRATEGY_NAMES = {BUILD_AUTO: "auto", BUILD_ATOMIC: "atomic", BUILD_LDS: "lds",
                  BUILD_PARTITION: "partition"}
PROF_SLOTS = 12

# Every symbol include/bloomhip.h and include/bloomhip_workload.h declare.
EXPORTED_SYMBOLS = (
    "bloomhip_abi_version", "bloomhip_kernel_sha", "bloomhip_strerror", "bloomhip_last_error",
    "bloomhip_device_count",
    "bloomhip_m_bits", "bloomhip_create", "bloomhip_destroy", "bloomhip_size",
    "bloomhip_nwords", "bloomhip_device", "bloomhip_device_words", "bloomhip_stream",
    "bloomhip_clear", "bloomhip_set_batch", "bloomhip_test_batch", "bloomhip_set",
    "bloomhip_is_set", "bloomhip_download", "bloomhip_upload", "bloomhip_sync",
    "bloomhip_set_strategy", "bloomhip_set_probe_strategy", "bloomhip_resolve_strategy", "bloomhip_profile_enable",
    "bloomhip_profile_read", "bloomhip_profile_reset", "bloomhip_trim", "bloomhip_host_positions",
    "bloomhip_gen_mt19937", "bloomhip_gen_glibc_rand", "bloomhip_gen_puts",
    "bloomhip_gen_workload", "bloomhip_set_batch_run", "bloomhip_set_run_meta",
    "bloomhip_get_run_meta", "bloomhip_route_gets", "bloomhip_route_gets_packed", "bloomhip_save", "bloomhip_load",
    "bloomhip_build_from_run_file", "bloomhip_compact", "bloomhip_clone",
)


class BloomHipError(RuntimeError):
    def __init__(self, status: int, what: str):
        lib = _lib()
        msg = lib.bloomhip_strerror(status).decode()
        detail = lib.bloomhip_last_error().decode()
        super().__init__(f"{what}: {msg} ({status}){' — ' + detail if detail else ''}")
        self.status = status


_LIB = None


def _lib():
    global _LIB
    if _LIB is None:
        # One HIP runtime per process: torch bundles its own libamdhip64 with the
        # same SONAME as /opt/rocm's.  Loading torch first makes the loader bind
        # this library to torch's copy, so device pointers and streams from
        # torch are valid here; loading ours first would leave torch with a
        # second runtime that cannot see the GPU.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"bloomhip: {LIB_PATH} is missing — build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)")
        L = ctypes.CDLL(LIB_PATH)
        P, I, U64, SZ = ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64, ctypes.c_size_t
        PU64 = ctypes.POINTER(ctypes.c_uint64)
        sig = {
            "bloomhip_abi_version": (I, []),
            "bloomhip_kernel_sha": (ctypes.c_char_p, []),
            "bloomhip_strerror": (ctypes.c_char_p, [I]),
            "bloomhip_last_error": (ctypes.c_char_p, []),
            "bloomhip_device_count": (I, [ctypes.POINTER(I)]),
            "bloomhip_m_bits": (I, [ctypes.c_int64, ctypes.c_float, PU64]),
            "bloomhip_create": (I, [I, U64, ctypes.POINTER(P)]),
            "bloomhip_destroy": (I, [P]),
            "bloomhip_size": (I, [P, PU64]),
            "bloomhip_nwords": (I, [P, PU64]),
            "bloomhip_device": (I, [P, ctypes.POINTER(I)]),
            "bloomhip_device_words": (I, [P, ctypes.POINTER(P)]),
            "bloomhip_stream": (I, [P, ctypes.POINTER(P)]),
            "bloomhip_clear": (I, [P, P]),
            "bloomhip_set_batch": (I, [P, P, SZ, SZ, I, P]),
            "bloomhip_test_batch": (I, [ctypes.POINTER(P), I, P, SZ, SZ, I, P, I, P]),
            "bloomhip_set": (I, [P, ctypes.c_int32]),
            "bloomhip_is_set": (I, [P, ctypes.c_int32, ctypes.POINTER(I)]),
            "bloomhip_download": (I, [P, P, SZ, P]),
            "bloomhip_upload": (I, [P, P, SZ, P]),
            "bloomhip_sync": (I, [P, P]),
            "bloomhip_set_strategy": (I, [P, I]),
            "bloomhip_set_probe_strategy": (I, [P, I]),
            "bloomhip_resolve_strategy": (I, [P, SZ, ctypes.POINTER(I)]),
            "bloomhip_profile_enable": (I, [P, I]),
            "bloomhip_profile_read": (I, [P, I, ctypes.POINTER(ctypes.c_char_p), PU64,
                                          ctypes.POINTER(ctypes.c_double)]),
            "bloomhip_profile_reset": (I, [P]),
            "bloomhip_trim": (I, []),
            "bloomhip_host_positions": (I, [U64, P, SZ, P]),
            "bloomhip_gen_mt19937": (I, [ctypes.c_uint32, SZ, P]),
            "bloomhip_gen_glibc_rand": (I, [ctypes.c_uint32, SZ, P]),
            "bloomhip_gen_puts": (I, [ctypes.c_uint32, SZ, P, P]),
            "bloomhip_gen_workload": (I, [ctypes.c_uint32, SZ, SZ, ctypes.c_float, ctypes.c_float,
                                          P, P]),
            "bloomhip_set_batch_run": (I, [P, P, SZ, SZ, I, P]),
            "bloomhip_set_run_meta": (I, [P, P, SZ, ctypes.c_int32]),
            "bloomhip_get_run_meta": (I, [P, P, SZ, ctypes.POINTER(SZ),
                                          ctypes.POINTER(ctypes.c_int32)]),
            "bloomhip_route_gets": (I, [ctypes.POINTER(P), I, P, SZ, SZ, I, P, P, P, I, P]),
            "bloomhip_route_gets_packed": (I, [ctypes.POINTER(P), I, P, SZ, SZ, I, P, P, I, P]),
            "bloomhip_compact": (I, [ctypes.POINTER(P), P, I, I, I, P, ctypes.POINTER(SZ), I, P,
                                     I, P]),
            "bloomhip_save": (I, [P, ctypes.c_char_p]),
            "bloomhip_clone": (I, [P, I, ctypes.POINTER(P)]),
            "bloomhip_load": (I, [ctypes.c_char_p, I, ctypes.POINTER(P)]),
            "bloomhip_build_from_run_file": (I, [ctypes.c_char_p, U64, ctypes.c_int64,
                                                 ctypes.c_float, I, ctypes.POINTER(P)]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _LIB = L
    return _LIB


def lib():
    return _lib()


def _check(rc: int, what: str) -> None:
    if rc != OK:
        raise BloomHipError(rc, what)


def device_count() -> int:
    n = ctypes.c_int(0)
    rc = _lib().bloomhip_device_count(ctypes.byref(n))
    return n.value if rc == OK else 0


def m_bits(max_size: int, bits_per_entry: float) -> int:
    """Run::Run's filter size (src/run.cpp:13-15): (long)((float)max_size * bpe)."""
    out = ctypes.c_uint64()
    _check(_lib().bloomhip_m_bits(int(max_size), float(bits_per_entry), ctypes.byref(out)),
           "bloomhip_m_bits")
    return out.value


def host_positions(m: int, keys) -> np.ndarray:
    """The engine's own position arithmetic evaluated on the host (self-test hook)."""
    k = np.ascontiguousarray(keys, dtype=np.int32)
    out = np.empty((k.size, 3), dtype=np.uint64)
    _check(_lib().bloomhip_host_positions(m, k.ctypes.data, k.size, out.ctypes.data),
           "bloomhip_host_positions")
    return out


def _nbytes(buf) -> int:
    return buf.nbytes if isinstance(buf, np.ndarray) else buf.numel() * buf.element_size()


def _is_tensor(buf) -> bool:
    # duck-typed so importing this module does not need torch
    return hasattr(buf, "data_ptr") and hasattr(buf, "is_cuda")


def _ptr_of(buf):
    """(address, on_device, keepalive) for a numpy array or a torch tensor."""
    if isinstance(buf, np.ndarray):
        if not buf.flags["C_CONTIGUOUS"]:
            buf = np.ascontiguousarray(buf)
        return buf.ctypes.data, 0, buf
    if _is_tensor(buf):
        if not buf.is_contiguous():
            raise ValueError("tensor must be contiguous")
        return buf.data_ptr(), 1 if buf.is_cuda else 0, buf
    arr = np.ascontiguousarray(buf, dtype=np.int32)
    return arr.ctypes.data, 0, arr


def _keys_ptr(keys, stride: int):
    """_ptr_of for a key vector (KEY_t = int32, src/types.h:4).  The engine
    reads int32 words at `stride` bytes; any other element type would be read
    as the wrong keys, so: numpy integer arrays at stride 4 are converted to
    int32 when every value fits, anything else that is not int32 is refused.
    Strided views (e.g. entry_t runs at stride 8) must be int32 buffers."""
    if isinstance(keys, np.ndarray):
        if keys.dtype != np.int32:
            if stride != 4 or keys.dtype.kind not in "iu":
                raise ValueError(f"keys must be int32 (got {keys.dtype} at stride {stride})")
            if keys.size and (keys.min() < -2**31 or keys.max() > 2**31 - 1):
                raise ValueError("keys out of int32 range")
            keys = keys.astype(np.int32)
    elif _is_tensor(keys):
        if str(keys.dtype) != "torch.int32":
            raise ValueError(f"key tensor must be torch.int32 (got {keys.dtype})")
    return _ptr_of(keys)


def _key_count(keep, stride: int, n):
    avail = _nbytes(keep)
    if n is None:
        return avail // stride
    if n and (n - 1) * stride + 4 > avail:
        raise ValueError(f"{n} keys at stride {stride} need more than the {avail} bytes given")
    return n


def _out_ptr(buf, need_bytes: int, itemsize: int, what: str):
    """_ptr_of for an output buffer: element size and capacity checked."""
    el = buf.itemsize if isinstance(buf, np.ndarray) else buf.element_size()
    if el != itemsize:
        raise ValueError(f"{what}: elements must be {itemsize} bytes (got {el})")
    if _nbytes(buf) < need_bytes:
        raise ValueError(f"{what}: {need_bytes} bytes needed, {_nbytes(buf)} given")
    if isinstance(buf, np.ndarray) and not buf.flags["C_CONTIGUOUS"]:
        raise ValueError(f"{what} must be contiguous")
    return _ptr_of(buf)


def _stream_ptr(stream):
    if stream is None:
        return None
    if isinstance(stream, int):
        return stream
    return stream.cuda_stream  # torch.cuda.Stream


class BloomFilter:
    """One device-resident filter (a ``bloomhip_filter`` handle)."""

    def __init__(self, m_bits: int, device: int = 0):
        if m_bits <= 0:
            raise BloomHipError(EINVAL, "BloomFilter(m_bits <= 0)")
        h = ctypes.c_void_p()
        _check(_lib().bloomhip_create(device, m_bits, ctypes.byref(h)), "bloomhip_create")
        self._h = h
        self.m = m_bits
        self.device = device
        n = ctypes.c_uint64()
        _check(_lib().bloomhip_nwords(h, ctypes.byref(n)), "bloomhip_nwords")
        self.nwords = n.value

    @classmethod
    def _adopt(cls, h: ctypes.c_void_p, device: int) -> "BloomFilter":
        self = cls.__new__(cls)
        self._h = h
        self.device = device
        m, n = ctypes.c_uint64(), ctypes.c_uint64()
        _check(_lib().bloomhip_size(h, ctypes.byref(m)), "bloomhip_size")
        _check(_lib().bloomhip_nwords(h, ctypes.byref(n)), "bloomhip_nwords")
        self.m, self.nwords = m.value, n.value
        return self

    @classmethod
    def load(cls, path: str, device: int = 0) -> "BloomFilter":
        """A filter saved with save() (bloomhip_load)."""
        h = ctypes.c_void_p()
        _check(_lib().bloomhip_load(os.fsencode(path), device, ctypes.byref(h)), "bloomhip_load")
        return cls._adopt(h, device)

    @classmethod
    def from_run_file(cls, path: str, n_entries: int, max_size: int, bits_per_entry: float,
                      device: int = 0) -> "BloomFilter":
        """Filter + run metadata rebuilt from a run file of entry_t records
        (bloomhip_build_from_run_file)."""
        h = ctypes.c_void_p()
        _check(_lib().bloomhip_build_from_run_file(os.fsencode(path), n_entries, max_size,
                                                   bits_per_entry, device, ctypes.byref(h)),
               "bloomhip_build_from_run_file")
        return cls._adopt(h, device)

    def clone(self, device: int | None = None) -> "BloomFilter":
        """bloomhip_clone: this filter (bitmap + run metadata) on `device`
        (peer copy over xGMI between GPUs)."""
        dev = self.device if device is None else device
        h = ctypes.c_void_p()
        _check(_lib().bloomhip_clone(self._h, dev, ctypes.byref(h)), "bloomhip_clone")
        return BloomFilter._adopt(h, dev)

    def save(self, path: str) -> None:
        _check(_lib().bloomhip_save(self._h, os.fsencode(path)), "bloomhip_save")

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            _lib().bloomhip_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    # --- reference surface ------------------------------------------------
    def set(self, key: int) -> None:
        _check(_lib().bloomhip_set(self._h, int(key)), "bloomhip_set")

    def is_set(self, key: int) -> bool:
        hit = ctypes.c_int(0)
        _check(_lib().bloomhip_is_set(self._h, int(key), ctypes.byref(hit)), "bloomhip_is_set")
        return bool(hit.value)

    # --- batches ----------------------------------------------------------
    def set_batch(self, keys, n: int | None = None, stride: int = 4, stream=None) -> None:
        ptr, on_dev, keep = _keys_ptr(keys, stride)
        n = _key_count(keep, stride, n)
        _check(_lib().bloomhip_set_batch(self._h, ptr, n, stride, on_dev, _stream_ptr(stream)),
               "bloomhip_set_batch")

    def set_batch_run(self, keys, n: int | None = None, stride: int = 4, stream=None) -> None:
        """set() of a whole run written in this key order, plus its fence
        pointers and max key (Run::put, src/run.cpp:158-174)."""
        ptr, on_dev, keep = _keys_ptr(keys, stride)
        n = _key_count(keep, stride, n)
        _check(_lib().bloomhip_set_batch_run(self._h, ptr, n, stride, on_dev,
                                             _stream_ptr(stream)), "bloomhip_set_batch_run")

    def set_run_meta(self, fences, max_key: int) -> None:
        f = np.ascontiguousarray(fences, dtype=np.int32)
        _check(_lib().bloomhip_set_run_meta(self._h, f.ctypes.data if f.size else None, f.size,
                                            max_key), "bloomhip_set_run_meta")

    def run_meta(self):
        """(fences int32[], max_key)."""
        nf, mk = ctypes.c_size_t(), ctypes.c_int32()
        _check(_lib().bloomhip_get_run_meta(self._h, None, 0, ctypes.byref(nf), None),
               "bloomhip_get_run_meta")
        out = np.empty(nf.value, dtype=np.int32)
        _check(_lib().bloomhip_get_run_meta(self._h, out.ctypes.data if out.size else None,
                                            out.size, ctypes.byref(nf), ctypes.byref(mk)),
               "bloomhip_get_run_meta")
        return out, mk.value

    def clear(self, stream=None) -> None:
        _check(_lib().bloomhip_clear(self._h, _stream_ptr(stream)), "bloomhip_clear")

    def words(self) -> np.ndarray:
        """Bitmap as ceil(m/64) uint64 blocks (dynamic_bitset layout)."""
        out = np.empty(self.nwords, dtype=np.uint64)
        _check(_lib().bloomhip_download(self._h, out.ctypes.data, out.size, None),
               "bloomhip_download")
        return out

    def load_words(self, words: np.ndarray) -> None:
        w = np.ascontiguousarray(words, dtype=np.uint64)
        _check(_lib().bloomhip_upload(self._h, w.ctypes.data, w.size, None), "bloomhip_upload")

    def device_words_ptr(self) -> int:
        p = ctypes.c_void_p()
        _check(_lib().bloomhip_device_words(self._h, ctypes.byref(p)), "bloomhip_device_words")
        return p.value

    def stream_ptr(self) -> int:
        p = ctypes.c_void_p()
        _check(_lib().bloomhip_stream(self._h, ctypes.byref(p)), "bloomhip_stream")
        return p.value or 0

    def sync(self, stream=None) -> None:
        _check(_lib().bloomhip_sync(self._h, _stream_ptr(stream)), "bloomhip_sync")

    def set_strategy(self, strategy: int) -> None:
        _check(_lib().bloomhip_set_strategy(self._h, strategy), "bloomhip_set_strategy")

    def set_probe_strategy(self, strategy: int) -> None:
        _check(_lib().bloomhip_set_probe_strategy(self._h, strategy), "bloomhip_set_probe_strategy")

    def resolve_strategy(self, n: int) -> int:
        s = ctypes.c_int()
        _check(_lib().bloomhip_resolve_strategy(self._h, n, ctypes.byref(s)),
               "bloomhip_resolve_strategy")
        return s.value

    # --- profiling ----------------------------------------------------------
    def profile(self, enable: bool = True) -> None:
        _check(_lib().bloomhip_profile_enable(self._h, 1 if enable else 0), "profile_enable")

    def profile_reset(self) -> None:
        _check(_lib().bloomhip_profile_reset(self._h), "profile_reset")

    def profile_read(self) -> dict:
        res = {}
        for slot in range(PROF_SLOTS):
            name = ctypes.c_char_p()
            launches = ctypes.c_uint64()
            ms = ctypes.c_double()
            _check(_lib().bloomhip_profile_read(self._h, slot, ctypes.byref(name),
                                                ctypes.byref(launches), ctypes.byref(ms)),
                   "profile_read")
            if launches.value:
                res[name.value.decode()] = {"launches": launches.value, "ms": ms.value}
        return res


def test_batch(filters: Sequence[BloomFilter], keys, n: int | None = None, stride: int = 4,
               out=None, stream=None):
    """is_set of every key against each filter.  Returns (or fills) a packed
    [nf, ceil(n/64)] uint64 array: bit i%64 of row j word i/64 = filters[j].is_set(key i)."""
    ptr, on_dev, keep = _keys_ptr(keys, stride)
    n = _key_count(keep, stride, n)
    nf = len(filters)
    nw = (n + 63) // 64
    if out is None:
        out = np.zeros((nf, nw), dtype=np.uint64)
    optr, out_dev, okeep = _out_ptr(out, nf * nw * 8, 8, "out")
    arr = (ctypes.c_void_p * nf)(*[f.handle.value for f in filters])
    _check(_lib().bloomhip_test_batch(arr, nf, ptr, n, stride, on_dev, optr, out_dev,
                                      _stream_ptr(stream)), "bloomhip_test_batch")
    return out


def route_gets(runs: Sequence[BloomFilter], keys, n: int | None = None, stride: int = 4,
               cand=None, first=None, page=None, stream=None):
    """Batched GET routing (bloomhip_route_gets): runs newest first.  Returns
    (cand [nruns, ceil(n/64)] uint64 packed, first int32[n], page int32[n]);
    pass device tensors for all three to keep the outputs on the device."""
    ptr, on_dev, keep = _keys_ptr(keys, stride)
    n = _key_count(keep, stride, n)
    nr = len(runs)
    nw = (n + 63) // 64
    if cand is None and first is None and page is None:
        cand = np.zeros((nr, nw), dtype=np.uint64)
        first = np.empty(n, dtype=np.int32)
        page = np.empty(n, dtype=np.int32)
    need = ((nr * nw * 8, 8, "cand"), (n * 4, 4, "first"), (n * 4, 4, "page"))
    outs = [_out_ptr(x, *nd) if x is not None else (None, None, None)
            for x, nd in zip((cand, first, page), need)]
    devs = {o[1] for o in outs if o[0] is not None}
    if len(devs) > 1:
        raise ValueError("route_gets outputs must be all host or all device buffers")
    out_dev = devs.pop() if devs else 0
    arr = (ctypes.c_void_p * nr)(*[r.handle.value for r in runs])
    _check(_lib().bloomhip_route_gets(arr, nr, ptr, n, stride, on_dev, outs[0][0], outs[1][0],
                                      outs[2][0], out_dev, _stream_ptr(stream)),
           "bloomhip_route_gets")
    return cand, first, page


ROUTE_NONE = 0xFFFFFFFF   # BLOOMHIP_ROUTE_NONE: no candidate run
ROUTE_PAGE_BITS = 28


def route_gets_packed(runs: Sequence[BloomFilter], keys, n: int | None = None, stride: int = 4,
                      cand=None, route=None, stream=None):
    """Batched GET routing with the packed output (bloomhip_route_gets_packed):
    runs newest first (at most 16).  Returns (cand [nruns, ceil(n/64)] uint64
    packed, route uint32[n]) with route[i] = first << 28 | page, or
    ROUTE_NONE; pass device tensors for both to keep them on the device."""
    ptr, on_dev, keep = _keys_ptr(keys, stride)
    n = _key_count(keep, stride, n)
    nr = len(runs)
    nw = (n + 63) // 64
    if cand is None and route is None:
        cand = np.zeros((nr, nw), dtype=np.uint64)
        route = np.empty(n, dtype=np.uint32)
    need = ((nr * nw * 8, 8, "cand"), (n * 4, 4, "route"))
    outs = [_out_ptr(x, *nd) if x is not None else (None, None, None)
            for x, nd in zip((cand, route), need)]
    devs = {o[1] for o in outs if o[0] is not None}
    if len(devs) > 1:
        raise ValueError("route_gets_packed outputs must be all host or all device buffers")
    out_dev = devs.pop() if devs else 0
    arr = (ctypes.c_void_p * nr)(*[r.handle.value for r in runs])
    _check(_lib().bloomhip_route_gets_packed(arr, nr, ptr, n, stride, on_dev, outs[0][0], outs[1][0],
                                             out_dev, _stream_ptr(stream)),
           "bloomhip_route_gets_packed")
    return cand, route


def unpack_route(route):
    """(first, page) int32 arrays from a packed route array, -1 where none."""
    r = np.asarray(route, dtype=np.uint32)
    none = r == ROUTE_NONE
    first = np.where(none, -1, (r >> ROUTE_PAGE_BITS).astype(np.int32)).astype(np.int32)
    page = np.where(none, -1, (r & ((1 << ROUTE_PAGE_BITS) - 1)).astype(np.int32)).astype(np.int32)
    return first, page


def compact(runs, drop_tombstones: bool = False, filter: BloomFilter | None = None,
            device: int = 0, out=None, stream=None):
    """Compaction (bloomhip_compact): runs = entry_t arrays (int32 [n, 2] numpy
    arrays or device tensors), newest first.  Returns the merged run (a
    [n_out, 2] int32 array, or the first n_out rows of `out` when given);
    builds `filter` (and its run metadata) from the merged keys when given."""
    nr = len(runs)
    for r in runs:  # entry_t {int32 key; int32 val;} (src/types.h:14-22)
        dt = str(r.dtype)
        if dt not in ("int32", "torch.int32") or len(r.shape) != 2 or r.shape[1] != 2:
            raise ValueError(f"runs must be int32 [n, 2] entry_t arrays (got {dt} {tuple(r.shape)})")
    keeps = [_ptr_of(r) for r in runs]
    ons = {k[1] for k in keeps}
    if len(ons) > 1:
        raise ValueError("runs must be all host or all device buffers")
    on_dev = ons.pop() if ons else 0
    sizes = [_nbytes(k[2]) // 8 for k in keeps]
    total = sum(sizes)
    if out is None:
        out = np.empty((max(total, 1), 2), dtype=np.int32)
    optr, out_dev, okeep = _out_ptr(out, total * 8, 4, "out")
    arr = (ctypes.c_void_p * max(nr, 1))(*[k[0] for k in keeps])
    ns = (ctypes.c_size_t * max(nr, 1))(*sizes)
    n_out = ctypes.c_size_t()
    _check(_lib().bloomhip_compact(arr, ns, nr, on_dev, 1 if drop_tombstones else 0, optr,
                                   ctypes.byref(n_out), out_dev,
                                   filter.handle if filter is not None else None,
                                   filter.device if filter is not None else device,
                                   _stream_ptr(stream)), "bloomhip_compact")
    return out[:n_out.value]


# --- workload streams (generator/generator.c restatement) --------------------
def gen_mt19937(seed: int, n: int) -> np.ndarray:
    out = np.empty(n, dtype=np.uint32)
    _check(_lib().bloomhip_gen_mt19937(seed, n, out.ctypes.data), "gen_mt19937")
    return out


def gen_glibc_rand(seed: int, n: int) -> np.ndarray:
    out = np.empty(n, dtype=np.int32)
    _check(_lib().bloomhip_gen_glibc_rand(seed, n, out.ctypes.data), "gen_glibc_rand")
    return out


def gen_puts(seed: int, n: int, with_vals: bool = False):
    keys = np.empty(n, dtype=np.int32)
    vals = np.empty(n, dtype=np.int32) if with_vals else None
    _check(_lib().bloomhip_gen_puts(seed, n, keys.ctypes.data,
                                    vals.ctypes.data if with_vals else None), "gen_puts")
    return (keys, vals) if with_vals else keys


def gen_workload(seed: int, n_puts: int, n_gets: int, skew: float, miss_ratio: float):
    puts = np.empty(n_puts, dtype=np.int32)
    gets = np.empty(n_gets, dtype=np.int32)
    _check(_lib().bloomhip_gen_workload(seed, n_puts, n_gets, skew, miss_ratio,
                                        puts.ctypes.data, gets.ctypes.data), "gen_workload")
    return puts, gets
