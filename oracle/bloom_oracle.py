"""TEST INFRASTRUCTURE ONLY — parity oracle for the Bloom-filter hot path.

Two independent CPU restatements of the reference filter
(jackdent/cs265-lsm-tree src/bloom_filter.{h,cpp}):

* ``np_*`` — vectorised numpy uint64 arithmetic (wraps mod 2**64 exactly like
  the reference's ``uint64_t`` chains, src/bloom_filter.cpp:8-47).
* ``COracle`` — ctypes binding of ``oracle/bloom_oracle.c`` (scalar C, the CPU
  baseline timed by bench.py).

Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg may
import this module.  The product (``cs265-lsm-tree_amd/``) never does.

Parity is pinned by SURVEY.md §8a/§8c known answers (tests/golden/); the
reference itself is unbuildable here (needs boost::dynamic_bitset).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

_U64 = np.uint64


def _sext(keys) -> np.ndarray:
    """KEY_t (int32) -> uint64 by sign extension: `uint64_t key; key = k;`
    src/bloom_filter.cpp:9-11."""
    k = np.asarray(keys, dtype=np.int32)
    return k.astype(np.int64).view(np.uint64)


def np_raw_hashes(keys) -> np.ndarray:
    """[n, 3] uint64: hash_1..hash_3 before the modulo (src/bloom_filter.cpp:8-47)."""
    x0 = _sext(keys)
    with np.errstate(over="ignore"):
        # hash_1, src/bloom_filter.cpp:8-20
        x = ~x0 + (x0 << _U64(15))
        x = x ^ (x >> _U64(12))
        x = x + (x << _U64(2))
        x = x ^ (x >> _U64(4))
        x = x * _U64(2057)
        h1 = x ^ (x >> _U64(16))
        # hash_2, src/bloom_filter.cpp:22-34
        x = (x0 + _U64(0x7ED55D16)) + (x0 << _U64(12))
        x = (x ^ _U64(0xC761C23C)) ^ (x >> _U64(19))
        x = (x + _U64(0x165667B1)) + (x << _U64(5))
        x = (x + _U64(0xD3A2646C)) ^ (x << _U64(9))
        x = (x + _U64(0xFD7046C5)) + (x << _U64(3))
        h2 = (x ^ _U64(0xB55A4F09)) ^ (x >> _U64(16))
        # hash_3, src/bloom_filter.cpp:36-47
        x = (x0 ^ _U64(61)) ^ (x0 >> _U64(16))
        x = x + (x << _U64(3))
        x = x ^ (x >> _U64(4))
        x = x * _U64(0x27D4EB2D)
        h3 = x ^ (x >> _U64(15))
    return np.stack([h1, h2, h3], axis=1)


def np_positions(keys, m: int) -> np.ndarray:
    """[n, 3] uint64 bit positions: hash_i(k) % table.size() (src/bloom_filter.cpp:19,33,46)."""
    if m <= 0:
        raise ValueError("m must be positive (reference divides by table.size())")
    return np_raw_hashes(keys) % _U64(m)


def np_m_bits(max_size: int, bits_per_entry: float) -> int:
    """Run::Run sizing: `bloom_filter(max_size * bf_bits_per_entry)` with long*float
    evaluated in float and truncated to long (src/run.cpp:13-15, src/bloom_filter.h:12)."""
    f = np.float32(np.float32(max_size) * np.float32(bits_per_entry))
    return int(np.int64(f))


def np_words(m: int) -> int:
    return (m + 63) // 64


def np_set_batch(words: np.ndarray, m: int, keys) -> None:
    """BloomFilter::set over a batch into uint64 blocks (src/bloom_filter.cpp:49-53)."""
    pos = np_positions(keys, m).reshape(-1)
    np.bitwise_or.at(words, (pos >> _U64(6)).astype(np.int64),
                     _U64(1) << (pos & _U64(63)))


def np_build(m: int, keys) -> np.ndarray:
    words = np.zeros(np_words(m), dtype=np.uint64)
    np_set_batch(words, m, keys)
    return words


def np_test_batch(words: np.ndarray, m: int, keys) -> np.ndarray:
    """BloomFilter::is_set per key (src/bloom_filter.cpp:55-59) as a bool array."""
    pos = np_positions(keys, m)
    bits = (words[(pos >> _U64(6)).astype(np.int64)] >> (pos & _U64(63))) & _U64(1)
    return bits.all(axis=1)


def pack_bools(b: np.ndarray) -> np.ndarray:
    """bool[n] -> uint64[ceil(n/64)], bit i%64 of word i/64 (little-endian bit order)."""
    b = np.asarray(b, dtype=bool)
    n = b.size
    pad = (-n) % 64
    bb = np.concatenate([b, np.zeros(pad, dtype=bool)]) if pad else b
    return np.packbits(bb.reshape(-1, 8), axis=1, bitorder="little").reshape(-1).view(np.uint64).copy()


def unpack_bools(packed: np.ndarray, n: int) -> np.ndarray:
    bits = np.unpackbits(np.asarray(packed, dtype=np.uint64).view(np.uint8), bitorder="little")
    return bits[:n].astype(bool)


# --------------------------------------------------------------------------
# C restatement (oracle/bloom_oracle.c) via ctypes.
# --------------------------------------------------------------------------
def build_c_oracle(force: bool = False, lib: str = "liboracle.so") -> str:
    src = os.path.join(HERE, "bloom_oracle.c")
    path = os.path.join(HERE, lib)
    if force or not os.path.exists(path) or os.path.getmtime(path) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", HERE, lib])
    return path


class COracle:
    """ctypes view of oracle/bloom_oracle.c.  flags="O0" loads the build at the
    reference Makefile's own flags (-O0 -g, Makefile:4), for the CPU baseline."""

    def __init__(self, flags: str = "O2"):
        L = ctypes.CDLL(build_c_oracle(lib="liboracle_O0.so" if flags == "O0" else "liboracle.so"))
        P = ctypes.c_void_p
        L.bo_m_bits.argtypes = [ctypes.c_int64, ctypes.c_float, ctypes.POINTER(ctypes.c_uint64)]
        L.bo_m_bits.restype = ctypes.c_int
        L.bo_positions_batch.argtypes = [P, ctypes.c_size_t, ctypes.c_uint64, P]
        L.bo_raw_batch.argtypes = [P, ctypes.c_size_t, P]
        L.bo_set_batch.argtypes = [P, ctypes.c_uint64, P, ctypes.c_size_t, ctypes.c_size_t]
        L.bo_set_batch.restype = ctypes.c_int
        L.bo_test_batch.argtypes = [P, ctypes.c_uint64, P, ctypes.c_size_t, ctypes.c_size_t, P]
        L.bo_test_batch.restype = ctypes.c_int
        L.bo_is_set.argtypes = [P, ctypes.c_uint64, ctypes.c_int32]
        L.bo_is_set.restype = ctypes.c_int
        L.bo_popcount.argtypes = [P, ctypes.c_size_t]
        L.bo_popcount.restype = ctypes.c_uint64
        L.bo_run_meta.argtypes = [P, ctypes.c_size_t, ctypes.c_size_t, P, P]
        L.bo_run_meta.restype = ctypes.c_size_t
        L.bo_route.argtypes = [ctypes.c_int, P, P, P, P, P, P, ctypes.c_size_t, ctypes.c_size_t,
                               P, P, P]
        L.bo_route.restype = ctypes.c_int
        L.bo_compact.argtypes = [P, P, ctypes.c_int, ctypes.c_int, P]
        L.bo_compact.restype = ctypes.c_size_t
        L.bo_build_mt.argtypes = [P, ctypes.c_uint64, P, ctypes.c_size_t, ctypes.c_size_t,
                                  ctypes.c_int]
        L.bo_build_mt.restype = ctypes.c_int
        L.bo_build_many.argtypes = [P, ctypes.c_uint64, P, ctypes.c_size_t, ctypes.c_int]
        L.bo_build_many.restype = ctypes.c_int
        L.bo_test_mt.argtypes = [P, ctypes.c_uint64, P, ctypes.c_size_t, ctypes.c_size_t, P,
                                 ctypes.c_int]
        L.bo_test_mt.restype = ctypes.c_int
        self.L = L

    def m_bits(self, max_size: int, bpe: float) -> int:
        out = ctypes.c_uint64()
        rc = self.L.bo_m_bits(max_size, bpe, ctypes.byref(out))
        if rc != 0:
            raise ValueError(f"bo_m_bits({max_size}, {bpe}) -> {rc}")
        return out.value

    def positions(self, keys, m: int) -> np.ndarray:
        k = np.ascontiguousarray(keys, dtype=np.int32)
        out = np.empty((k.size, 3), dtype=np.uint64)
        self.L.bo_positions_batch(k.ctypes.data, k.size, m, out.ctypes.data)
        return out

    def raw(self, keys) -> np.ndarray:
        k = np.ascontiguousarray(keys, dtype=np.int32)
        out = np.empty((k.size, 3), dtype=np.uint64)
        self.L.bo_raw_batch(k.ctypes.data, k.size, out.ctypes.data)
        return out

    def build(self, m: int, keys, stride: int = 4, n: int | None = None) -> np.ndarray:
        """Bitmap (uint64 blocks) after set() of every key.  `keys` may be an
        AoS buffer read at `stride` bytes (entry_t runs: stride 8)."""
        buf = np.ascontiguousarray(keys)
        if n is None:
            n = buf.nbytes // stride
        words = np.zeros(np_words(m), dtype=np.uint64)
        rc = self.L.bo_set_batch(words.ctypes.data, m, buf.ctypes.data, n, stride)
        if rc != 0:
            raise ValueError(f"bo_set_batch rc={rc}")
        return words

    def set_into(self, words: np.ndarray, m: int, keys, stride: int = 4) -> None:
        buf = np.ascontiguousarray(keys)
        rc = self.L.bo_set_batch(words.ctypes.data, m, buf.ctypes.data, buf.nbytes // stride, stride)
        if rc != 0:
            raise ValueError(f"bo_set_batch rc={rc}")

    def test(self, words: np.ndarray, m: int, keys, stride: int = 4) -> np.ndarray:
        """Packed uint64 results, bit i%64 of word i/64 = is_set(key i)."""
        buf = np.ascontiguousarray(keys)
        n = buf.nbytes // stride
        out = np.zeros((n + 63) // 64, dtype=np.uint64)
        w = np.ascontiguousarray(words, dtype=np.uint64)
        rc = self.L.bo_test_batch(w.ctypes.data, m, buf.ctypes.data, n, stride, out.ctypes.data)
        if rc != 0:
            raise ValueError(f"bo_test_batch rc={rc}")
        return out

    def build_mt(self, m: int, keys, threads: int) -> np.ndarray:
        """build() on `threads` native threads (one shared bitmap, atomic ORs)."""
        buf = np.ascontiguousarray(keys, dtype=np.int32)
        words = np.zeros(np_words(m), dtype=np.uint64)
        rc = self.L.bo_build_mt(words.ctypes.data, m, buf.ctypes.data, buf.size, 4, threads)
        if rc != 0:
            raise ValueError(f"bo_build_mt rc={rc}")
        return words

    def build_many(self, m: int, keys_2d) -> np.ndarray:
        """One filter per row of keys_2d, one native thread each."""
        k = np.ascontiguousarray(keys_2d, dtype=np.int32)
        words = np.zeros((k.shape[0], np_words(m)), dtype=np.uint64)
        rc = self.L.bo_build_many(words.ctypes.data, m, k.ctypes.data, k.shape[1], k.shape[0])
        if rc != 0:
            raise ValueError(f"bo_build_many rc={rc}")
        return words

    def test_mt(self, words: np.ndarray, m: int, keys, threads: int) -> np.ndarray:
        """test() on `threads` native threads."""
        buf = np.ascontiguousarray(keys, dtype=np.int32)
        out = np.zeros((buf.size + 63) // 64, dtype=np.uint64)
        w = np.ascontiguousarray(words, dtype=np.uint64)
        rc = self.L.bo_test_mt(w.ctypes.data, m, buf.ctypes.data, buf.size, 4, out.ctypes.data,
                               threads)
        if rc != 0:
            raise ValueError(f"bo_test_mt rc={rc}")
        return out

    def popcount(self, words: np.ndarray) -> int:
        w = np.ascontiguousarray(words, dtype=np.uint64)
        return int(self.L.bo_popcount(w.ctypes.data, w.size))


def _run_meta(L, keys, stride: int = 4, n: int | None = None):
    buf = np.ascontiguousarray(keys)
    if n is None:
        n = buf.nbytes // stride
    fences = np.empty(max(1, (n + 4095) // 4096), dtype=np.int32)
    mx = ctypes.c_int32()
    nf = L.bo_run_meta(buf.ctypes.data, n, stride, fences.ctypes.data, ctypes.byref(mx))
    return fences[:nf].copy(), mx.value


def _route(L, runs, keys, stride: int = 4):
    """runs: [(words, m, fences, max_key)] newest first.  Returns
    (cand [nruns, ceil(n/64)] uint64, first int32[n], page int32[n])."""
    buf = np.ascontiguousarray(keys)
    n = buf.nbytes // stride
    nr = len(runs)
    keep = [(np.ascontiguousarray(w, dtype=np.uint64), np.ascontiguousarray(f, dtype=np.int32))
            for w, _, f, _ in runs]
    W = (ctypes.c_void_p * nr)(*[k[0].ctypes.data for k in keep])
    F = (ctypes.c_void_p * nr)(*[k[1].ctypes.data if k[1].size else None for k in keep])
    ms = np.array([r[1] for r in runs], dtype=np.uint64)
    nfs = np.array([k[1].size for k in keep], dtype=np.uint64)
    mks = np.array([r[3] for r in runs], dtype=np.int32)
    cand = np.zeros((nr, (n + 63) // 64), dtype=np.uint64)
    first = np.empty(n, dtype=np.int32)
    page = np.empty(n, dtype=np.int32)
    rc = L.bo_route(nr, W, ms.ctypes.data, F, nfs.ctypes.data, mks.ctypes.data, buf.ctypes.data, n,
                    stride, cand.ctypes.data, first.ctypes.data, page.ctypes.data)
    if rc != 0:
        raise ValueError(f"bo_route rc={rc}")
    return cand, first, page


COracle.run_meta = lambda self, keys, stride=4, n=None: _run_meta(self.L, keys, stride, n)
COracle.run_meta.__doc__ = "(fences, max_key) of a run written in this key order (src/run.cpp:158-174)."
COracle.route = lambda self, runs, keys, stride=4: _route(self.L, runs, keys, stride)
COracle.route.__doc__ = _route.__doc__


def _compact(L, runs, drop_tombstones: bool = False):
    """Merged run (int32 [n, 2]) of entry_t runs, newest first."""
    keep = [np.ascontiguousarray(r, dtype=np.int32).reshape(-1, 2) for r in runs]
    R = (ctypes.c_void_p * max(1, len(keep)))(*[k.ctypes.data for k in keep])
    ns = np.array([k.shape[0] for k in keep] or [0], dtype=np.uint64)
    out = np.empty((max(1, int(ns.sum())), 2), dtype=np.int32)
    w = L.bo_compact(R, ns.ctypes.data, len(keep), 1 if drop_tombstones else 0, out.ctypes.data)
    return out[:w]


COracle.compact = lambda self, runs, drop_tombstones=False: _compact(self.L, runs, drop_tombstones)
COracle.compact.__doc__ = _compact.__doc__
