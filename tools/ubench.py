#!/usr/bin/env python3
"""Prices the gfx950 primitives the Bloom kernels are made of:
random 4-B global atomicOr (agent / workgroup scope), random 4-B gathers,
random LDS ds_or, the exact hash+mod arithmetic, and a streaming read.
Prints one JSON object per measurement."""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = ctypes.CDLL(os.path.join(ROOT, "cs265-lsm-tree_amd", "lib", "libbloomhip_ubench.so"))
LIB.ubench_run.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64,
                           ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
LIB.ubench_run.restype = ctypes.c_int
LIB.ubench_part_bin.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64,
                                ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
LIB.ubench_part_bin.restype = ctypes.c_int
LIB.ubench_part_apply.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                  ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
LIB.ubench_part_apply.restype = ctypes.c_int
LIB.ubench_stack.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                             ctypes.c_void_p, ctypes.c_void_p] + [ctypes.c_void_p] * 6
LIB.ubench_stack.restype = ctypes.c_int
LIB.ubench_stack_geometry.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_void_p]
LIB.ubench_stack_geometry.restype = ctypes.c_int


def timeit(which, buf, nbytes, m, grid, block, iters, reps=5):
    s = torch.cuda.current_stream()
    rc = LIB.ubench_run(which, buf.data_ptr(), nbytes, m, grid, block, iters, s.cuda_stream)
    assert rc == 0, rc
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(reps):
        LIB.ubench_run(which, buf.data_ptr(), nbytes, m, grid, block, iters, s.cuda_stream)
    b.record(s)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def part_ablation(n=16_777_216, bpe=10.0):
    """Pass 1 of the partition build (C2 by default) with phases removed, and
    pass-2 variants on its output."""
    sys.path.insert(0, os.path.join(ROOT, "cs265-lsm-tree_amd"))
    import bloomhip as bh
    keys = torch.from_numpy(bh.gen_puts(13141, n)).cuda()
    m = bh.m_bits(n, bpe)
    ntiles = (keys.numel() + 4095) // 4096
    nbins = 4096  # upper bound for the run-start table
    pos = torch.empty(ntiles * 12288, dtype=torch.int32, device="cuda")
    rs = torch.empty(ntiles * (nbins + 1) * 2, dtype=torch.int32, device="cuda")  # both layouts
    s = torch.cuda.current_stream()
    names = {0: "product", 1: "no tile store", 2: "no scatter/store", 3: "hash only",
             4: "full, column runs", 5: "full, row runs", 6: "transpose only"}
    for ab in range(7):
        for _ in range(3):
            LIB.ubench_part_bin(ab, keys.data_ptr(), keys.numel(), m, pos.data_ptr(),
                                rs.data_ptr(), s.cuda_stream)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        for _ in range(10):
            LIB.ubench_part_bin(ab, keys.data_ptr(), keys.numel(), m, pos.data_ptr(),
                                rs.data_ptr(), s.cuda_stream)
        b.record(s)
        torch.cuda.synchronize()
        print(json.dumps({"op": "k_part_bin", "ablate": names[ab],
                          "us": round(a.elapsed_time(b) / 10 * 1e3, 2)}), flush=True)
    # pass 2 variants on the positions of a full pass 1 (sub-segment order,
    # then segment order)
    words = torch.zeros((m + 63) // 64 * 2, dtype=torch.int32, device="cuda")
    for layout, ab in (("sub-sorted", 0),):
        LIB.ubench_part_bin(ab, keys.data_ptr(), keys.numel(), m, pos.data_ptr(), rs.data_ptr(),
                            s.cuda_stream)
        torch.cuda.synchronize()
        for batch in (0, 4, 8, 16, 402, 404, 408, 416, 502, 504, 508, 516, 0):
            for _ in range(2):
                rc = LIB.ubench_part_apply(batch, pos.data_ptr(), rs.data_ptr(), keys.numel(), m,
                                           words.data_ptr(), s.cuda_stream)
                assert rc == 0, (batch, rc)
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            for _ in range(10):
                LIB.ubench_part_apply(batch, pos.data_ptr(), rs.data_ptr(), keys.numel(), m,
                                      words.data_ptr(), s.cuda_stream)
            b.record(s)
            torch.cuda.synchronize()
            print(json.dumps({"op": "k_part_apply", "n": n, "variant": batch,
                              "us": round(a.elapsed_time(b) / 10 * 1e3, 2)}), flush=True)


def part_stagger(n=16_777_216, bpe=10.0):
    """Pass 1 (C2) as the product launches it (0), with one workgroup per CU
    (7), and with the second half of the grid started late (8..10)."""
    sys.path.insert(0, os.path.join(ROOT, "cs265-lsm-tree_amd"))
    import bloomhip as bh
    keys = torch.from_numpy(bh.gen_puts(13141, n)).cuda()
    m = bh.m_bits(n, bpe)
    ntiles = (keys.numel() + 4095) // 4096
    pos = torch.empty(ntiles * 12288, dtype=torch.int32, device="cuda")
    rs = torch.empty(ntiles * 4097 * 2, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    names = {0: "product", 7: "one workgroup per CU", 8: "stagger 8K cycles",
             9: "stagger 16K cycles", 10: "stagger 24K cycles"}
    ref = None
    for ab in (0, 7, 8, 9, 10, 0):
        for _ in range(3):
            assert LIB.ubench_part_bin(ab, keys.data_ptr(), keys.numel(), m, pos.data_ptr(),
                                       rs.data_ptr(), s.cuda_stream) == 0
        torch.cuda.synchronize()
        same = None
        if ab in (0, 8):
            h = (pos.sum().item(), rs[:ntiles * 257].sum().item())
            ref = h if ref is None else ref
            same = h == ref
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        for _ in range(20):
            LIB.ubench_part_bin(ab, keys.data_ptr(), keys.numel(), m, pos.data_ptr(),
                                rs.data_ptr(), s.cuda_stream)
        b.record(s)
        torch.cuda.synchronize()
        print(json.dumps({"op": "k_part_bin", "variant": names[ab], "same_output": same,
                          "us": round(a.elapsed_time(b) / 20 * 1e3, 2)}), flush=True)


def overlap(n=16_777_216, bpe=10.0):
    """Does pass 1 of one half-batch overlap pass 2 of the other on two
    streams?  Times bin(A) apply(A) bin(B) apply(B) on one stream against
    bin(A); {bin(B) || apply(A)}; apply(B), for both pass-1 grids."""
    sys.path.insert(0, os.path.join(ROOT, "cs265-lsm-tree_amd"))
    import bloomhip as bh
    m = bh.m_bits(n, bpe)
    half = n // 2
    keys = torch.from_numpy(bh.gen_puts(13141, n)).cuda()
    ka, kb = keys[:half], keys[half:]
    ntiles = (half + 4095) // 4096
    bufs = []
    for _ in range(2):
        bufs.append((torch.empty(ntiles * 12288, dtype=torch.int32, device="cuda"),
                     torch.empty(ntiles * 4097 * 2, dtype=torch.int32, device="cuda")))
    words = torch.zeros((m + 63) // 64 * 2, dtype=torch.int32, device="cuda")
    s1 = torch.cuda.current_stream()
    s2 = torch.cuda.Stream()

    def binp(variant, k, b, s):
        rc = LIB.ubench_part_bin(variant, k.data_ptr(), k.numel(), m, b[0].data_ptr(),
                                 b[1].data_ptr(), s.cuda_stream)
        assert rc == 0, rc

    def apply(k, b, s):
        rc = LIB.ubench_part_apply(0, b[0].data_ptr(), b[1].data_ptr(), k.numel(), m,
                                   words.data_ptr(), s.cuda_stream)
        assert rc == 0, rc

    def seq(variant):
        binp(variant, ka, bufs[0], s1)
        apply(ka, bufs[0], s1)
        binp(variant, kb, bufs[1], s1)
        apply(kb, bufs[1], s1)

    def ovl(variant):
        binp(variant, ka, bufs[0], s1)
        e = torch.cuda.Event()
        e.record(s1)
        s2.wait_event(e)
        apply(ka, bufs[0], s2)
        binp(variant, kb, bufs[1], s1)
        e2 = torch.cuda.Event()
        e2.record(s2)
        s1.wait_event(e2)
        apply(kb, bufs[1], s1)

    for name, fn, v in (("seq grid2x", seq, 4), ("ovl grid2x", ovl, 4), ("seq grid1x", seq, 7),
                        ("ovl grid1x", ovl, 7)):
        for _ in range(3):
            fn(v)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s1)
        for _ in range(20):
            fn(v)
        b.record(s1)
        torch.cuda.synchronize()
        print(json.dumps({"op": "half-batch pipeline", "mode": name,
                          "us": round(a.elapsed_time(b) / 20 * 1e3, 2)}), flush=True)


def stack_ablation(levels_sel=(0, 1, 2, 3, 4)):
    """The stacked C3 probe by phase (ubench_stack variants), and pass 2 with
    its result stores or 4 of its 5 member reads removed."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "cs265-lsm-tree_amd"))
    import bloomhip as bh
    from bloomhip import workloads as W
    gets, levels = W.c3()
    filters, ms = [], []
    for lvl, keys, m in levels:
        if lvl in levels_sel:
            f = bh.BloomFilter(m)
            f.set_batch(keys)
            filters.append(f)
            ms.append(m)
    nf = len(ms)
    msa = np.array(ms, dtype=np.uint64)
    wp = (ctypes.c_void_p * nf)(*[f.device_words_ptr() for f in filters])
    nb, sb = ctypes.c_uint64(), ctypes.c_uint64()
    assert LIB.ubench_stack_geometry(nf, msa.ctypes.data, ctypes.byref(nb), ctypes.byref(sb)) == 0
    n = gets.size
    ntiles = (n + 4095) // 4096
    dk = torch.from_numpy(gets).cuda()
    pos = torch.empty(ntiles * 12288, dtype=torch.int32, device="cuda")
    runs = torch.empty(2 * ntiles * (nb.value + 1), dtype=torch.int32, device="cuda")
    res = torch.empty(ntiles * 12288, dtype=torch.uint8, device="cuda")
    slots = torch.empty(ntiles * 12288, dtype=torch.int16, device="cuda")
    out = torch.empty(nf * ((n + 63) // 64), dtype=torch.int64, device="cuda")
    s = torch.cuda.current_stream()

    def run(v):
        return LIB.ubench_stack(v, dk.data_ptr(), n, nf, msa.ctypes.data, wp, pos.data_ptr(),
                                runs.data_ptr(), res.data_ptr(), slots.data_ptr(), out.data_ptr(),
                                s.cuda_stream)
    assert run(0) == 0
    names = {0: "all three", 1: "pass 1 (+slots, +transpose)", 2: "pass 2",
             3: "pass 2, no result stores", 4: "pass 2, member 0 image only", 5: "combine",
             6: "pass 2, non-temporal position loads",
             102: "pass 2 G=2", 104: "pass 2 G=4", 108: "pass 2 G=8", 116: "pass 2 G=16",
             8: "pass 2, 512-thread blocks", 10: "pass 2, 512-thread blocks, no result stores",
             11: "pass 2, image staging only", 201: "pass 2 G=8 depth 1",
             203: "pass 2 G=8 depth 3", 204: "pass 2 G=8 depth 4"}
    for v in names:
        if run(v) != 0:
            continue
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        for _ in range(20):
            run(v)
        b.record(s)
        torch.cuda.synchronize()
        print(json.dumps({"op": "stacked probe", "levels": list(levels_sel), "nbins": nb.value,
                          "seg_bits": sb.value, "phase": names[v],
                          "us": round(a.elapsed_time(b) / 20 * 1e3, 1)}), flush=True)


def mixed():
    """Can LDS atomics and VALU hashing overlap on a CU?  Some of 16 waves
    hash, the rest do random ds_add_rtn: time both together vs each alone."""
    buf = torch.zeros(1 << 20, dtype=torch.int32, device="cuda")
    nb = buf.numel() * 4
    for base, lds_op in ((10, "ds_add_rtn"), (20, "ds_write"), (30, "ds_read")):
      for vw in (8, 4, 12):
        t = {}
        for mode, name in ((0, "both"), (1, "valu only"), (2, "lds only")):
            t[name] = timeit(base + mode, buf, nb, 0, 512, vw, 64)
        print(json.dumps({"op": "valu/lds overlap", "lds_op": lds_op, "valu_waves": vw,
                          **{k: round(v * 1e3, 1) for k, v in t.items()},
                          "sum": round((t["valu only"] + t["lds only"]) * 1e3, 1)}), flush=True)


def main():
    torch.cuda.set_device(0)
    if len(sys.argv) > 1 and sys.argv[1] == "mixed":
        return mixed()
    if len(sys.argv) > 1 and sys.argv[1] == "stack":
        stack_ablation()
        return stack_ablation((0, 1, 2, 3))
    if len(sys.argv) > 1 and sys.argv[1] == "isa":
        return isa_rates()
    if len(sys.argv) > 1 and sys.argv[1] == "stagger":
        return part_stagger()
    if len(sys.argv) > 1 and sys.argv[1] == "part":
        return part_ablation()
    if len(sys.argv) > 1 and sys.argv[1] == "part_c5":
        return part_ablation(67_108_864, 10.0)
    if len(sys.argv) > 1 and sys.argv[1] == "overlap":
        return overlap()
    if len(sys.argv) > 1 and sys.argv[1] == "part_c4":
        return part_ablation(268_435_456, 12.0)
    grid, block = 2048, 256
    threads = grid * block
    out = []
    for size in [80 << 10, 2 << 20, 20 << 20, 80 << 20, 384 << 20]:
        buf = torch.zeros(size // 4 + 4, dtype=torch.int32, device="cuda")
        nb = buf.numel() * 4
        for which, name, iters in [(0, "atomic_or_agent", 64), (1, "atomic_or_workgroup", 64),
                                   (2, "gather", 256)]:
            ms = timeit(which, buf, nb, 0, grid, block, iters)
            ops = threads * iters
            out.append({"op": name, "table_bytes": size, "Gops_s": round(ops / ms / 1e6, 2),
                        "ms": round(ms, 4)})
            print(json.dumps(out[-1]), flush=True)
    buf = torch.zeros(1 << 20, dtype=torch.int32, device="cuda")
    ms = timeit(3, buf, buf.numel() * 4, 0, grid, 1024, 256)
    print(json.dumps({"op": "lds_or", "Gops_s": round(grid * 1024 * 256 / ms / 1e6, 1),
                      "ms": round(ms, 4)}), flush=True)
    for m in [167_772_160, 655_360, 3_221_225_472]:
        ms = timeit(4, buf, buf.numel() * 4, m, grid, block, 256)
        print(json.dumps({"op": "hash3+mod_fast", "m": m,
                          "Gkeys_s": round(threads * 256 / ms / 1e6, 1), "ms": round(ms, 4)}),
              flush=True)
    ms = timeit(5, buf, buf.numel() * 4, 0, grid, block, 256)
    print(json.dumps({"op": "hash3_raw", "Gkeys_s": round(threads * 256 / ms / 1e6, 1),
                      "ms": round(ms, 4)}), flush=True)
    big = torch.zeros(1 << 28, dtype=torch.int32, device="cuda")  # 1 GiB
    ms = timeit(6, big, big.numel() * 4, 0, 4096, 256, 1)
    print(json.dumps({"op": "stream_read", "GB_s": round(big.numel() * 4 / ms / 1e6, 1),
                      "ms": round(ms, 4)}), flush=True)


if __name__ == "__main__":
    sys.exit(main())
