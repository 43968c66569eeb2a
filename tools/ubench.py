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
LIB = ctypes.CDLL(os.environ.get("UBENCH_LIB") or
                  os.path.join(ROOT, "cs265-lsm-tree_amd", "lib", "libbloomhip_ubench.so"))
LIB.ubench_run.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64,
                           ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
LIB.ubench_run.restype = ctypes.c_int
LIB.ubench_part_geometry.argtypes = [ctypes.c_size_t, ctypes.c_uint64, ctypes.c_void_p]
LIB.ubench_part_geometry.restype = ctypes.c_int
LIB.ubench_part.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64,
                            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
LIB.ubench_part.restype = ctypes.c_int
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


def _events(fn, reps):
    s = torch.cuda.current_stream()
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(reps):
        fn()
    b.record(s)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def part_phases(n=16_777_216, bpe=10.0, reps=50):
    """The product's partition build (C2 by default) by pass, and pass 2 with
    each lane count G (ubench_part)."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "cs265-lsm-tree_amd"))
    import bloomhip as bh
    keys = torch.from_numpy(bh.gen_puts(13141, n)).cuda()
    m = bh.m_bits(n, bpe)
    geo = np.zeros(4, dtype=np.uint64)
    assert LIB.ubench_part_geometry(n, m, geo.ctypes.data) == 0
    nbins, seg_bits, tk, ntiles = (int(x) for x in geo)
    pos = torch.empty(ntiles * tk, dtype=torch.int64, device="cuda")
    runs = torch.empty(ntiles * (nbins + 1) * 4, dtype=torch.int32, device="cuda")  # room for the 2x-segment plans
    words = torch.zeros((m + 63) // 64 * 2, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()

    def run(v):
        rc = LIB.ubench_part(v, keys.data_ptr(), n, m, pos.data_ptr(), runs.data_ptr(),
                             words.data_ptr(), s.cuda_stream)
        assert rc == 0, (v, rc)
    names = {0: "pass 1", 1: "pass 2 (product G)", 4: "pass 2 G=4",
             8: "pass 2 G=8", 16: "pass 2 G=16", 32: "pass 2 G=32",
             3001: "pass 2 indep groups G=1", 3002: "pass 2 indep G=2", 3004: "pass 2 indep G=4",
             3008: "pass 2 indep G=8"}
    if os.environ.get("UB_P1"):
        # order matters: the 21xx pass-2 variants read the table the last
        # 2048-key-tile pass 1 (2007) wrote
        names = {0: "pass 1", 2001: "pass 1 TB512 maxb1024 4w", 2002: "pass 1 TB512 maxb1024 5w 3wg",
                 2003: "pass 1 TB512 maxb1024 6w 3wg", 2011: "pass 1 TB512 maxb511 4w",
                 2013: "pass 1 TB512 maxb511 6w 3wg",
                 2004: "pass 1 TB256 5w 5wg", 2006: "pass 1 TB256 4w 4wg",
                 2008: "pass 1 TB256 maxb511 6w 6wg", 2007: "pass 1 TB256 maxb511 5w 5wg",
                 2122: "pass 2 (2048-key tiles) G=2 d=2", 2142: "pass 2 (2048) G=4 d=2",
                 2192: "pass 2 (2048) indep G=2", 2194: "pass 2 (2048) indep G=4",
                 2191: "pass 2 (2048) indep G=1"}
    if os.environ.get("UB_T4K"):  # C5 etc. on 4096-key tiles (TB = 512 pass 1)
        names = {0: "pass 1 (product)", 1: "pass 2 (product)", 3002: "pass 2 indep G=2",
                 3004: "pass 2 indep G=4",
                 2021: "pass 1 TB512 4096-key tiles maxb1023", 2242: "pass 2 (4096) G=4 d=2",
                 2282: "pass 2 (4096) G=8 d=2", 2291: "pass 2 (4096) indep G=1",
                 2292: "pass 2 (4096) indep G=2", 2294: "pass 2 (4096) indep G=4",
                 2022: "pass 1 TB512 4096-key tiles maxb4096"}
    if os.environ.get("UB_GD"):
        names = {0: "pass 1", 1: "pass 2 (product G)"}
        names.update({1000 + 10 * g + d: f"pass 2 G={g} depth={d}"
                      for g in (1, 2, 4) for d in (1, 2, 4)})
    run(0)
    # time-based prewarm: the chip's clocks ramp over the first ~0.1-0.5 s of
    # work, which otherwise makes the first phases measured look slower
    import time
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < float(os.environ.get("UB_PREWARM", "0.5")):
        for _ in range(20):
            run(0)
        torch.cuda.synchronize()
    if os.environ.get("UB_P1"):
        run(0); run(1)
        ref = words.clone()
        for p2 in (2142, 2192, 2194):
            words.zero_(); run(2007); run(p2)
            torch.cuda.synchronize()
            print(json.dumps({"check": f"2048-key tiles {p2} bitmap == product", "ok": bool(torch.equal(ref, words))}))
    if os.environ.get("UB_T4K"):
        run(0); run(1)
        ref = words.clone()
        p1 = 2021 if nbins <= 1023 else 2022
        for p2 in (2242, 2294):
            words.zero_(); run(p1); run(p2)
            torch.cuda.synchronize()
            print(json.dumps({"check": f"4096-key tiles {p2} bitmap == product", "ok": bool(torch.equal(ref, words))}))
    run(0); run(1)
    ref = words.clone()
    for v in (3001, 3002, 3004, 3008):
        words.zero_(); run(v)
        torch.cuda.synchronize()
        print(json.dumps({"check": f"indep walk {v} bitmap == product", "ok": bool(torch.equal(ref, words))}), flush=True)
    if os.environ.get("UB_QUICK"):
        names = {0: "pass 1", 1: "pass 2 (product)"}
    if os.environ.get("UB_2X"):  # segments for twice the CU count (two pass-2 WGs per CU)
        run(4000); run(4001)
        w2 = words.clone()
        run(0); run(1)
        print(json.dumps({"check": "2x-segment plan bitmap == product", "ok": bool(torch.equal(w2, words))}), flush=True)
        names = {0: "pass 1", 1: "pass 2 (product)", 4000: "pass 1 (2x segments)",
                 4001: "pass 2 (2x segments)", -4000: "pass 1 (2x) again", -5: "pass 2 again",
                 -4001: "pass 2 (2x) again"}
    names = dict(names)
    names[-1] = "pass 1 (again, last)"
    if os.environ.get("UB_ALT"):
        names = {0: "pass 1 product", 2014: "2011 at run_starts", -1: "product", -2014: "2011 again",
                 -2: "product", -3: "2011 again"}
    for v, name in names.items():
        ms = _events(lambda: run({-1: 0, -2: 0, -3: 2014, -5: 1}.get(v, abs(v))), reps)
        print(json.dumps({"op": "partition build", "n": n, "m": m, "nbins": nbins,
                          "seg_bits": seg_bits, "tile_keys": tk, "phase": name,
                          "us": round(ms * 1e3, 1)}), flush=True)





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
    tk = 8192 if nb.value > 256 else 4096
    ntiles = (n + tk - 1) // tk
    dk = torch.from_numpy(gets).cuda()
    pos = torch.empty(ntiles * tk, dtype=torch.int64, device="cuda")
    runs = torch.empty(2 * ntiles * (nb.value + 1), dtype=torch.int32, device="cuda")
    res = torch.empty(ntiles * tk * 3, dtype=torch.uint8, device="cuda")
    slots = torch.empty(ntiles * tk * 3, dtype=torch.int16, device="cuda")
    out = torch.empty(nf * ((n + 63) // 64), dtype=torch.int64, device="cuda")
    s = torch.cuda.current_stream()

    def run(v):
        return LIB.ubench_stack(v, dk.data_ptr(), n, nf, msa.ctypes.data, wp, pos.data_ptr(),
                                runs.data_ptr(), res.data_ptr(), slots.data_ptr(), out.data_ptr(),
                                s.cuda_stream)
    assert run(0) == 0
    torch.cuda.synchronize()
    ref = out.clone()
    for v in (3001, 3002, 3004, 3008, 3900, 3952, 3954, 3958):
        out.zero_()
        assert run(1) == 0 and run(v) == 0 and run(5) == 0
        torch.cuda.synchronize()
        print(json.dumps({"check": f"stack indep walk {v} == product", "ok": bool(torch.equal(ref, out))}), flush=True)
    names = {0: "all three", 1: "pass 1 (+slots, +transpose)", 2: "pass 2", 5: "combine",
             102: "pass 2 G=2", 104: "pass 2 G=4", 108: "pass 2 G=8", 116: "pass 2 G=16",
             1021: "pass 2 G=2 d=1", 1024: "pass 2 G=2 d=4", 1041: "pass 2 G=4 d=1",
             1044: "pass 2 G=4 d=4", 1012: "pass 2 G=1 d=2",
             3001: "pass 2 indep G=1", 3002: "pass 2 indep G=2", 3004: "pass 2 indep G=4",
             3008: "pass 2 indep G=8", 3900: "pass 2 runtime nf G=4 (old product)", -2: "pass 2 again",
             3952: "pass 2 nf const indep G=2", 3954: "pass 2 nf const indep G=4",
             3958: "pass 2 nf const batch G=8", -3954: "nf const indep G=4 again"}
    for v in names:
        vv = abs(v)
        if run(vv) != 0:
            continue
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        for _ in range(20):
            run(vv)
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
    if len(sys.argv) > 1 and sys.argv[1] == "part":
        return part_phases()
    if len(sys.argv) > 1 and sys.argv[1] == "part_c5":
        return part_phases(67_108_864, 10.0, 20)
    if len(sys.argv) > 1 and sys.argv[1] == "part_c4":
        return part_phases(268_435_456, 12.0, 5)
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
