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
                            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                            ctypes.c_size_t, ctypes.c_size_t]
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


def _part_setup(n, bpe, m=None):
    """Keys, geometry and buffers of the product's partition build of n keys
    (into m bits, else n * bpe as Run::Run sizes it)."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "cs265-lsm-tree_amd"))
    import bloomhip as bh
    keys = torch.from_numpy(bh.gen_puts(13141, n)).cuda()
    m = m or bh.m_bits(n, bpe)
    geo = np.zeros(4, dtype=np.uint64)
    assert LIB.ubench_part_geometry(n, m, geo.ctypes.data) == 0
    nbins, seg_bits, tk, ntiles = (int(x) for x in geo)
    pos = torch.empty(ntiles * tk, dtype=torch.int64, device="cuda")
    runs = torch.empty(ntiles * (nbins + 1) * 2, dtype=torch.int32, device="cuda")
    words = torch.zeros((m + 63) // 64 * 2, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()

    def run(v):
        return LIB.ubench_part(v, keys.data_ptr(), n, m, pos.data_ptr(), runs.data_ptr(),
                               words.data_ptr(), s.cuda_stream, pos.numel(), runs.numel())
    return run, words, {"n": n, "m": m, "nbins": nbins, "seg_bits": seg_bits, "tile_keys": tk}


def _prewarm(run, v, secs=0.5):
    import time
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < secs:
        for _ in range(20):
            run(v)
        torch.cuda.synchronize()


def part_phases(n=16_777_216, bpe=10.0, reps=50):
    """The product's partition build by pass (pass 2 timed over pass 1's
    output), and pass 2 at other lane counts / walks, two rounds."""
    run, words, geo = _part_setup(n, bpe)
    assert run(0) == 0 and run(1) == 0
    torch.cuda.synchronize()
    ref = words.clone()
    names = {0: "pass 1 (product)", 1: "pass 2 (product)"}
    # the segment geometry (round 2) against the product's plan_build
    words.zero_()
    if run(20) == 0 and run(21) == 0:
        torch.cuda.synchronize()
        print(json.dumps({"check": "segment-geometry bitmap == product", "ok": bool(torch.equal(ref, words))}),
              flush=True)
        names[20] = "pass 1 segments"
        names[21] = "pass 2 segments"
    _prewarm(run, 0)
    for rnd in range(2):
        for v in names:
            if v == 21:
                run(20)  # pass 2 over its own pass 1's output
            elif v == 1:
                run(0)
            ms = _events(lambda: run(v), reps)
            print(json.dumps({"op": "partition build", **geo, "phase": names[v], "round": rnd,
                              "us": round(ms * 1e3, 1)}), flush=True)


def p1_ab(variants, n=16_777_216, bpe=10.0, rounds=3, reps=50):
    """Interleaved A/B of pass-1 variants (ubench_part 5xxx) against the
    product (0): each variant's output goes through the product's pass 2
    and must give the product's bitmap; then rounds x variants timed."""
    run, words, geo = _part_setup(n, bpe)
    assert run(0) == 0 and run(1) == 0
    torch.cuda.synchronize()
    ref = words.clone()
    ok_vars = [0]
    for v in variants:
        words.zero_()
        if run(v) != 0:
            print(json.dumps({"variant": v, "skipped": "not applicable"}), flush=True)
            continue
        run(1)
        torch.cuda.synchronize()
        ok = bool(torch.equal(ref, words))
        print(json.dumps({"check": f"pass-1 variant {v} bitmap == product", "ok": ok}), flush=True)
        if ok:
            ok_vars.append(v)
    _prewarm(run, 0)
    res = {v: [] for v in ok_vars}
    for _ in range(rounds):
        for v in res:
            res[v].append(round(_events(lambda: run(v), reps) * 1e3, 2))
    for v, ts in res.items():
        print(json.dumps({"op": "pass 1 A/B", **geo, "variant": v, "us": ts, "min_us": min(ts)}),
              flush=True)


def p2_ab(variants, n=16_777_216, bpe=10.0, rounds=3, reps=50):
    """Interleaved A/B of pass-2 variants (ubench_part 2xxx / 3xxx) against
    the product's pass 2 (1), all over the product's pass-1 output; each
    variant's bitmap must equal the product's."""
    run, words, geo = _part_setup(n, bpe)
    assert run(0) == 0 and run(1) == 0
    torch.cuda.synchronize()
    ref = words.clone()
    ok_vars = [1]
    for v in variants:
        words.zero_()
        if run(v) != 0:
            print(json.dumps({"variant": v, "skipped": "not applicable"}), flush=True)
            continue
        torch.cuda.synchronize()
        ok = bool(torch.equal(ref, words))
        print(json.dumps({"check": f"pass-2 variant {v} bitmap == product", "ok": ok}), flush=True)
        if ok:
            ok_vars.append(v)
    _prewarm(run, 1)
    res = {v: [] for v in ok_vars}
    for _ in range(rounds):
        for v in res:
            res[v].append(round(_events(lambda: run(v), reps) * 1e3, 2))
    for v, ts in res.items():
        print(json.dumps({"op": "pass 2 A/B", **geo, "variant": v, "us": ts, "min_us": min(ts)}),
              flush=True)


def p1_ablation(n=16_777_216, bpe=10.0, rounds=3, reps=50):
    """C2's pass 1 cut after each stage (ubench_part 5100 + ABL, k_part_bin's
    ABL): 1 hash + bin/entry, 2 + rank atomics, 3 + scan and run table,
    4 + scatter, 5 + packing (no tile stores), 0 = the whole pass.  Variant
    5100 must give the product's bitmap through the product's pass 2;
    interleaved rounds."""
    run, words, geo = _part_setup(n, bpe)
    assert run(0) == 0 and run(1) == 0
    torch.cuda.synchronize()
    ref = words.clone()
    words.zero_()
    assert run(5100) == 0 and run(1) == 0
    torch.cuda.synchronize()
    print(json.dumps({"check": "ablation variant 5100 bitmap == product", "ok": bool(torch.equal(ref, words))}),
          flush=True)
    names = {5101: "hash + bin/entry", 5102: "+ rank atomics", 5103: "+ scan, run table",
             5105: "+ scatter + packing (no stores)", 5100: "whole pass 1", 0: "product pass 1"}
    # (ABL 4, the scatter without the packing, is left out: nothing reads the
    # scattered image, so the compiler drops the scatter and the entries)
    _prewarm(run, 0)
    res = {v: [] for v in names}
    for _ in range(rounds):
        for v in names:
            assert run(v) == 0
            res[v].append(round(_events(lambda: run(v), reps) * 1e3, 2))
    for v, ts in res.items():
        print(json.dumps({"op": "pass 1 ablation", **geo, "variant": v, "stage": names[v], "us": ts,
                          "min_us": min(ts)}), flush=True)


def p1_tail(m=167_772_160, reps=50):
    """The product's pass 1 at whole and partial last rounds: C2's 4096
    tiles are 5 1/3 rounds of the 768 resident workgroups (3 per CU); the
    filter stays C2's (m = 5 << 25), only the key count changes."""
    for ntiles in (3840, 4096, 4352, 4608, 3840, 4096):
        n = ntiles * 4096
        run, words, geo = _part_setup(n, 0.0, m)
        _prewarm(run, 0, 0.3)
        ts = [round(_events(lambda: run(0), reps) * 1e3, 2) for _ in range(3)]
        print(json.dumps({"op": "pass 1 tail", "tiles": ntiles, "rounds": round(ntiles / 768, 3),
                          "us": ts, "min_us": min(ts), "us_per_round": round(min(ts) / (ntiles / 768), 2)}),
              flush=True)
        del run, words
        torch.cuda.empty_cache()


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


LIB.ubench_ladder.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
                              ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p] + [ctypes.c_void_p] * 6
LIB.ubench_ladder.restype = ctypes.c_int
LIB.ubench_ladder_geometry.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
LIB.ubench_ladder_geometry.restype = ctypes.c_int


def ladder_ablation(levels_sel=(0, 1, 2, 3, 4), reps=20):
    """The C3 probe as a ladder stack (bins = hash bits), by phase, per tile
    size and pass-2 lane count, each checked against the segment stack's
    answers (ubench_stack variant 0, the round-2 product kind)."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "cs265-lsm-tree_amd"))
    import bloomhip as bh
    from bloomhip import workloads as W
    gets, levels = W.c3()
    filters, ms = [], []
    for lvl, keys, m in sorted(levels, key=lambda x: -x[2]):
        if lvl in levels_sel:
            f = bh.BloomFilter(m)
            f.set_batch(keys)
            filters.append(f)
            ms.append(m)
    nf = len(ms)
    msa = np.array(ms, dtype=np.uint64)
    wp = (ctypes.c_void_p * nf)(*[f.device_words_ptr() for f in filters])
    geo = np.zeros(6, dtype=np.uint64)
    assert LIB.ubench_ladder_geometry(nf, msa.ctypes.data, geo.ctypes.data) == 0
    n = gets.size
    ntiles = (n + 4095) // 4096
    dk = torch.from_numpy(gets).cuda()
    # padded runs (kernels.h padded_tile_entries) need up to 6 more entries
    # per bin and tile: twice the unpadded room covers them
    pos = torch.empty(2 * ntiles * 4096, dtype=torch.int64, device="cuda")
    runs = torch.empty(2 * ntiles * 4097, dtype=torch.int32, device="cuda")
    res = torch.empty(2 * ntiles * 4096 * 3, dtype=torch.uint8, device="cuda")
    slots = torch.empty(ntiles * 4096 * 3, dtype=torch.int16, device="cuda")
    out = torch.empty(nf * ((n + 63) // 64), dtype=torch.int64, device="cuda")
    s = torch.cuda.current_stream()
    nb, sb = ctypes.c_uint64(), ctypes.c_uint64()
    assert LIB.ubench_stack_geometry(nf, msa.ctypes.data, ctypes.byref(nb), ctypes.byref(sb)) == 0
    assert LIB.ubench_stack(0, dk.data_ptr(), n, nf, msa.ctypes.data, wp, pos.data_ptr(),
                            runs.data_ptr(), res.data_ptr(), slots.data_ptr(), out.data_ptr(),
                            s.cuda_stream) == 0
    torch.cuda.synchronize()
    ref = out.clone()

    def run(v, tk):
        return LIB.ubench_ladder(v, tk, dk.data_ptr(), n, nf, msa.ctypes.data, wp, pos.data_ptr(),
                                 runs.data_ptr(), res.data_ptr(), slots.data_ptr(),
                                 out.data_ptr(), s.cuda_stream)

    def stack(v):
        return LIB.ubench_stack(v, dk.data_ptr(), n, nf, msa.ctypes.data, wp, pos.data_ptr(),
                                runs.data_ptr(), res.data_ptr(), slots.data_ptr(), out.data_ptr(),
                                s.cuda_stream)
    variants = [int(v) for v in os.environ.get("UB_LADDER", "2,102").split(",")]
    for tk in (8192, 4096):
        for v in variants:
            out.zero_()
            if v >= 200:  # a whole (chunked) probe
                ok = run(v, tk) == 0
            else:
                b0 = 100 if v >= 100 else 0  # the table planner's own pass 1 / combine
                ok = run(b0 + 1, tk) == 0 and run(v, tk) == 0 and run(b0 + 5, tk) == 0
            torch.cuda.synchronize()
            print(json.dumps({"check": f"ladder tk={tk} pass-2 variant {v} == segment stack",
                              "ok": bool(ok and torch.equal(ref, out))}), flush=True)
    names = {0: "all three", 1: "pass 1 (+slots)", 2: "pass 2 (product)", 5: "combine",
             11: "pass 1 without the slot stores", 12: "pass 1 without slot and tile stores",
             100: "all three (table planner)", 102: "pass 2 (table planner)"}
    names.update({v: (f"all three, chunks of {v - 200} Mi keys" if v > 200 else f"pass 2 variant {v}")
                  for v in variants if v not in names})
    _prewarm(lambda v: run(0, 8192), 0)
    for rnd in range(2):
        t = _events(lambda: stack(0), reps)
        print(json.dumps({"op": "segment stack (round 2 kind)", "levels": list(levels_sel),
                          "round": rnd, "us": round(t * 1e3, 1)}), flush=True)
        for tk in (8192, 4096):
            for v in names:
                if run(v, tk) != 0:
                    continue
                t = _events(lambda: run(v, tk), reps)
                print(json.dumps({"op": "ladder stack", "levels": list(levels_sel), "tile_keys": tk,
                                  "nbins": int(geo[0]), "s": int(geo[1]), "hb": int(geo[2]),
                                  "lds_bytes": int(geo[3]), "k": int(geo[4]), "bpp": int(geo[5]),
                                  "phase": names[v], "round": rnd,
                                  "us": round(t * 1e3, 1)}), flush=True)


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


LIB.ubench_cal.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                           ctypes.c_int, ctypes.c_void_p]
LIB.ubench_cal_bytes.argtypes = [ctypes.c_int, ctypes.c_size_t, ctypes.c_int, ctypes.c_int]
LIB.ubench_cal_bytes.restype = ctypes.c_uint64

CAL_SHAPES = [(0, 1, 1, "read: coalesced 16-B vectors"), (1, 1, 1, "read: first 64 B of each 128-B line"),
              (2, 1, 1, "read: one 16-B vector per 128-B line"),
              (3, 1, 2458, "read: pass-2 walk, runs of 1 vector, 2458 segments (C4)"),
              (3, 2, 2458, "read: pass-2 walk, runs of 2 vectors, 2458 segments (C4)"),
              (3, 8, 256, "read: pass-2 walk, runs of 8 vectors, 256 segments (C2)"),
              (3, 16, 256, "read: pass-2 walk, runs of 16 vectors, 256 segments (C3)"),
              (10, 1, 1, "write: coalesced 16-B vectors"),
              (11, 1, 1, "write: 2-byte stores at 6i, 6i+2, 6i+4 (probe result bytes)"),
              (12, 1, 1, "write: one 4-B store per 128-B line (run-table columns)")]


def cal():
    """Calibration shapes (ubench_cal) over a 512 MiB buffer (beyond the
    Infinity Cache), three dispatches each; run under rocprofv3 --pmc
    FETCH_SIZE / WRITE_SIZE, then tools/pmc_cal.py reads the counters against
    the known bytes printed here."""
    nv = (512 << 20) // 16
    buf = torch.zeros(nv * 4, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    for i, (shape, R, nseg, name) in enumerate(CAL_SHAPES):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        assert LIB.ubench_cal(shape, buf.data_ptr(), nv, R, nseg, s.cuda_stream) == 0
        a.record(s)
        for rep in range(2):
            assert LIB.ubench_cal(shape, buf.data_ptr(), nv, R, nseg, s.cuda_stream) == 0
        b.record(s)
        torch.cuda.synchronize()
        known = int(LIB.ubench_cal_bytes(shape, nv, R, nseg))
        us = a.elapsed_time(b) / 2 * 1e3
        print(json.dumps({"cal": i, "shape": shape, "R": R, "nseg": nseg, "what": name,
                          "known_bytes": known, "us": round(us, 1),
                          "known_GBps": round(known / us / 1e3, 1)}), flush=True)


LIB.ubench_pass1_arith.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                   ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                   ctypes.POINTER(ctypes.c_int)]
LIB.ubench_pass1_arith.restype = ctypes.c_int
MK_NAMES = {0: "mod_fast (segments)", 1: "mod_wide (segments)", 2: "p2 (segments)",
            3: "ladder stack", 4: "ladder build", 5: "ladder build, block (x >> 24) % d"}
# the product's geometries: (name, filter sizes); one size = a build, several = a stacked probe
PASS1_CASES = [("C2 build", [167_772_160]), ("C5 build", [671_088_640]),
               ("C4 build", [3_221_225_472]), ("C3 probe (5-level ladder)",
                                               [655_360 * 4 ** i for i in range(4, -1, -1)]),
               ("f10 build (b=1000, f=10, r=10: m = 15625 << 15)", [512_000_000]),
               ("f10 probe (3 levels, m = 5.12M * 10^i)", [512_000_000, 51_200_000, 5_120_000])]


def pass1_arith(buf, grid, block, iters=256, reps=5):
    """The compute ceiling of pass 1 per geometry: the three hashes plus the
    bin and entry of each position, exactly as k_part_bin forms them
    (ubench_pass1_arith), compute only."""
    import numpy as np
    s = torch.cuda.current_stream()
    for name, sizes in PASS1_CASES:
        ms_arr = np.array(sizes, dtype=np.uint64)
        mk = ctypes.c_int(-1)
        run = lambda: LIB.ubench_pass1_arith(len(sizes), ms_arr.ctypes.data, grid, block, iters,  # noqa: E731
                                             buf.data_ptr(), s.cuda_stream, ctypes.byref(mk))
        if run() != 0:
            print(json.dumps({"op": "pass1 arithmetic", "case": name, "skipped": True}), flush=True)
            continue
        ms = _events(run, reps)
        print(json.dumps({"op": "pass1 arithmetic", "case": name, "m": sizes,
                          "reduction": MK_NAMES.get(mk.value, mk.value),
                          "Gkeys_s": round(grid * block * iters / ms / 1e6, 1), "ms": round(ms, 4)}),
              flush=True)


def transpose(reps=20):
    """The run-table transpose at C4's shape (16,384 super-tiles x 2,458
    segments) with the column stride = ntiles (the product) and padded by
    16-256 words: the padding tests whether 64 KiB-strided column rows
    collide in the caches."""
    LIB.ubench_transpose.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                     ctypes.c_size_t, ctypes.c_void_p]
    LIB.ubench_transpose.restype = ctypes.c_int
    LIB.ubench_transpose2.argtypes = [ctypes.c_int] + LIB.ubench_transpose.argtypes
    LIB.ubench_transpose2.restype = ctypes.c_int
    variants = [("product", 0), ("loads first, 64 rows", 64), ("loads first, 128 rows", 128)]
    for ntiles, width in ((16384, 2458), (32768, 2458), (4096, 256)):
        rows = torch.randint(0, 2**31 - 1, (ntiles * width,), dtype=torch.int32, device="cuda")
        for name, tr in variants:
            cols = torch.zeros(width * ntiles, dtype=torch.int32, device="cuda")
            s = torch.cuda.current_stream()
            call = (lambda: LIB.ubench_transpose(rows.data_ptr(), cols.data_ptr(), ntiles, width, ntiles,
                                                 s.cuda_stream)) if tr == 0 else \
                (lambda: LIB.ubench_transpose2(tr, rows.data_ptr(), cols.data_ptr(), ntiles, width, ntiles,
                                               s.cuda_stream))
            assert call() == 0
            torch.cuda.synchronize()
            assert torch.equal(cols.view(width, ntiles), rows.view(ntiles, width).t()), (name, ntiles)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            for _ in range(reps):
                call()
            b.record(s)
            torch.cuda.synchronize()
            us = a.elapsed_time(b) / reps * 1000
            print(json.dumps({"op": "transpose", "variant": name, "ntiles": ntiles, "width": width,
                              "us": round(us, 1), "GBps": round(2 * ntiles * width * 4 / us / 1e3, 1)}),
                  flush=True)
            del cols
        for pad in (0, 32):
            cstride = ntiles + pad
            cols = torch.zeros(width * cstride, dtype=torch.int32, device="cuda")
            s = torch.cuda.current_stream()
            rc = LIB.ubench_transpose(rows.data_ptr(), cols.data_ptr(), ntiles, width, cstride, s.cuda_stream)
            assert rc == 0, rc
            torch.cuda.synchronize()
            # correctness: column b, tile t == rows[t * width + b]
            c = cols.view(width, cstride)[:, :ntiles]
            assert torch.equal(c, rows.view(ntiles, width).t()), (ntiles, width, pad)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            for _ in range(reps):
                LIB.ubench_transpose(rows.data_ptr(), cols.data_ptr(), ntiles, width, cstride, s.cuda_stream)
            b.record(s)
            torch.cuda.synchronize()
            us = a.elapsed_time(b) / reps * 1000
            print(json.dumps({"op": "transpose", "ntiles": ntiles, "width": width, "pad_words": pad,
                              "us": round(us, 1),
                              "GBps": round(2 * ntiles * width * 4 / us / 1e3, 1)}), flush=True)
            del cols
        del rows


def main():
    torch.cuda.set_device(0)
    if len(sys.argv) > 1 and sys.argv[1] == "transpose":
        return transpose()
    if len(sys.argv) > 1 and sys.argv[1] == "mixed":
        return mixed()
    if len(sys.argv) > 1 and sys.argv[1] == "cal":
        return cal()
    if len(sys.argv) > 1 and sys.argv[1] == "ladder":
        ladder_ablation()
        return ladder_ablation((0, 1, 2, 3))
    if len(sys.argv) > 1 and sys.argv[1] == "stack":
        stack_ablation()
        return stack_ablation((0, 1, 2, 3))
    if len(sys.argv) > 1 and sys.argv[1] == "p1ab":
        vs = [int(v) for v in os.environ.get("UB_VARIANTS", "5001,5003").split(",")]
        return p1_ab(vs)
    if len(sys.argv) > 1 and sys.argv[1].startswith("p2ab"):
        vs = [int(v) for v in os.environ.get("UB_VARIANTS", "2041").split(",")]
        size = {"p2ab": (16_777_216, 10.0, 50), "p2ab_c5": (67_108_864, 10.0, 20),
                "p2ab_c4": (268_435_456, 12.0, 5)}[sys.argv[1]]
        return p2_ab(vs, *size)
    if len(sys.argv) > 1 and sys.argv[1] == "ldsidle":
        buf = torch.zeros(1 << 20, dtype=torch.int32, device="cuda")
        names = {40: "all lanes random", 41: "odd lanes OR 0 into one shared word",
                 42: "odd lanes masked off", 43: "odd lanes OR 0 into private words",
                 44: "odd lanes OR 0 into random words"}
        for rnd in range(3):
            for v, nm in names.items():
                ms = timeit(v, buf, buf.numel() * 4, 0, 512, 1024, 256)
                print(json.dumps({"op": "lds_or idle lanes", "variant": v, "mode": nm, "round": rnd,
                                  "ms": round(ms, 4)}), flush=True)
        return
    if len(sys.argv) > 1 and sys.argv[1] == "p1abl":
        return p1_ablation()
    if len(sys.argv) > 1 and sys.argv[1] == "p1tail":
        return p1_tail()
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
    for m in [167_772_160, 671_088_640, 3_221_225_472]:  # C2, C5, C4: m = d << t, d | 255
        ms = timeit(7, buf, buf.numel() * 4, m, grid, block, 256)
        print(json.dumps({"op": "hash3+mod_p2", "m": m,
                          "Gkeys_s": round(threads * 256 / ms / 1e6, 1), "ms": round(ms, 4)}),
              flush=True)
    pass1_arith(buf, grid, block)
    ms = timeit(5, buf, buf.numel() * 4, 0, grid, block, 256)
    print(json.dumps({"op": "hash3_raw", "Gkeys_s": round(threads * 256 / ms / 1e6, 1),
                      "ms": round(ms, 4)}), flush=True)
    big = torch.zeros(1 << 28, dtype=torch.int32, device="cuda")  # 1 GiB
    ms = timeit(6, big, big.numel() * 4, 0, 4096, 256, 1)
    print(json.dumps({"op": "stream_read", "GB_s": round(big.numel() * 4 / ms / 1e6, 1),
                      "ms": round(ms, 4)}), flush=True)


if __name__ == "__main__":
    sys.exit(main())
