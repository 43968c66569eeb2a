#!/usr/bin/env python3
"""Throughput of single gfx950 VALU instructions (csrc/ubench_isa.hip): SIMD
cycles per wave instruction at the busy clock, 8 independent chains per lane.
Prints one JSON line per instruction.  Usage: python tools/ubench_isa.py"""
import ctypes
import json
import os

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = ctypes.CDLL(os.path.join(ROOT, "cs265-lsm-tree_amd", "lib", "libbloomhip_ubisa.so"))
NAMES = ["mad_u64_u32", "lshl_add_u64", "lshlrev_b64", "lshrrev_b64", "add_u64 (lshl_add 0)",
         "xor_b32", "mul_lo_u32", "mul_hi_u32", "alignbit", "mad_u32_u24", "add_u32",
         "lshl_add_u32", "bitop3_b32 (xor3)", "alignbit (same reg)"]
CHAINS, ITERS, BLOCK = 8, 4096, 256


def main():
    dev = torch.device("cuda", 0)
    sink = torch.zeros(1, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream(dev)
    props = torch.cuda.get_device_properties(dev)
    grid = props.multi_processor_count * 8  # 8 waves per SIMD
    waves = grid * BLOCK // 64
    sclk = 2.4e9
    for which, name in enumerate(NAMES):
        for _ in range(3):  # warm
            LIB.ubench_isa(which, ctypes.c_void_p(sink.data_ptr()), grid, BLOCK, ITERS,
                           ctypes.c_void_p(s.cuda_stream))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(5):
            rc = LIB.ubench_isa(which, ctypes.c_void_p(sink.data_ptr()), grid, BLOCK, ITERS,
                                ctypes.c_void_p(s.cuda_stream))
            assert rc == 0, rc
        e1.record(s)
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) / 5 * 1e-3
        inst = waves * ITERS * CHAINS  # wave instructions
        per_simd = inst / (props.multi_processor_count * 4)
        print(json.dumps({"instr": name, "ms": round(t * 1e3, 4),
                          "simd_cycles_per_wave_instr_at_2.4GHz": round(t * sclk / per_simd, 2)}))


if __name__ == "__main__" and not os.environ.get("UB_CHECK"):
    main()


def lshl_add_check(n=1 << 20):
    """v_lshl_add_u64 with immediate shifts 0..7 against (a << s) + b."""
    import numpy as np
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(5)
    ab = rng.integers(0, 2**63, size=2 * n, dtype=np.int64).view(np.uint64)
    ab[:64] = np.uint64(2**64 - 1)
    inp = torch.from_numpy(ab.view(np.int64)).to(dev)
    out = torch.empty(8 * n, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream(dev)
    assert LIB.ubench_lshl_add_check(ctypes.c_void_p(inp.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                     n, ctypes.c_void_p(s.cuda_stream)) == 0
    got = out.cpu().numpy().view(np.uint64).reshape(n, 8)
    a, b = ab[0::2], ab[1::2]
    for sh in range(8):
        want = (a << np.uint64(sh)) + b
        print(json.dumps({"v_lshl_add_u64_shift": sh, "exact": bool((got[:, sh] == want).all()),
                          "mismatches": int((got[:, sh] != want).sum())}))


if __name__ == "__main__" and os.environ.get("UB_CHECK"):
    lshl_add_check()
