#!/usr/bin/env python3
"""Diagnosis of the one-pass k-way compaction (ubench_kway): the bench's
fan-in-4 runs, each ablation timed with HIP events over 20 launches."""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cs265-lsm-tree_amd"))
from bloomhip import workloads as W  # noqa: E402

LIB = ctypes.CDLL(os.path.join(ROOT, "cs265-lsm-tree_amd", "lib", "libbloomhip_ubench.so"))
LIB.ubench_kway.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                            ctypes.c_void_p]
LIB.ubench_kway_ws.argtypes = [ctypes.c_void_p, ctypes.c_int]
LIB.ubench_kway_ws.restype = ctypes.c_uint64


def main():
    runs, _ = W.compaction_fanin()
    dr = [torch.from_numpy(r).cuda() for r in runs]
    k = len(dr)
    ptrs = (ctypes.c_void_p * k)(*[d.data_ptr() for d in dr])
    ns = (ctypes.c_uint64 * k)(*[d.shape[0] for d in dr])
    total = sum(d.shape[0] for d in dr)
    out = torch.empty(2 * total + 2 * 4096 * 16384, dtype=torch.int32, device="cuda")
    keys = torch.empty(total + 4096 * 16384, dtype=torch.int32, device="cuda")
    ws = torch.empty(LIB.ubench_kway_ws(ns, k) // 4 + 64, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(4, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    names = {0: "product", 1: "no look-back", 2: "no merge rounds", 3: "no staging loads",
             4: "samples + split only", 5: "blockIdx, no ticket", 6: "no output writes",
             7: "no ticket, no look-back", 8: "no ticket, no look-back, no writes"}
    for rnd in range(2):
        for abl in names:
            def run():
                assert LIB.ubench_kway(abl, ptrs, ns, k, out.data_ptr(), keys.data_ptr(),
                                       ws.data_ptr(), cnt.data_ptr(), s.cuda_stream) == 0
            for _ in range(5):
                run()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            for _ in range(20):
                run()
            b.record(s)
            torch.cuda.synchronize()
            print(json.dumps({"round": rnd, "variant": names[abl], "us": round(a.elapsed_time(b) / 20 * 1e3, 1),
                              "kept": int(cnt[0].item())}), flush=True)


if __name__ == "__main__":
    main()
