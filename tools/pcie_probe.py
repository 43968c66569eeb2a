#!/usr/bin/env python3
"""PCIe floor of the e2e legs: pinned H2D of C2's 67 MB of keys
and D2H of its 21 MB bitmap, alone, split over streams, and both directions
at once.  Prints one JSON object per measurement."""
import json
import time

import torch


def timed(fn, reps=10):
    ts = []
    for i in range(reps + 2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        if i >= 2:
            ts.append(time.perf_counter() - t0)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    torch.cuda.set_device(0)
    n_in, n_out = 16_777_216 * 4, 167_772_160 // 8
    hin = torch.empty(n_in, dtype=torch.uint8).pin_memory()
    hout = torch.empty(n_out, dtype=torch.uint8).pin_memory()
    din = torch.empty(n_in, dtype=torch.uint8, device="cuda")
    dout = torch.empty(n_out, dtype=torch.uint8, device="cuda")
    streams = [torch.cuda.Stream() for _ in range(4)]

    def rep(name, t, nbytes):
        print(json.dumps({"op": name, "ms": round(t * 1e3, 3), "GB_s": round(nbytes / t / 1e9, 1)}),
              flush=True)

    rep("h2d 67 MB", timed(lambda: din.copy_(hin, non_blocking=True)), n_in)
    rep("d2h 21 MB", timed(lambda: hout.copy_(dout, non_blocking=True)), n_out)
    for k in (2, 4):
        def split():
            c = n_in // k
            for i in range(k):
                with torch.cuda.stream(streams[i % len(streams)]):
                    din[i * c:(i + 1) * c].copy_(hin[i * c:(i + 1) * c], non_blocking=True)
        rep(f"h2d 67 MB in {k} chunks on {min(k, 4)} streams", timed(split), n_in)

    def both():
        with torch.cuda.stream(streams[0]):
            din.copy_(hin, non_blocking=True)
        with torch.cuda.stream(streams[1]):
            hout.copy_(dout, non_blocking=True)
    rep("h2d 67 MB || d2h 21 MB", timed(both), n_in + n_out)


if __name__ == "__main__" and len(__import__("sys").argv) == 1:
    main()


def e2e_parts():
    """The C2 e2e build's parts: copy-then-build vs host keys staged by the
    library, each with and without the bitmap D2H."""
    import os
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "cs265-lsm-tree_amd"))
    import bloomhip as bh
    from bloomhip import workloads as W
    keys, m = W.c2()
    pinned = torch.from_numpy(keys).pin_memory()
    dk = torch.empty_like(pinned, device="cuda")
    f = bh.BloomFilter(m)
    hw = torch.empty(f.nwords, dtype=torch.int64).pin_memory()
    s = torch.cuda.current_stream()

    def copy_build():
        dk.copy_(pinned, non_blocking=True)
        f.clear(stream=s)
        f.set_batch(dk, stream=s)

    def host_build():
        f.clear(stream=s)
        f.set_batch(pinned, stream=s)

    def dl():
        bh.lib().bloomhip_download(f.handle, hw.data_ptr(), f.nwords, s.cuda_stream)
    for name, fn in (("copy+build", copy_build), ("host build", host_build),
                     ("copy+build+d2h", lambda: (copy_build(), dl())),
                     ("host build+d2h", lambda: (host_build(), dl())), ("d2h", dl)):
        print(json.dumps({"op": name, "ms": round(timed(fn) * 1e3, 3)}), flush=True)


if __name__ == "__main__" and len(__import__("sys").argv) > 1:
    e2e_parts()
