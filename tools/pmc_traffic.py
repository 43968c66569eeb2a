#!/usr/bin/env python3
"""HBM bytes per build from two rocprofv3 PMC passes (tools/gpu_steps.sh):
FETCH_SIZE and WRITE_SIZE are in KiB.  Each kernel's FETCH_SIZE is scaled by
the line factor measured for the access shapes it issues (KERNEL_SHAPES; all
measure 2.00, below) and WRITE_SIZE taken as it is, by the calibration of
every access shape the product issues
(profiles/pmc_calibration.json, tools/ubench.py cal + tools/pmc_cal.py): on
gfx950 every read request the L2 sends is a whole 128-B line tallied at 64 B
(TCC_BUBBLE stays 0, FETCH_SIZE = TCC_EA0_RDREQ x 64 B), whatever part of
the line the kernel asked for -- coalesced vectors 0.50, half lines 1.00, one
16-B vector per line 4.00, pass 2's walk over runs of 1 / 2 / 8 / 16 vectors
4.00 / 2.00 / 0.50 / 0.50 of the requested bytes, and the half-line and
vector-per-line reads take as long as reading every whole line -- so 2 x
FETCH_SIZE is the line traffic in each shape; WRITE_SIZE equals the stored
bytes for 16-B vector stores and for 2-byte stores that fill their lines
(WRREQ_64B), and counts 32 B per isolated 4-B store (8x: the run table's
column stores), which is the request the memory receives.
Per kernel, the median over the dispatches of its largest grid (the
workload's own build; smaller grids are the tests' warm-up builds).

Usage: pmc_traffic.py WORKLOAD TAG  -> profiles/pmc_WORKLOAD.json
(WORKLOAD c3: the C3 probe's kernels, tools/probe_prof.py; hbm_bytes_per_probe)
(TAG = the tools/gpu_steps.sh tag whose pmc_W step wrote gpurun_out/TAG/pmc_W_*)
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import pmc_summary  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD_KERNELS = ("k_part_bin", "k_part_bin2", "k_runs_transpose", "k_part_apply", "k_build_lds",
                 "k_build_atomic")


PROBE_KERNELS = ("k_part_bin", "k_runs_transpose", "k_part_apply", "k_probe_combine",
                 "k_probe_lds", "k_probe")


def per_kernel_probe(d):
    """The C3 probe's kernels (tools/probe_prof.py): pass 1 with slots, the
    stacked / partitioned pass 2, the combine (and any per-filter probe),
    each at its largest grid."""
    best = {}
    for key, ctrs in pmc_summary.main(d).items():
        name, grid = key.rsplit(" grid=", 1)
        base = name.split("<")[0]
        if base not in PROBE_KERNELS:
            continue
        if base == "k_part_apply" and name.startswith(("k_part_apply<0", "k_part_apply<4")):
            continue  # a build's pass 2
        if base == "k_part_bin":
            targs = [a.strip() for a in name.split("<", 1)[1].split(">")[0].split(",")]
            if len(targs) > 1 and targs[1] != "true":
                continue  # the level builds' pass 1
        if base not in best or int(grid) > best[base][0]:
            best[base] = (int(grid), name, ctrs)
    return best


def per_kernel(d):
    best = {}
    for key, ctrs in pmc_summary.main(d).items():
        name, grid = key.rsplit(" grid=", 1)
        base = name.split("<")[0]
        if base not in BUILD_KERNELS:
            continue
        if base == "k_part_apply" and not name.startswith(("k_part_apply<0", "k_part_apply<4")):
            continue  # probe modes (builds: 0 segments, 4 plan_build's ladder)
        if base == "k_part_bin":
            targs = [a.strip() for a in name.split("<", 1)[1].split(">")[0].split(",")]
            if len(targs) > 1 and targs[1] == "true":
                continue  # SLOTS (probe) variant: k_part_bin<LAYOUT, SLOTS, COLS, TB, WIDE>
        if base not in best or int(grid) > best[base][0]:
            best[base] = (int(grid), name, ctrs)
    return best


# Calibration shapes (profiles/pmc_calibration.json, "cal" ids) each kernel's
# reads and writes take; the read factor of a kernel is the measured line
# bytes per FETCH_SIZE byte over its shapes (128 B x TCC_EA0_RDREQ /
# FETCH_SIZE: every request the L2 sends is one 128-B line, tallied at 64 B).
KERNEL_SHAPES = {
    "k_part_bin": {"read": [0], "write": [7, 9]},        # keys; sorted tiles + run-table columns
    "k_part_bin2": {"read": [0], "write": [7, 9]},       # the same on super-tiles
    "k_runs_transpose": {"read": [0], "write": [7]},
    "k_part_apply": {"read": [3, 4, 5, 6], "write": [7, 8]},  # run walks; segments / result bytes
    "k_probe_combine": {"read": [0], "write": [7]},       # slots + result bytes (+ keys when routing)
    "k_build_lds": {"read": [0], "write": [7]},
    "k_build_atomic": {"read": [0, 2], "write": [9]},
    "k_probe_lds": {"read": [0], "write": [7]},
    "k_probe": {"read": [0, 2], "write": [7]},            # keys + one line per gathered word
}
CAL = os.path.join(ROOT, "profiles", "pmc_calibration.json")


def shape_factors():
    """Per calibration shape: (line bytes per FETCH_SIZE byte, WRITE_SIZE per
    byte the memory receives).  WRITE_SIZE is exact for vector and
    line-filling stores and counts the 32-B request of an isolated 4-B
    store, which is what the memory receives: factor 1 for every shape."""
    out = {}
    for sh in json.load(open(CAL))["shapes"]:
        c = sh["counters"]
        fetch = c.get("FETCH_SIZE", 0.0) * 1024
        out[sh["cal"]] = (128.0 * c["TCC_EA0_RDREQ_sum"] / fetch if fetch else None, 1.0)
    return out


def kernel_factor(base, sf):
    ks = KERNEL_SHAPES.get(base, {"read": [0], "write": [7]})
    rf = [sf[i][0] for i in ks["read"] if sf.get(i) and sf[i][0]]
    return (sum(rf) / len(rf) if rf else 2.0), 1.0, ks


def main(w, tag):
    probe = w == "c3"
    pk = per_kernel_probe if probe else per_kernel
    f = pk(os.path.join(ROOT, "gpurun_out", tag, f"pmc_{w}_FETCH_SIZE"))
    wr = pk(os.path.join(ROOT, "gpurun_out", tag, f"pmc_{w}_WRITE_SIZE"))
    kernels = {}
    total = 0
    sf = shape_factors()
    for base in (PROBE_KERNELS if probe else BUILD_KERNELS):
        if base not in f or base not in wr:
            continue
        rfac, wfac, ks = kernel_factor(base, sf)
        fetch = rfac * f[base][2]["FETCH_SIZE"] * 1024
        write = wfac * wr[base][2]["WRITE_SIZE"] * 1024
        kernels[base] = {"name": f[base][1], "grid": f[base][0], "fetch_bytes": int(fetch),
                         "write_bytes": int(write), "fetch_factor": round(rfac, 4),
                         "write_factor": wfac, "calibration_shapes": ks}
        total += fetch + write
    if not kernels:  # a pass is missing (e.g. the GPU call failed): keep the old summary
        sys.exit(f"pmc_traffic: no build kernels in gpurun_out/{tag}/pmc_{w}_*; nothing written")
    sys.path.insert(0, ROOT)
    from bench import library_kernel_sha as kernel_source_sha
    out = {"workload": w, "round": tag,
           ("hbm_bytes_per_probe" if probe else "hbm_bytes_per_build"): int(total),
           "kernels": kernels,
           "kernel_source_sha": kernel_source_sha(),
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes "
                     "(tools/gpu_steps.sh pmc_W); KiB -> bytes; FETCH_SIZE x each kernel's "
                     "measured line factor and WRITE_SIZE x its write factor over the "
                     "calibration shapes it issues (profiles/pmc_calibration.json); median per "
                     "dispatch of each kernel's largest grid, summed over the call"}
    path = os.path.join(ROOT, "profiles", f"pmc_{w}.json")
    json.dump(out, open(path, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
