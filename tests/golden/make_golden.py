"""Regenerates tests/golden/ fixtures.

Two kinds of vectors live here, kept apart on purpose:

* ``kat.json`` / the ``reference`` block of ``pins.json``: values produced by
  the compiled REFERENCE (src/bloom_filter.cpp) and recorded in SURVEY.md §8a
  (known-answer positions), §0 F4 (m sizing) and §8c (C2 popcount, C3
  per-level popcounts and GET hit counts).  They are transcribed, not
  computed, and they pin the oracle.
* the ``oracle`` block of ``pins.json``: SHA-256 / popcount summaries of the
  full-size config bitmaps and probe results, computed by the C oracle
  (oracle/bloom_oracle.c) once it reproduces every reference value above, so
  the GPU tests can check full-size outputs without re-running the oracle on
  the GPU box.  ``c1_bitmap.npy`` is the complete C1 bitmap.

Run:  python tests/golden/make_golden.py   (about a minute, ~6 GB RAM)
      python tests/golden/make_golden.py f10   (adds / refreshes only the
      f = 10 tree's pins in pins.json, leaving the rest as they are)
      python tests/golden/make_golden.py route   (only the routing pins of
      C3 and of the f = 10 tree, and the fan-in-4 compaction's pins)
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "cs265-lsm-tree_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

from bloom_oracle import COracle  # noqa: E402
from bloomhip import workloads as W  # noqa: E402

# SURVEY.md §8a — positions (h1, h2, h3) from the compiled reference.
KAT = [
    (64, 0, 0, 39, 42),
    (64, -1, 27, 2, 42),
    (65, 1, 4, 50, 46),
    (655_360, 13141, 217_482, 93_735, 604_771),
    (167_772_160, 1, 148_245_494, 4_227_510, 52_440_221),
    (167_772_160, -1, 148_263_835, 77_775_234, 34_163_050),
    (167_772_160, -2_147_483_648, 460_113, 95_837_670, 131_010_982),
    (167_772_160, 2_147_483_647, 65_286_525, 9_110_449, 30_347_686),
    (3_221_225_472, 0, 1_073_741_824, 1_535_891_751, 2_148_092_266),
    (3_221_225_472, -2_652_462, 2_157_924_537, 2_778_713_131, 2_380_357_233),
    (1_000_003, 2_147_483_647, 392_887, 423_937, 974_107),
]
# SURVEY.md §0 F4 — Run::Run sizing (float product truncated to long).
M_BITS = [
    (16_777_217, 10.0, 167_772_160),
    (33_554_431, 0.5, 16_777_216),
    (51_200, 7.7, 394_240),
    (512, 0.5, 256),
    (51_200, 10.0, 512_000),
    (16_777_216, 10.0, 167_772_160),
    (268_435_456, 12.0, 3_221_225_472),
    (67_108_864, 10.0, 671_088_640),
]
# SURVEY.md §8c — from the compiled reference.
REFERENCE = {
    "c2_popcount": 43_405_815,
    "c3_popcount": [169_910, 678_737, 2_717_085, 10_866_343, 43_405_315],
    "c3_hits": [291_488, 292_356, 294_875, 306_086, 10_207_638],
}


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def f10_pins(C):
    """The reference's published tree geometry (workloads F10): the build of
    16.8M keys into level 2's filter, and each level's filter + hit rows."""
    kb, mb = W.f10_build()
    wb = C.build(mb, kb)
    out = {"build": {"m": mb, "n": int(kb.size), "sha256": sha(wb), "popcount": C.popcount(wb)}}
    del wb
    gets, levels = W.f10()
    out["gets_sha256"] = sha(gets)
    out["levels"] = []
    for lvl, keys, m in levels:
        w = C.build(m, keys)
        hits = C.test(w, m, gets)
        out["levels"].append({"level": lvl, "m": m, "n": int(keys.size), "sha256": sha(w),
                              "popcount": C.popcount(w), "hits_sha256": sha(hits),
                              "hits": int(np.unpackbits(hits.view(np.uint8)).sum())})
    return out


def route_pins(C, gets, levels):
    """bo_route (src/run.cpp:93-99 over LSMTree::get's runs) of `gets` over
    the level runs (distinct keys ascending, newest level first): SHA-256 of
    the candidate rows, of first and page, and of their packed form
    (first << 28 | page, 0xFFFFFFFF for none: bloomhip_route_gets_packed)."""
    runs = []
    for lvl, keys, m in levels:
        fences, mk = C.run_meta(keys)
        runs.append((C.build(m, keys), m, fences, mk))
    cand, first, page = C.route(runs, gets)
    packed = np.where(first < 0, np.uint32(0xFFFFFFFF),
                      (first.astype(np.uint32) << np.uint32(28)) | page.astype(np.uint32))
    return {"cand_sha256": sha(cand), "first_sha256": sha(first), "page_sha256": sha(page),
            "route_sha256": sha(packed.astype(np.uint32)),
            "keys_with_candidate": int((first >= 0).sum())}


def compact_pins(C):
    """bo_compact (src/merge.cpp:17-35, newest wins, tombstones dropped) of
    the fan-in-4 compaction (workloads.compaction_fanin) and the new run's
    filter built over the merged keys (entry_t stride 8)."""
    runs, m = W.compaction_fanin()
    merged = C.compact(runs, drop_tombstones=True)
    w = C.build(m, merged.reshape(-1), stride=8, n=merged.shape[0])
    return {"m": m, "entries_in": int(sum(r.shape[0] for r in runs)),
            "entries_out": int(merged.shape[0]), "merged_sha256": sha(merged),
            "filter_sha256": sha(w)}


def main():
    C = COracle()
    if sys.argv[1:] in (["f10"], ["route"]):
        path = os.path.join(HERE, "pins.json")
        with open(path) as f:
            pins = json.load(f)
        if sys.argv[1] == "f10":
            pins["oracle"]["f10"] = f10_pins(C)
        else:
            pins["oracle"]["route_c3"] = route_pins(C, *W.c3_runs())
            pins["oracle"]["f10"]["route"] = route_pins(C, *W.f10_runs())
            pins["oracle"]["compact_fanin4"] = compact_pins(C)
        with open(path, "w") as f:
            json.dump(pins, f, indent=1)
        print("updated", path)
        return
    for m, k, a, b, c in KAT:
        assert C.positions([k], m)[0].tolist() == [a, b, c], (m, k)
    for size, bpe, m in M_BITS:
        assert C.m_bits(size, bpe) == m
    oracle = {}

    run, m1 = W.c1_run()
    w1 = C.build(m1, run.reshape(-1), stride=8, n=run.shape[0])
    np.save(os.path.join(HERE, "c1_bitmap.npy"), w1)
    oracle["c1"] = {"m": m1, "n": int(run.shape[0]), "sha256": sha(w1), "popcount": C.popcount(w1),
                    "run_sha256": sha(run)}

    k2, m2 = W.c2()
    w2 = C.build(m2, k2)
    assert C.popcount(w2) == REFERENCE["c2_popcount"]
    oracle["c2"] = {"m": m2, "n": int(k2.size), "sha256": sha(w2), "popcount": C.popcount(w2),
                    "keys_sha256": sha(k2)}
    del w2

    gets, levels = W.c3()
    c3 = {"gets_sha256": sha(gets), "levels": []}
    for lvl, keys, m in levels:
        w = C.build(m, keys)
        hits = C.test(w, m, gets)
        assert C.popcount(w) == REFERENCE["c3_popcount"][lvl]
        assert int(np.unpackbits(hits.view(np.uint8)).sum()) == REFERENCE["c3_hits"][lvl]
        c3["levels"].append({"level": lvl, "m": m, "n": int(keys.size), "sha256": sha(w),
                             "popcount": C.popcount(w), "hits_sha256": sha(hits),
                             "hits": int(np.unpackbits(hits.view(np.uint8)).sum())})
    oracle["c3"] = c3
    del gets, levels

    k4, m4 = W.c4()
    w4 = C.build(m4, k4)
    oracle["c4"] = {"m": m4, "n": int(k4.size), "sha256": sha(w4), "popcount": C.popcount(w4)}
    del k4, w4

    c5 = []
    for r in range(W.C5_RUNS):
        k5, m5 = W.c5_run(r)
        w5 = C.build(m5, k5)
        c5.append({"run": r, "m": m5, "n": int(k5.size), "sha256": sha(w5),
                   "popcount": C.popcount(w5)})
    oracle["c5"] = c5
    oracle["f10"] = f10_pins(C)
    oracle["route_c3"] = route_pins(C, *W.c3_runs())
    oracle["f10"]["route"] = route_pins(C, *W.f10_runs())
    oracle["compact_fanin4"] = compact_pins(C)

    with open(os.path.join(HERE, "kat.json"), "w") as f:
        json.dump({"source": "SURVEY.md §8a / §0 F4 (compiled reference)",
                   "positions": [dict(m=m, key=k, h=[a, b, c]) for m, k, a, b, c in KAT],
                   "m_bits": [dict(max_size=s, bpe=b, m=m) for s, b, m in M_BITS]}, f, indent=1)
    with open(os.path.join(HERE, "pins.json"), "w") as f:
        json.dump({"reference": REFERENCE, "oracle": oracle}, f, indent=1)
    print("wrote", HERE)


if __name__ == "__main__":
    main()
