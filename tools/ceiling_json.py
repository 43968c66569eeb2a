#!/usr/bin/env python3
"""profiles/<round>/compute_ceiling.json from a `tools/ubench.py` (prim) log:
the hash + remainder rates and pass 1's whole per-key arithmetic per product
geometry (bench.py's compute_ceiling reads it).
Usage: ceiling_json.py UB_PRIM_LOG OUT_JSON"""
import json
import sys


def main(log, out_path):
    rows = [json.loads(l) for l in open(log) if l.startswith("{")]
    out = {"source": f"{log} (tools/ubench.py, compute only: grid 2048 x 256 threads x 256 keys "
                     f"each, MI355X)",
           "note": "pass1_arithmetic = the three hashes plus, per hash, the bin and entry exactly "
                   "as k_part_bin forms them for the product's geometry (bin_entry): the VALU "
                   "ceiling of a build's or probe's pass 1",
           "hash3_raw": None, "hash3_mod_fast": {}, "hash3_mod_p2": {}, "pass1_arithmetic": {}}
    for r in rows:
        op = r.get("op")
        if op == "hash3_raw":
            out["hash3_raw"] = r["Gkeys_s"]
        elif op == "hash3+mod_fast":
            out["hash3_mod_fast"][str(r["m"])] = r["Gkeys_s"]
        elif op == "hash3+mod_p2":
            out["hash3_mod_p2"][str(r["m"])] = r["Gkeys_s"]
        elif op == "pass1 arithmetic" and not r.get("skipped"):
            out["pass1_arithmetic"][r["case"]] = {"m": r["m"], "reduction": r["reduction"],
                                                  "Gkeys_s": r["Gkeys_s"]}
    json.dump(out, open(out_path, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
