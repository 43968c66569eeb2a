#!/usr/bin/env python3
"""Turns the reference's own golden tests (jackdent/cs265-lsm-tree
test/test-{1..6}/{in,out,params,data.bin}, run by scripts/test.py:15-46) into
DATA fixtures: tests/golden/ref_tests.json holds, per test, the CLI params, the
workload as a list of operations (["p", key, val], ["g", key], ["r", lo, hi],
["d", key], ["l", file]), the load files' bytes (hex) and the expected stdout.
No reference text is stored: the operations are parsed into numbers here and
the DSL lines are rebuilt from them at test time (tests/test_dropin.py).

Run in the build container (where /root/reference exists):
    python tests/golden/make_ref_tests.py
"""
import json
import os
import sys

REF = os.environ.get("BLOOMHIP_REFERENCE", "/root/reference")
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "ref_tests.json")


def parse_ops(text):
    # the reference's command_loop (src/main.cpp:15-47): whitespace-separated
    # tokens, except `l` which takes the rest of the line as a quoted path
    ops = []
    for line in text.splitlines():
        line = line.strip()
        if not line:
            continue
        c = line[0]
        rest = line[1:].strip()
        if c == "l":
            ops.append(["l", rest.strip('"')])
        elif c in "pr":
            a, b = rest.split()
            ops.append([c, int(a), int(b)])
        elif c in "gd":
            ops.append([c, int(rest)])
        else:
            raise ValueError(f"unknown command {line!r}")
    return ops


def main():
    tests = {}
    root = os.path.join(REF, "test")
    for name in sorted(os.listdir(root)):
        d = os.path.join(root, name)
        if not name.startswith("test-") or not os.path.isdir(d):
            continue
        with open(os.path.join(d, "in")) as f:
            ops = parse_ops(f.read())
        with open(os.path.join(d, "out")) as f:
            expected = f.read()
        params = []
        if os.path.exists(os.path.join(d, "params")):
            with open(os.path.join(d, "params")) as f:
                params = f.read().split()
        files = {}
        for op in ops:
            if op[0] == "l":
                with open(os.path.join(d, op[1]), "rb") as f:
                    files[op[1]] = f.read().hex()
        tests[name] = {"params": params, "ops": ops, "files": files, "expected_stdout": expected}
    with open(OUT, "w") as f:
        json.dump({"source": "jackdent/cs265-lsm-tree test/test-*/ (scripts/test.py:15-46)",
                   "tests": tests}, f, separators=(",", ":"))
    print(f"wrote {OUT}: {', '.join(tests)}", file=sys.stderr)


if __name__ == "__main__":
    main()
