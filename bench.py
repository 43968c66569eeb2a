#!/usr/bin/env python3
"""bench.py — device-resident Bloom-filter build throughput on MI355X.

Workload (BASELINE.json configs[1]): one LSM run of
16,777,216 int32 keys (generator --puts 16777216, seed 13141 + rank),
m = (long)(16777216 * 10.0f) = 167,772,160 bits, k = 3 (the reference's
three fixed hashes; config 2's "k=7" is not expressible bit-exactly).
A step = clear the filter + build it from the device-resident key vector
(bloomhip_set_batch).  With --gpus N every rank builds its own run on its own
GPU (per-run sharding, no collective on the data path): weak scaling.

Also reported at N=1: the C3 batched probe (16.7M GETs x 5 level filters),
the end-to-end (host keys -> filter -> host bitmap) rate, and the CPU
baseline (the oracle's C restatement, 1 thread) on the same keys.

Prints ONE JSON line on rank 0.
"""
import argparse
import hashlib
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "cs265-lsm-tree_amd"))

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
BASELINE_METRIC = "Bloom build+probe Gkeys/s device-resident; achieved HBM GB/s vs roofline"

WORKLOADS = {
    # name: (keys per run, bits per entry)
    "c2": (16_777_216, 10.0),
    "c5": (67_108_864, 10.0),
    "c4": (268_435_456, 12.0),
    # a run whose filter needs 64-bit positions: m = 2^32 bits (512 MiB)
    "c4w": (268_435_456, 16.0),
}
BUILD_SLOTS = ("k_build_atomic", "k_build_lds", "k_part_bin", "k_part_apply",
               "part_counts(memset)")


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def _med(fn, reps=3):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts)


def host_cpu_info():
    """nproc as the verdict asks (os.cpu_count), plus what this process may
    actually run on: its affinity mask and the cgroup CPU quota."""
    info = {"host_cpus": os.cpu_count()}
    try:
        info["affinity_cpus"] = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        info["affinity_cpus"] = None
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()
            quota = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    info["cgroup_cpu_quota"] = quota
    try:
        with open("/proc/cpuinfo") as f:
            info["cpu_model"] = next(l.split(":", 1)[1].strip() for l in f
                                     if l.startswith("model name"))
    except (OSError, StopIteration):
        info["cpu_model"] = "unknown"
    return info


def usable_cpus(info):
    """The CPUs this process can actually run on: min(nproc, affinity mask,
    cgroup CPU quota) — the box shows 256 CPUs but grants a 16-CPU quota."""
    c = [info["host_cpus"] or 1]
    if info.get("affinity_cpus"):
        c.append(info["affinity_cpus"])
    if info.get("cgroup_cpu_quota"):
        c.append(max(1, int(info["cgroup_cpu_quota"])))
    return min(c)


def cpu_baseline(keys, m, reps=5):
    """The oracle's C restatement (oracle/bloom_oracle.c, -O2) building the same
    C2 filter on T = nproc native threads (bo_build_mt: contiguous key slices,
    atomic ORs into the one bitmap; bit-identical to the sequential build)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from bloom_oracle import COracle
    C = COracle()
    info = host_cpu_info()
    T = usable_cpus(info)
    C.build_mt(m, keys[:1_000_000], T)  # warm-up (threads, pages)
    t = _med(lambda: C.build_mt(m, keys, T), reps)
    return {"value": round(keys.size / t / 1e9, 5), "unit": "Gkeys/s", "cores": T,
            "kind": "port", "nproc": info["host_cpus"],
            "cgroup_cpu_quota": info["cgroup_cpu_quota"],
            "sample": f"full C2 run: {keys.size} keys, m={m}; oracle/bloom_oracle.c -O2 on "
                      f"{T} native threads = min(nproc {info['host_cpus']}, affinity "
                      f"{info['affinity_cpus']}, cgroup quota {info['cgroup_cpu_quota']}), "
                      f"median of {reps} ({t * 1e3:.1f} ms each)"}


def cpu_baseline_detail(keys, m):
    """SURVEY §8d's CPU plan beside the headline baseline: T = 1 and T = nproc;
    the reference's own flags (-O0 -g, Makefile:4) on the full C2 run; one
    filter per thread (per-run builds, as C5); the C3 probe split over T
    threads.  Native threads inside the oracle library (no Python threads).
    Bounded: a few seconds of CPU in all."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from bloom_oracle import COracle
    from bloomhip import workloads as W
    import numpy as np
    T = usable_cpus(host_cpu_info())
    C0, C2 = COracle("O0"), COracle()
    t_o0 = _med(lambda: C0.build(m, keys), 1)
    t_1 = _med(lambda: C2.build(m, keys), 3)
    # T per-run builds: each thread builds its own filter from a C2-sized
    # slice of keys (the key stream repeated; per-thread work = one C2 build)
    many_n = 1 << 22
    many = np.resize(keys, T * many_n).reshape(T, many_n)
    t_many = _med(lambda: C2.build_many(m, many), 2)
    gets, levels = W.c3()
    filt = [(C2.build(mm, k), mm) for _, k, mm in levels]
    t_probe1 = _med(lambda: [C2.test(w, mm, gets[:1 << 22]) for w, mm in filt], 1)
    t_probe = _med(lambda: [C2.test_mt(w, mm, gets, T) for w, mm in filt], 2)
    out = host_cpu_info()
    out.update({
        "threads": T,
        "build_O0_1thread_gkeys_s": round(keys.size / t_o0 / 1e9, 5),
        "build_O0": f"full C2 run ({keys.size} keys), oracle at the reference's -O0 -g, 1 thread",
        "build_O2_1thread_gkeys_s": round(keys.size / t_1 / 1e9, 5),
        "build_O2_per_run_threads_gkeys_s": round(T * many_n / t_many / 1e9, 4),
        "build_O2_per_run_threads": f"{T} filters (m={m}) of {many_n} keys each, one per "
                                    f"native thread, median of 2",
        "probe_c3_O2_1thread_gkeys_s": round((1 << 22) / t_probe1 / 1e9, 5),
        "probe_c3_O2_threads_gkeys_s": round(gets.size / t_probe / 1e9, 4),
        "probe_c3_O2_threads": f"16.8M C3 GETs x 5 level filters, keys split over {T} threads"})
    return out


def kernel_sources():
    """The device code and its dispatch: csrc/Makefile's KERNEL_SRCS, in order
    (the list the library's compiled-in digest is taken over)."""
    import re
    mk = open(os.path.join(ROOT, "cs265-lsm-tree_amd", "csrc", "Makefile")).read()
    return tuple(re.search(r"^KERNEL_SRCS\s*:?=\s*(.+)$", mk, re.M).group(1).split())


def kernel_source_sha():
    """Digest of the kernel sources: a PMC summary counts for the bench line
    only if it was taken from exactly these kernels."""
    h = hashlib.sha256()
    for name in kernel_sources():
        with open(os.path.join(ROOT, "cs265-lsm-tree_amd", "csrc", name), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def library_kernel_sha():
    """The same digest as compiled into the loaded library (the kernels that
    actually run); differs from kernel_source_sha() when lib/ is stale."""
    import bloomhip as bh
    return bh.lib().bloomhip_kernel_sha().decode()


def pmc_traffic(workload):
    """HBM bytes per build from the committed rocprofv3 PMC summary
    (tools/pmc_traffic.py: FETCH_SIZE x 2 + WRITE_SIZE, MI355X_MICROARCH.md
    HBM section), or None when it is missing or was taken from other kernels."""
    path = os.path.join(ROOT, "profiles", f"pmc_{workload}.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        d = json.load(f)
    if d.get("kernel_source_sha") != library_kernel_sha():
        return {"stale": True, "file": os.path.relpath(path, ROOT)}
    return d


def sysfs_clocks():
    """Current sclk / mclk (MHz) of the GPUs from sysfs (the '*' level of
    pp_dpm_sclk / pp_dpm_mclk); {} where not readable."""
    import glob
    import re
    out = {}
    for dev in sorted(glob.glob("/sys/class/drm/card*/device")):
        rec = {}
        for clk in ("sclk", "mclk"):
            try:
                with open(os.path.join(dev, f"pp_dpm_{clk}")) as f:
                    for line in f:
                        if line.rstrip().endswith("*"):
                            mm = re.search(r"(\d+)\s*Mhz", line, re.I)
                            if mm:
                                rec[clk] = int(mm.group(1))
            except OSError:
                pass
        if rec:
            out[os.path.basename(os.path.dirname(dev))] = rec
    return out


def prewarm(step_fn, torch, min_s=0.3):
    """Untimed, time-based warm-up (>= min_s of back-to-back steps) before the
    --warmup steps: the driver's short runs otherwise time a cold chip.
    Samples the sysfs clocks while the GPU is busy."""
    samples = []
    t0 = time.perf_counter()
    n = 0
    while time.perf_counter() - t0 < min_s:
        for _ in range(50):
            step_fn()
        n += 50
        samples.append(sysfs_clocks())
    torch.cuda.synchronize()
    sclk = [r.get("sclk") for smp in samples for r in smp.values() if r.get("sclk")]
    mclk = [r.get("mclk") for smp in samples for r in smp.values() if r.get("mclk")]
    return {"prewarm_steps": n, "prewarm_s": round(time.perf_counter() - t0, 3),
            "sclk_mhz_busy": max(sclk) if sclk else None,
            "mclk_mhz_busy": max(mclk) if mclk else None,
            "source": "sysfs pp_dpm_sclk/pp_dpm_mclk current level, sampled during prewarm"}


LEG_PREWARM_S = 0.3   # untimed, time-based warm-up of every secondary leg
LEG_MIN_CALLS = 20    # timed calls per secondary leg, whatever --steps is


def time_leg(call, torch, prewarm_s=LEG_PREWARM_S, calls=LEG_MIN_CALLS, sync=None):
    """Wall time per call of a secondary leg: `call` repeated for >= prewarm_s
    untimed, then `calls` calls timed back to back between two device syncs.
    Independent of --steps, so the driver's short runs time a warm chip."""
    sync = sync or torch.cuda.synchronize
    t0 = time.perf_counter()
    n = 0
    while time.perf_counter() - t0 < prewarm_s:
        call()
        n += 1
    sync()
    t0 = time.perf_counter()
    for _ in range(calls):
        call()
    sync()
    return (time.perf_counter() - t0) / max(calls, 1), n


COMPUTE_CEILING = os.path.join("profiles", "r06", "compute_ceiling.json")


def compute_ceiling(case, achieved):
    """The VALU ceiling of a workload's pass 1 (tools/ubench.py prim: the three
    hashes plus each position's bin and entry exactly as k_part_bin forms
    them for this geometry, compute only; profiles/r06/compute_ceiling.json)
    beside the achieved rate: the build cannot beat its own arithmetic."""
    path = os.path.join(ROOT, COMPUTE_CEILING)
    if not os.path.exists(path):
        return None
    d = json.load(open(path))
    c = d["pass1_arithmetic"].get(case)
    if not c:
        return None
    return {"bound": "valu", "unit": "Gkeys/s", "pass1_arithmetic": c["Gkeys_s"],
            "reduction": c["reduction"], "achieved": round(achieved, 2),
            "frac": round(achieved / c["Gkeys_s"], 4),
            "hash3_mod_p2": d["hash3_mod_p2"].get(str(c["m"][0])),
            "source": f"{COMPUTE_CEILING} ({case}; from {d['source'].split(' ')[0]})"}


def load_pins():
    path = os.path.join(ROOT, "tests", "golden", "pins.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        return json.load(f)


def probe_leg(torch, bh, workload="c3"):
    """configs[2] / SURVEY §8d C3 (workload "c3"): 16.8M GETs against the five
    level filters in one call; "f10": the same GETs against the three level
    filters of the reference's published f = 10 tree (workloads.f10).  Each
    level's packed hit row is checked against the oracle's SHA-256 pin
    (tests/golden/pins.json), not only its hit count."""
    import numpy as np
    from bloomhip import workloads as W
    gets, levels = W.c3() if workload == "c3" else W.f10()
    filters = []
    for lvl, keys, m in levels:
        f = bh.BloomFilter(m)
        f.set_batch(keys)
        filters.append(f)
    dgets = torch.from_numpy(gets).cuda()
    nw = (gets.size + 63) // 64
    dout = torch.empty((len(filters), nw), dtype=torch.int64, device="cuda")
    s = torch.cuda.current_stream()
    call = lambda: bh.test_batch(filters, dgets, out=dout, stream=s)  # noqa: E731
    wall, n_pre = time_leg(call, torch)
    # per-launch device time: HIP events on the launch stream, separate pass
    f0 = filters[0]
    f0.profile(True)
    f0.profile_reset()
    for _ in range(LEG_MIN_CALLS):
        call()
    torch.cuda.synchronize()
    prof = f0.profile_read()
    f0.profile(False)
    kms = sum(v["ms"] for k, v in prof.items()
              if k in ("k_probe", "probe_partitioned", "k_probe_lds", "probe_stacked")) / LEG_MIN_CALLS
    hits = dout.cpu().numpy().view("uint64")
    hit_counts = [int(np.unpackbits(hits[j].view(np.uint8)).sum()) for j in range(len(filters))]
    pins = load_pins()
    sha_ok = None
    if pins and workload in pins["oracle"]:
        want = {lv["level"]: lv["hits_sha256"] for lv in pins["oracle"][workload]["levels"]}
        got = {lvl: hashlib.sha256(hits[j].tobytes()).hexdigest()
               for j, (lvl, _, _) in enumerate(levels)}
        sha_ok = got == want
        if not sha_ok:
            log(f"probe {workload}: HIT ROWS DIFFER from the oracle pins")
    algo = 4 * gets.size + sum((m + 63) // 64 * 8 for _, _, m in levels) + len(levels) * nw * 8
    pmc = pmc_traffic(workload) if workload == "c3" else None
    traffic = None if not pmc or pmc.get("stale") else pmc.get("hbm_bytes_per_probe")
    return {"gkeys_s": round(gets.size / (wall * 1e9), 3),
            "kernel_ms": round(kms, 4), "wall_ms": round(wall * 1e3, 4),
            "levels_m_bits": [m for _, _, m in levels],
            "timed_calls": LEG_MIN_CALLS, "prewarm_calls": n_pre,
            "kernels": {k: round(v["ms"] / LEG_MIN_CALLS, 4) for k, v in prof.items()},
            "algorithmic_bytes": algo,
            "achieved_GBps": round(algo / (kms * 1e-3) / 1e9, 1),
            "frac": round(algo / (kms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
            "traffic": traffic,
            "traffic_ratio": round(traffic / algo, 2) if traffic else None,
            "traffic_source": "profiles/pmc_c3.json" if traffic else None,
            "hits_per_level": hit_counts,
            "compute_ceiling": compute_ceiling("C3 probe (5-level ladder)" if workload == "c3"
                                               else "f10 probe (3 levels, m = 5.12M * 10^i)",
                                               gets.size / (kms * 1e-3) / 1e9),
            "hits_sha_match": sha_ok}


def probe_c3(torch, bh):
    return probe_leg(torch, bh, "c3")


def route_c3(torch, bh, workload="c3"):
    """§8f row 1: batched GET routing of C3's 16.8M GETs over the five level
    runs (range check + filter probe + newest candidate + page index), all
    outputs device-resident, the answer packed one u32 per GET
    (bloomhip_route_gets_packed: run << 28 | page); workload "f10": the same
    GETs over the f = 10 tree's three level runs (13,875 fences).  The
    candidate rows and the packed answers of the last timed call are checked
    against the oracle's pins (bo_route, tests/golden/pins.json)."""
    import numpy as np
    from bloomhip import workloads as W
    gets, levels = W.c3_runs() if workload == "c3" else W.f10_runs()
    runs = []
    for lvl, keys, m in levels:
        f = bh.BloomFilter(m)
        f.set_batch_run(keys)
        runs.append(f)
    n = gets.size
    dgets = torch.from_numpy(gets).cuda()
    dc = torch.empty((len(runs), (n + 63) // 64), dtype=torch.int64, device="cuda")
    dr = torch.empty(n, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    wall, n_pre = time_leg(
        lambda: bh.route_gets_packed(runs, dgets, cand=dc, route=dr, stream=s), torch)
    route = dr.cpu().numpy().view(np.uint32)
    routed = int((route != bh.ROUTE_NONE).sum())
    pins = load_pins()
    pin = None
    if pins:
        pin = pins["oracle"].get("route_c3") if workload == "c3" else \
            (pins["oracle"].get("f10") or {}).get("route")
    sha_ok = None
    if pin:
        sha_ok = (hashlib.sha256(dc.cpu().numpy().view(np.uint64).tobytes()).hexdigest() == pin["cand_sha256"]
                  and hashlib.sha256(route.tobytes()).hexdigest() == pin["route_sha256"])
        if not sha_ok:
            log(f"route {workload}: OUTPUTS DIFFER from the oracle pins")
    # SURVEY §8(d)'s probe bytes (keys, every filter, a bit per key and run)
    # plus the routing output (the packed answer: 4 B per key)
    algo = 4 * n + sum((m + 7) // 8 for _, _, m in levels) + len(runs) * n // 8 + 4 * n
    return {"gkeys_s": round(n / (wall * 1e9), 3), "wall_ms": round(wall * 1e3, 4),
            "timed_calls": LEG_MIN_CALLS, "prewarm_calls": n_pre,
            "output": "packed u32 per GET (bloomhip_route_gets_packed)",
            "keys_with_candidate": routed, "algorithmic_bytes": algo,
            "achieved_GBps": round(algo / wall / 1e9, 1),
            "frac": round(algo / wall / 1e9 / HBM_PEAK_GBPS, 4),
            "route_sha_match": sha_ok}


def probe_c3_sharded(torch, bh, dist, rank, world, coll_dev):
    """SURVEY §8e's probe side at N > 1: every rank holds the five C3 level
    filters (built locally from the same run keys: replicas, no collective)
    and probes its contiguous slice of the 16.8M GETs (shard.probe_slice).
    Aggregate rate = all GETs / max over ranks of the timed region."""
    import numpy as np
    from bloomhip import shard
    from bloomhip import workloads as W
    gets, levels = W.c3()
    filters = []
    for lvl, keys, m in levels:
        f = bh.BloomFilter(m, device=torch.cuda.current_device())
        f.set_batch(keys)
        filters.append(f)
    lo, hi = shard.probe_slice(gets.size, rank, world)
    dg = torch.from_numpy(gets[lo:hi]).cuda()
    nw = (hi - lo + 63) // 64
    dout = torch.empty((len(filters), max(nw, 1)), dtype=torch.int64, device="cuda")
    s = torch.cuda.current_stream()

    def sync():
        torch.cuda.synchronize()
        dist.barrier()
    call = lambda: bh.test_batch(filters, dg, out=dout, stream=s)  # noqa: E731
    time_leg(call, torch, calls=0)
    sync()
    el, _ = time_leg(call, torch, prewarm_s=0.0, sync=sync)
    el = shard.max_over_ranks(el, dist, device=coll_dev)
    hits = [int(np.unpackbits(dout[j].cpu().numpy().view(np.uint8)).sum())
            for j in range(len(filters))] if hi > lo else [0] * len(filters)
    tot = [int(shard.sum_over_ranks(h, dist, device=coll_dev)) for h in hits]
    want = None
    pins_path = os.path.join(ROOT, "tests", "golden", "pins.json")
    if os.path.exists(pins_path):
        want = json.load(open(pins_path))["reference"]["c3_hits"]
    return {"gkeys_s": round(gets.size / el / 1e9, 3), "ms": round(el * 1e3, 4),
            "keys_per_rank": hi - lo, "hits_per_level": tot,
            "hits_match_reference": (tot == want) if want is not None else None,
            "note": "filters replicated per GPU, GET keys sharded contiguously, no data collective"}


def c5_eight_runs(torch, bh, dist, rank, world, coll_dev):
    """BASELINE configs[4] / SURVEY §8d C5: 8 independent runs r = 0..7 of
    67,108,864 keys (seed 13141 + r, 10 bits/key), run r built on rank
    r % N, its runs alternating over two streams of its GPU (one run's pass 2
    overlaps the next one's pass 1 at the kernel edges: 3.42 -> 3.36 ms per
    job at N = 1; four streams 3.55, tools/c5_streams.py); no collective on
    the data path.
    A step builds every run once; rate = 8 runs' keys / max over ranks of
    the timed region, so N = 1, 2, 4, 8 time the same fixed job (strong
    scaling of the fan-in).  Each run's bitmap is checked against its
    pinned SHA-256 (tests/golden/pins.json)."""
    from bloomhip import workloads as W
    mine = [r for r in range(8) if r % world == rank]
    built = []
    for r in mine:
        keys, m = W.c5_run(r)
        dk = torch.from_numpy(keys).cuda()
        del keys
        f = bh.BloomFilter(m, device=torch.cuda.current_device())
        built.append((r, dk, f))
    streams = [torch.cuda.current_stream(), torch.cuda.Stream()]

    def step():
        for j, (_, dk, f) in enumerate(built):
            s = streams[j % 2]
            f.clear(stream=s)
            f.set_batch(dk, stream=s)
    step()
    torch.cuda.synchronize()
    pins = None
    pins_path = os.path.join(ROOT, "tests", "golden", "pins.json")
    if os.path.exists(pins_path):
        pins = json.load(open(pins_path))["oracle"]["c5"]
    ok = None if pins is None else all(
        hashlib.sha256(f.words().tobytes()).hexdigest() == pins[r]["sha256"] for r, _, f in built)

    def sync():
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
    # every rank warms up on its own, then the timed calls start together
    time_leg(step, torch, calls=0)
    sync()
    el, _ = time_leg(step, torch, prewarm_s=0.0, sync=sync)
    if dist:
        from bloomhip import shard
        el = shard.max_over_ranks(el, dist, device=coll_dev)
        if ok is not None:
            ok = shard.all_ranks_ok(ok, dist, device=coll_dev)
    n_all = 8 * W.C5_N
    return {"gkeys_s": round(n_all / el / 1e9, 3), "ms": round(el * 1e3, 4),
            "runs_per_rank": len(mine), "keys_per_run": W.C5_N, "m_bits": built[0][2].m if built else None,
            "verified_vs_oracle": ok,
            "note": "8 runs x 64M keys (configs[4]); run r on rank r % N, a rank's runs alternating "
                    "over two streams; rate = all 8 runs / max-rank time"}


def compact_fanin(torch, bh):
    """§8f row 3: a fan-in-4 compaction (4 runs x 4M entries, newest first)
    merged on the device and fused with the new run's filter + fence build
    (bloomhip_compact, synchronous), device-resident in and out."""
    from bloomhip import workloads as W
    runs, m = W.compaction_fanin()
    druns = [torch.from_numpy(r).cuda() for r in runs]
    total = sum(r.shape[0] for r in runs)
    dout = torch.empty((total, 2), dtype=torch.int32, device="cuda")
    f = bh.BloomFilter(m)
    got = [None]

    def call():
        f.clear()
        got[0] = bh.compact(druns, drop_tombstones=True, filter=f, out=dout)
    t, n_pre = time_leg(call, torch)
    n_out = int(got[0].shape[0])
    # the last timed call's merged run and filter against the oracle's pins
    # (bo_compact, src/merge.cpp:17-35, and the filter over its keys)
    pins = load_pins()
    pin = pins["oracle"].get("compact_fanin4") if pins else None
    sha_ok = None
    if pin:
        merged = got[0].cpu().numpy() if hasattr(got[0], "cpu") else got[0]
        sha_ok = (hashlib.sha256(merged.tobytes()).hexdigest() == pin["merged_sha256"]
                  and hashlib.sha256(f.words().tobytes()).hexdigest() == pin["filter_sha256"])
        if not sha_ok:
            log("compaction fan-in 4: OUTPUTS DIFFER from the oracle pins")
    algo = 8 * total + 8 * n_out + (m + 7) // 8  # runs in, merged run out, the new filter
    return {"gentries_s": round(total / t / 1e9, 3), "ms": round(t * 1e3, 3),
            "merged_and_filter_sha_match": sha_ok,
            "timed_calls": LEG_MIN_CALLS, "prewarm_calls": n_pre,
            "entries_in": total, "entries_out": n_out, "algorithmic_bytes": algo,
            "achieved_GBps": round(algo / t / 1e9, 1), "frac": round(algo / t / 1e9 / HBM_PEAK_GBPS, 4),
            "note": "4 sorted runs merged newest-wins + tombstones dropped + filter/fences "
                    "of the merged run built; wall clock per synchronous call"}


def build_leg(torch, bh, keys, m, pin_sha, traffic_workload=None, reps=LEG_MIN_CALLS,
              ceiling_case=None):
    """One device-resident build of `keys` into m bits, repeated: the bitmap
    is checked against the oracle's SHA-256 pin; the device time per build
    comes from HIP events on the launch stream around `reps` back-to-back
    builds (after a time-based prewarm), the roofline from (4N + m/8) per
    build, traffic from profiles/pmc_<traffic_workload>.json."""
    n = keys.size
    dk = torch.from_numpy(keys).cuda()
    f = bh.BloomFilter(m)
    s = torch.cuda.current_stream()

    def step():
        f.clear(stream=s)
        f.set_batch(dk, stream=s)
    step()
    torch.cuda.synchronize()
    ok = None
    if pin_sha:
        ok = hashlib.sha256(f.words().tobytes()).hexdigest() == pin_sha
        if not ok:
            log(f"build of {n} keys into m={m}: BITMAP MISMATCH vs oracle fixture")
    time_leg(step, torch, calls=0)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(s)
    for _ in range(reps):
        step()
    ev1.record(s)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / reps
    dev_ms = ev0.elapsed_time(ev1) / reps
    f.profile(True)
    f.profile_reset()
    for _ in range(reps):
        step()
    torch.cuda.synchronize()
    prof = f.profile_read()
    f.profile(False)
    algo = 4 * n + (m + 63) // 64 * 8
    achieved = algo / (dev_ms * 1e-3) / 1e9
    pmc = pmc_traffic(traffic_workload) if traffic_workload else None
    traffic = None if not pmc or pmc.get("stale") else pmc.get("hbm_bytes_per_build")
    out = {"gkeys_s": round(n / (dev_ms * 1e-3) / 1e9, 3), "device_ms": round(dev_ms, 4),
           "wall_ms": round(wall * 1e3, 4), "builds_timed": reps,
           "keys": n, "m_bits": m, "strategy": bh.STRATEGY_NAMES[f.resolve_strategy(n)],
           "kernels": {k: round(v["ms"] / v["launches"], 4) for k, v in prof.items()},
           "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS,
                        "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                        "traffic": traffic,
                        "traffic_ratio": round(traffic / algo, 2) if traffic else None,
                        "traffic_source": f"profiles/pmc_{traffic_workload}.json" if traffic else None,
                        "algorithmic_bytes": algo},
           "compute_ceiling": compute_ceiling(ceiling_case, n / (dev_ms * 1e-3) / 1e9)
           if ceiling_case else None,
           "verified_vs_oracle": ok}
    del dk, f
    return out


def c4_build(torch, bh, reps=LEG_MIN_CALLS):
    """configs[3] / SURVEY §8d C4: one run of 268,435,456 keys at 12 bits/key
    (m = 3,221,225,472 bits, a 384 MiB bitmap: beyond LDS, L2 and most of
    the Infinity Cache), checked against its oracle pin (build_leg)."""
    from bloomhip import workloads as W
    keys, m = W.c4()
    pins = load_pins()
    out = build_leg(torch, bh, keys, m, pins["oracle"]["c4"]["sha256"] if pins else None,
                    traffic_workload="c4", reps=reps, ceiling_case="C4 build")
    bh.lib().bloomhip_trim()  # the 3 GB partition workspace of this size
    torch.cuda.empty_cache()
    return out


def f10_legs(torch, bh):
    """The reference's own published tree (b = 1000, f = 10, at -r 10:
    doc/final/final.tex:195-212, src/main.cpp:89, src/lsm_tree.cpp:36-41,
    workloads F10): level sizes m = 5,120,000 * 10^i bits, whose odd part
    625 * 5^i takes none of the p2 / ladder paths that C2-C5 (d | 255) take.
    A build of 16.8M keys into level 2's filter (m = 512,000,000) and the
    16.8M C3-style GETs against levels 0..2, each checked against its pin."""
    from bloomhip import workloads as W
    keys, m = W.f10_build()
    pins = load_pins()
    pin = pins["oracle"].get("f10") if pins else None
    return {"build": build_leg(torch, bh, keys, m, pin["build"]["sha256"] if pin else None,
                               ceiling_case="f10 build (b=1000, f=10, r=10: m = 15625 << 15)"),
            "probe": probe_leg(torch, bh, "f10"),
            "route": route_c3(torch, bh, "f10"),
            "note": "reference's published tree b=1000 f=10 at 10 bits/entry: "
                    "m_i = 5,120,000*10^i (odd part 625*5^i)"}


def c1_check(bh):
    """configs[0] / SURVEY §8d C1: the first flushed run of generator --puts
    100000 (-b 100 -r 10) as AoS entry_t {key, val} at stride 8, built on the
    GPU and compared word for word with the oracle's whole bitmap
    (tests/golden/c1_bitmap.npy)."""
    import numpy as np
    from bloomhip import workloads as W
    run, m = W.c1_run()
    f = bh.BloomFilter(m)
    f.set_batch(run.reshape(-1), n=run.shape[0], stride=8)
    got = f.words()
    path = os.path.join(ROOT, "tests", "golden", "c1_bitmap.npy")
    ok = bool((got == np.load(path)).all()) if os.path.exists(path) else None
    return {"entries": int(run.shape[0]), "m_bits": m, "stride": 8,
            "strategy": bh.STRATEGY_NAMES[f.resolve_strategy(run.shape[0])],
            "verified_vs_oracle": ok}


def e2e_build(torch, bh, keys_np, m, reps=10):
    """Host keys (pinned) -> device -> filter -> host bitmap (pinned), wall
    clock: north_star's end-to-end rate (never `value`)."""
    pinned = torch.from_numpy(keys_np).pin_memory()
    f = bh.BloomFilter(m)
    host_words = torch.empty(f.nwords, dtype=torch.int64).pin_memory()
    s = torch.cuda.current_stream()
    dk = torch.empty_like(pinned, device="cuda")
    times = []
    for i in range(reps + 2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        dk.copy_(pinned, non_blocking=True)
        f.clear(stream=s)
        f.set_batch(dk, stream=s)
        bh.lib().bloomhip_download(f.handle, host_words.data_ptr(), f.nwords, s.cuda_stream)
        t = time.perf_counter() - t0
        if i >= 2:
            times.append(t)
    t = statistics.median(times)
    h2d = 4 * keys_np.size
    d2h = 8 * f.nwords
    return {"gkeys_s": round(keys_np.size / t / 1e9, 3), "ms": round(t * 1e3, 3),
            "pcie_bytes": h2d + d2h,
            "note": "pinned host keys H2D + clear + build + bitmap D2H into pinned memory, "
                    "one stream, wall clock, median of 10"}


def e2e_probe_c3(torch, bh, reps=10):
    """north_star's end-to-end probe: pinned host GET keys -> H2D -> the 5-level
    C3 probe -> packed results D2H into pinned memory, wall clock."""
    import numpy as np
    from bloomhip import workloads as W
    gets, levels = W.c3()
    filters = []
    for _, keys, m in levels:
        f = bh.BloomFilter(m)
        f.set_batch(keys)
        filters.append(f)
    nw = (gets.size + 63) // 64
    pinned = torch.from_numpy(gets).pin_memory()
    host_out = torch.empty((len(filters), nw), dtype=torch.int64).pin_memory()
    dg = torch.empty_like(pinned, device="cuda")
    dout = torch.empty((len(filters), nw), dtype=torch.int64, device="cuda")
    s = torch.cuda.current_stream()
    times = []
    for i in range(reps + 2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        dg.copy_(pinned, non_blocking=True)
        bh.test_batch(filters, dg, out=dout, stream=s)
        host_out.copy_(dout, non_blocking=True)
        s.synchronize()
        t = time.perf_counter() - t0
        if i >= 2:
            times.append(t)
    t = statistics.median(times)
    hits = [int(np.unpackbits(host_out[j].numpy().view(np.uint8)).sum())
            for j in range(len(filters))]
    return {"gkeys_s": round(gets.size / t / 1e9, 3), "ms": round(t * 1e3, 3),
            "pcie_bytes": 4 * gets.size + len(filters) * nw * 8, "hits_per_level": hits,
            "note": "pinned host GET keys H2D + 5-level C3 probe + packed results D2H into "
                    "pinned memory, one stream, wall clock, median of 10"}


def scalar_is_set(bh, f, keys_np, calls=4000):
    """Latency of the reference-shaped scalar call (BloomFilter::is_set per
    key, src/run.cpp:93) through bloomhip_is_set: one launch + one sync each.
    Checked against the batch probe of the same keys."""
    import numpy as np
    sample = keys_np[:calls]
    L = bh.lib()
    import ctypes
    hit = ctypes.c_int(0)
    h = f.handle
    for k in sample[:100]:
        L.bloomhip_is_set(h, int(k), ctypes.byref(hit))
    lat = []
    got = np.empty(sample.size, dtype=bool)
    for i, k in enumerate(sample):
        t0 = time.perf_counter()
        rc = L.bloomhip_is_set(h, int(k), ctypes.byref(hit))
        lat.append(time.perf_counter() - t0)
        if rc:
            raise RuntimeError(f"bloomhip_is_set rc={rc}")
        got[i] = bool(hit.value)
    want = np.unpackbits(bh.test_batch([f], sample)[0].view(np.uint8),
                         bitorder="little")[:sample.size].astype(bool)
    lat.sort()
    return {"median_us": round(lat[len(lat) // 2] * 1e6, 2),
            "p99_us": round(lat[int(len(lat) * 0.99)] * 1e6, 2),
            "calls": int(sample.size), "matches_batch": bool((got == want).all()),
            "note": "ctypes -> bloomhip_is_set: key as kernel argument, one single-lane "
                    "kernel on the default stream, answer in a pinned mapped host word"}


def launch_ranks(n):
    """bench.py --gpus N without a launcher (no WORLD_SIZE in the environment):
    start N copies of this command as ranks 0..N-1 of one process group on
    127.0.0.1, one per GPU (LOCAL_RANK = rank), and wait for them.  This
    process never touches a GPU (no torch, no bloomhip), so nothing is
    initialised before the children start.  Returns the first non-zero exit
    status of a rank (the others are then stopped), else 0."""
    import socket
    import subprocess
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env))
    status = 0
    live = list(procs)
    while live:
        for p in list(live):
            rc = p.poll()
            if rc is None:
                continue
            live.remove(p)
            if rc != 0 and status == 0:
                status = rc if rc > 0 else 1
                log(f"bench: rank {procs.index(p)} exited with {rc}; stopping the others")
                for q in live:
                    q.terminate()
        time.sleep(0.05)
    return status


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--workload", default="c2", choices=sorted(WORKLOADS))
    ap.add_argument("--strategy", default="auto", choices=["auto", "atomic", "lds", "partition"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="skip probe/e2e legs")
    ap.add_argument("--no-c5", action="store_true", help="skip the C5 eight-run leg")
    ap.add_argument("--prewarm-s", type=float, default=1.0,
                    help="untimed time-based warm-up before --warmup (0 under profilers)")
    ap.add_argument("--no-c4", action="store_true", help="skip the C4 build leg")
    args = ap.parse_args()
    if args.gpus < 1:
        log(f"--gpus must be >= 1 (got {args.gpus})")
        sys.exit(2)

    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        # Not started by a launcher: become one (nothing has touched a GPU yet).
        sys.exit(launch_ranks(args.gpus))
    world = int(env_world or "1")
    if world != args.gpus:
        log(f"WORLD_SIZE={world} but --gpus {args.gpus}: refusing to measure a different "
            f"number of GPUs than asked for")
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    import numpy as np
    import torch

    import bloomhip as bh
    from bloomhip import shard
    from bloomhip import workloads as W

    # One process per GPU over RCCL.  BLOOMHIP_DIST_BACKEND=gloo rehearses the
    # N > 1 path with several ranks sharing the visible GPUs (CPU collectives).
    backend = os.environ.get("BLOOMHIP_DIST_BACKEND", "nccl")
    if backend == "gloo":
        local = local % max(1, torch.cuda.device_count())
    coll_dev = "cuda" if backend == "nccl" else None
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        else:
            dist.init_process_group(backend)

    n, bpe = WORKLOADS[args.workload]
    seed = W.SEED + rank
    keys = bh.gen_puts(seed, n)
    m = bh.m_bits(n, bpe)
    dkeys = torch.from_numpy(keys).cuda()
    f = bh.BloomFilter(m, device=local)
    strat = {"auto": bh.BUILD_AUTO, "atomic": bh.BUILD_ATOMIC, "lds": bh.BUILD_LDS,
             "partition": bh.BUILD_PARTITION}[args.strategy]
    f.set_strategy(strat)
    resolved = bh.STRATEGY_NAMES[f.resolve_strategy(n)]
    s = torch.cuda.current_stream()

    # Validity: the bitmap a step produces is the oracle-pinned one.
    f.clear(stream=s)
    f.set_batch(dkeys, stream=s)
    torch.cuda.synchronize()
    verified = None
    pins_path = os.path.join(ROOT, "tests", "golden", "pins.json")
    if os.path.exists(pins_path):
        pins = json.load(open(pins_path))["oracle"]
        want = None
        if args.workload == "c2" and seed == W.SEED:
            want = pins["c2"]["sha256"]
        elif args.workload == "c5" and rank < len(pins["c5"]):
            want = pins["c5"][rank]["sha256"]
        elif args.workload == "c4" and seed == W.SEED:
            want = pins["c4"]["sha256"]
        if want is not None:
            got = hashlib.sha256(f.words().tobytes()).hexdigest()
            verified = got == want
            if not verified:
                log(f"rank {rank}: BITMAP MISMATCH vs oracle fixture")

    def step():
        f.clear(stream=s)
        f.set_batch(dkeys, stream=s)

    # Time-based prewarm (untimed), then the --warmup steps, directly before
    # the timed loop (clocks ramp down while idle).
    clocks = prewarm(step, torch, args.prewarm_s)
    for _ in range(args.warmup):
        step()
    # HIP events on the launch stream bracket the K steps as a whole (no
    # per-launch events inside the timed region): the device time per step.
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(s)
    for _ in range(args.steps):
        step()
    ev1.record(s)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    dev_ms_per_step = ev0.elapsed_time(ev1) / args.steps
    if dist:
        elapsed = shard.max_over_ranks(elapsed, dist, device=coll_dev)
        dev_ms_per_step = shard.max_over_ranks(dev_ms_per_step, dist, device=coll_dev)

    # Per-kernel device time: the same K steps again with every launch
    # bracketed by HIP events on the launch stream (kept out of the timed
    # loop above so event records do not perturb it).
    f.profile(True)
    f.profile_reset()
    for _ in range(args.steps):
        f.clear(stream=s)
        f.set_batch(dkeys, stream=s)
    torch.cuda.synchronize()
    prof = f.profile_read()
    f.profile(False)

    if dist:
        all_ok = shard.all_ranks_ok(verified is not False, dist, device=coll_dev)
    else:
        all_ok = verified is not False

    extras = {}
    cpu = None
    if not args.no_extras and not args.no_c5:
        if rank == 0:
            log("C5 eight runs ...")
        extras["c5_eight_runs"] = c5_eight_runs(torch, bh, dist, rank, world, coll_dev)
        torch.cuda.empty_cache()
    if world > 1 and not args.no_extras:
        if rank == 0:
            log("sharded probe C3 ...")
        extras["probe_c3_sharded"] = probe_c3_sharded(torch, bh, dist, rank, world, coll_dev)
    if rank == 0 and world == 1 and not args.no_extras:
        log("C1 stride-8 run ...")
        extras["c1_check"] = c1_check(bh)
        if not args.no_c4:
            log("C4 build ...")
            extras["c4_build"] = c4_build(torch, bh)
        log("probe C3 ...")
        extras["probe_c3"] = probe_c3(torch, bh)
        log("f = 10 tree ...")
        extras["f10"] = f10_legs(torch, bh)
        log("route C3 ...")
        extras["route_c3"] = route_c3(torch, bh)
        log("compact ...")
        extras["compact_fanin4"] = compact_fanin(torch, bh)
        log("e2e ...")
        extras["e2e_build"] = e2e_build(torch, bh, keys, m)
        extras["e2e_probe_c3"] = e2e_probe_c3(torch, bh)
        log("scalar is_set ...")
        extras["scalar_is_set"] = scalar_is_set(bh, f, keys)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        log("cpu baseline ...")
        cpu = cpu_baseline(keys, m)
        if not args.no_extras:
            log("cpu baseline detail ...")
            extras["cpu_baseline_detail"] = cpu_baseline_detail(keys, m)

    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return

    ms_per_step = elapsed / args.steps * 1e3
    value = world * n * args.steps / elapsed / 1e9
    kernels = {k: {"launches": v["launches"], "avg_ms": round(v["ms"] / v["launches"], 5)}
               for k, v in prof.items()}
    build_ms = sum(v["ms"] / v["launches"] for k, v in prof.items() if k in BUILD_SLOTS)
    dominant = max((k for k in prof if k in BUILD_SLOTS),
                   key=lambda k: prof[k]["ms"] / prof[k]["launches"])
    algo = 4 * n + (m + 63) // 64 * 8
    # The build is one unit of work done by its kernels in sequence (two for
    # the partition build), so the roofline is priced on the device time of a
    # whole build in the UNPROFILED timed loop (events around the K steps).
    achieved = algo / (dev_ms_per_step * 1e-3) / 1e9
    pmc = pmc_traffic(args.workload)
    traffic = None if not pmc or pmc.get("stale") else pmc.get("hbm_bytes_per_build")
    line = {
        # BASELINE.json's metric, verbatim; `value` is its build leg on the
        # configs[1] workload (config.workload), the probe leg is probe_c3.
        "metric": BASELINE_METRIC,
        "value": round(value, 4),
        "unit": "Gkeys/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 5),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int32 keys, u64 hash arithmetic",
        "data": "synthetic: generator --puts stream (MT19937 seed 13141+rank), device-resident",
        "config": {"workload": f"{args.workload}: one run per GPU, {n} keys, m={m} bits "
                               f"({bpe} bits/key), k=3, build strategy {resolved}",
                   "keys_per_run": n, "m_bits": m, "parallelism": f"per-run sharding x{world}"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                     "traffic": traffic,
                     "traffic_source": (pmc or {}).get("file") if pmc and pmc.get("stale")
                     else (f"profiles/pmc_{args.workload}.json" if pmc else None),
                     "traffic_stale": bool(pmc and pmc.get("stale")),
                     "kernel": "+".join(k for k in prof if k in BUILD_SLOTS),
                     "dominant": dominant,
                     "algorithmic_bytes": algo,
                     "device_ms_per_build": round(dev_ms_per_step, 5),
                     "profiled_kernel_ms": {k: round(prof[k]["ms"] / prof[k]["launches"], 5)
                                            for k in prof if k in BUILD_SLOTS},
                     "note": "achieved = (4N + m/8) per build / device time per build, HIP "
                             "events on the launch stream around the unprofiled timed loop; "
                             "profiled_kernel_ms = per-launch events in a separate pass"},
        # The build's real ceiling is the VALU: pass 1's own arithmetic (the reference's
        # three 64-bit hashes, the p2 remainder and the bin/entry of each position as
        # k_part_bin forms them) runs at ~531 Gkeys/s on this chip for C2 (compute only,
        # DESIGN.md §4), i.e. 2.8 TB/s = 0.35 of HBM at 5.25 B/key.
        "compute_ceiling": compute_ceiling({"c2": "C2 build", "c5": "C5 build",
                                            "c4": "C4 build"}.get(args.workload, ""),
                                           n / (dev_ms_per_step * 1e-3) / 1e9),
        "clocks": clocks,
        "library": {"kernel_sha": library_kernel_sha(),
                    "matches_sources": library_kernel_sha() == kernel_source_sha()},
        "cpu_baseline": cpu,
        "kernels": kernels,
        "verified_vs_oracle": all_ok if verified is not None or dist else None,
    }
    line.update(extras)
    # Every BASELINE config this run exercised, with its oracle check (None:
    # not run, or no pin for it).
    line["parity"] = {
        "c1_stride8_bitmap": (extras.get("c1_check") or {}).get("verified_vs_oracle"),
        f"{args.workload}_bitmap_sha": line["verified_vs_oracle"],
        "c3_hits_sha": (extras.get("probe_c3") or {}).get("hits_sha_match"),
        "c4_bitmap_sha": (extras.get("c4_build") or {}).get("verified_vs_oracle"),
        "c5_eight_bitmaps_sha": (extras.get("c5_eight_runs") or {}).get("verified_vs_oracle"),
        "f10_build_bitmap_sha": ((extras.get("f10") or {}).get("build") or {}).get("verified_vs_oracle"),
        "f10_hits_sha": ((extras.get("f10") or {}).get("probe") or {}).get("hits_sha_match"),
        "route_c3_sha": (extras.get("route_c3") or {}).get("route_sha_match"),
        "f10_route_sha": ((extras.get("f10") or {}).get("route") or {}).get("route_sha_match"),
        "compact_fanin4_sha": (extras.get("compact_fanin4") or {}).get("merged_and_filter_sha_match"),
    }
    print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
