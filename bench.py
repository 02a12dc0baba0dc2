"""Benchmark: multi-source SSSP path-table rows on MI355X (BASELINE.json metric
"SSSP sources/sec + full path-table time, % HBM roofline, at 1/2/4/8 GPU").

Workload (default, config C3 of BASELINE.json / SURVEY.md §8d): synthetic
Barabasi-Albert n=50,000, m=3, seed 3, latency U(1,100) ms, loss U(0,0.01),
every vertex attached (A = 50,000 sources x 50,000 targets; slots in the
engine's clustered order, spe_order_sources).  A step = one WHOLE path table:
every source row (latency, reliability, next hop, hops) written into the
HBM-resident table.  With N GPUs (one rank each) the sources are dealt
round-robin in chunks of one build launch and the latency/reliability records
of every chunk are all-gathered over RCCL, overlapped with the next chunk's
build, so each step ends with the whole table replicated on every GPU (strong
scaling: fixed work per step).  Rank 0 prints one JSON line.

Run: python bench.py [--gpus N --steps K --warmup W]
     torchrun --nproc-per-node N bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import math
import os
import platform
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "SSSP sources/sec + full path-table time, % HBM roofline, at 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
# FP64 vector: 78.6 TFLOP/s counts an FMA as two flops; an add or a min is one
# instruction, so (min, +) work issues at most 39.3 T single-op instructions/s
FP64_OP_PEAK_TOPS = 39.3


def workload(name: str):
    from shadow_amd import graphs
    if name == "c3":
        top = graphs.gen_ba(50000, 3, 3)
        att = np.arange(top.n, dtype=np.int32)
        desc = "C3: Barabasi-Albert n=50000 m=3 seed=3, latency U(1,100), A=50000 (all vertices)"
    elif name == "c4":
        top = graphs.gen_tiered()
        att = graphs.tiered_attached(top)
        desc = "C4: tiered BA core 20k + 180k stubs, A=100000 stubs"
    elif name in ("c1", "c1all"):
        # the reference's shipped topology (resource/topology.graphml.xml.xz, 183 vertices,
        # complete => DIRECT regime), committed as data in tests/golden.  c1: the examples
        # config's 150 un-hinted hosts attached through Shadow's seed chain;
        # c1all: every vertex attached
        from shadow_amd import shadow_random as sr
        z = np.load(os.path.join(ROOT, "tests", "golden", "shipped_topology.npz"))
        top = graphs.Topology(n=int(z["n"]), esrc=z["esrc"], edst=z["edst"], elat=z["elat"], eloss=z["eloss"],
                              vloss=z["vloss"], directed=bool(z["directed"]), prefer_direct=bool(z["prefer_direct"]))
        if name == "c1all":
            att = np.arange(top.n, dtype=np.int32)
            desc = "C1: shipped resource/topology.graphml.xml.xz (183 V, complete: DIRECT), all 183 vertices attached"
        else:
            hosts = sr.host_streams([("server", 50), ("webclient", 50), ("bulkclient", 50)], seed=1)
            verts = [sr.unhinted_vertex(h, top.n) for _, h in hosts]
            att = np.array(list(dict.fromkeys(verts)), dtype=np.int32)   # slots in first-attach order
            desc = (f"C1: shipped resource/topology.graphml.xml.xz (183 V, complete: DIRECT) with the examples "
                    f"config's 150 hosts (seed chain 1): {att.shape[0]} attached vertices")
    elif name == "c2":
        top = graphs.gen_rgg(10000, 2)
        att = np.arange(top.n, dtype=np.int32)
        desc = "C2: random geometric graph n=10000 seed=2, A=all"
    else:
        raise SystemExit(f"unknown config {name}")
    return top, att, desc


def host_cores():
    """The host cores this job may use: its affinity mask (on the GPU box the whole
    machine, 256 threads) within the cgroup CPU quota (16 CPUs there) -- the
    all-cores CPU legs run one thread per usable core and state the machine's count,
    the quota and the threads used (256 threads on a 16-CPU quota ran 4-5x slower
    than 16: time-slicing, measured r05)."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = round(float(q) / float(per), 2)
    except (OSError, ValueError):
        pass
    return (min(n, max(1, math.ceil(quota))) if quota else n), quota


def cpu_baseline(top, att, seconds: float, sources: int = 0, seed: int = 6):
    """Oracle (C restatement of igraph Dijkstra + Shadow row rules, -O2) timed on a
    sample of this workload's sources: 1 core (the reference serialises its
    Dijkstra runs under graphLock, shd-topology.c:1732-1766), then all cores
    (OpenMP over sources: a bound the reference cannot reach).  The 1-core leg
    times exactly `sources` seeded-random sources when given (BASELINE.md plans
    1,000 for C3 and C4), else as many as fit `seconds`; sources cycle when the
    sample outlasts A (C1)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle import Oracle
    o = Oracle(top)
    A = att.shape[0]
    order = np.random.default_rng(seed).permutation(A)

    def take(start, k):
        return att[order[np.arange(start, start + k) % A]]

    done, t0, dj = 0, time.perf_counter(), 0.0
    while (done < sources) if sources > 0 else (time.perf_counter() - t0 < seconds):
        k = min(8, sources - done) if sources > 0 else 8
        r = o.rows(take(done, k), att, nthreads=1, want_dijkstra_time=True)
        dj += r["dijkstra_seconds"]
        done += k
    el = time.perf_counter() - t0
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    nt, quota = host_cores()
    done_all, t1 = 0, time.perf_counter()
    while time.perf_counter() - t1 < seconds / 4:
        o.rows(take(done + done_all, 2 * nt), att, nthreads=nt)
        done_all += 2 * nt
    el_all = time.perf_counter() - t1
    dij = (f"Dijkstra-only {done / dj:.1f} sources/s" if dj > 0
           else "no Dijkstra runs: every pair is DIRECT (complete graph, shd-topology.c:2002-2008)")
    return {"value": round(done / el, 1), "unit": "sources/s", "cores": 1, "kind": "port",
            "sample": f"{done} seeded-random source rows (seed {seed}, cycling over A = {A}) x {A} targets, full "
                      f"row build, {el:.1f} s; {dij}",
            "optimistic_all_cores": {"value": round(done_all / el_all, 1), "threads": nt,
                                     "cgroup_cpu_quota": quota, "host_nproc": os.cpu_count(),
                                     "sample": f"{done_all} source rows, {el_all:.1f} s"},
            "cpu_model": model, "host_nproc": os.cpu_count()}


def pmc_key(config: str, world: int, groups: int, exact: bool = False) -> str:
    """What a PMC summary must have been measured on to be this line's traffic:
    the config, the GPU count and the build shape (groups per launch, exact mode)."""
    return f"{config}|n{world}|g{groups}|{'exact' if exact else 'default'}"


def pmc_traffic(args, kernel, config=None, key=None):
    """HBM bytes per dispatch of `kernel` from a PMC summary (separate rocprofv3
    --pmc passes of this same bench command, tools/pmc_to_json.py), or None.  A
    summary is attached only when it records the same pmc_key as this run (config,
    N, groups per launch, build mode): traffic measured on another shape is not
    this line's traffic."""
    path = args.pmc_json
    if path is None:   # the newest committed summary of this config
        for rnd in ("r06", "r05", "r04", "r03", "r02", "r01"):
            cand = os.path.join(ROOT, "profiles", f"{rnd}_pmc_{config or args.config}.json")
            if os.path.exists(cand):
                path = cand
                break
    if not path:
        return None
    try:
        doc = json.load(open(path))
        if key is not None and doc.get("pmc_key") != key:
            return None
        k = doc["kernels"][kernel]
        if kernel == "k_lookup":   # random 16-B reads: FETCH_SIZE is 64 B per location (profiles/r06_line_fetch.json)
            fetch = k["fetch_bytes_raw_per_dispatch"]
            return {"hbm_bytes_per_launch": round(fetch + k["write_bytes_per_dispatch"]),
                    "fetch_bytes_per_launch": round(fetch), "write_bytes_per_launch": round(k["write_bytes_per_dispatch"]),
                    "fetch_basis": "FETCH_SIZE raw: the streaming-read x2 does not apply to random 16-B reads "
                                   "(tools/probe_line_fetch.hip)",
                    "source": os.path.relpath(path, ROOT), "pmc_key": doc.get("pmc_key")}
        return {"hbm_bytes_per_launch": round(k["hbm_bytes_per_dispatch"]),
                "fetch_bytes_per_launch": round(k["fetch_bytes_per_dispatch"]),
                "write_bytes_per_launch": round(k["write_bytes_per_dispatch"]),
                "source": os.path.relpath(path, ROOT), "pmc_key": doc.get("pmc_key")}
    except (KeyError, OSError, ValueError):
        return None


def bench_lookup(args, rank=0, world=1, local=0, dist=None):
    """C5: batched per-packet lookups (s_slot, t_slot) -> (latency, reliability, ok)
    against the HBM-resident C3 table; 41 algorithmic bytes per query.  N > 1:
    replicas (the table is replicated after the all-gather; queries
    split with no communication) -- every rank holds the whole table and answers
    its own 100M queries per step (weak scaling)."""
    import torch
    from shadow_amd import spe
    dev = torch.device("cuda", local)
    if world > 1:
        # the replicated table the N > 1 table build leaves on every GPU (sharded +
        # all-gathered records, the remainder recomputed): each rank's lookups read
        # its own replica
        rep = bench_table(args, rank, world, local, dist, config=args.c5_table, replica_only=True)
        g, att, desc = rep["graph"], rep["attached"], rep["desc"]
        lr = rep["lr"]
        t = spe.PathTable(g, att, blocks=(0, rep["nblk"]), ext=[lr.data_ptr(), lr.data_ptr(), lr.data_ptr()],
                          ext_filled=True)
    else:
        top, att, desc = workload(args.c5_table)
        g = spe.Graph(top, device=local)
        if args.c5_table != "c3":
            att = g.order_sources(att)
        t = spe.PathTable(g, att)
        t.build()
    q = args.queries
    gen = torch.Generator(device=dev).manual_seed(5 + rank)
    pairs = torch.randint(0, t.A, (q, 2), dtype=torch.int32, device=dev, generator=gen)
    lat = torch.empty(q, dtype=torch.float64, device=dev)
    rel = torch.empty(q, dtype=torch.float64, device=dev)
    ok = torch.empty(q, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    steps = args.steps if args.steps > 0 else 10
    for _ in range(args.warmup):
        t.lookup_batch(pairs.data_ptr(), q, lat.data_ptr(), rel.data_ptr(), ok.data_ptr(), stream)
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    for _ in range(steps):
        t.lookup_batch(pairs.data_ptr(), q, lat.data_ptr(), rel.data_ptr(), ok.data_ptr(), stream)
    ev1.record()
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    el = time.perf_counter() - t0
    kern_s = ev0.elapsed_time(ev1) / 1e3 / steps
    assert bool(ok.all().item())
    if dist is not None:
        x = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(x, op=dist.ReduceOp.MAX)
        el = float(x.item())
    if rank != 0:
        return
    c5name = "c5" if args.c5_table == "c3" else "c5_on_c4"
    value = world * q * steps / el
    ach = 41.0 * q / kern_s / 1e9
    cpu = None
    if not args.no_cpu_baseline and world == 1:
        cpu = cpu_lookup_baseline(t.A, args.cpu_seconds)
    line = {"metric": "per-packet lookup queries/s against the GPU-resident path table (config C5)",
            "value": round(value, 1), "unit": "queries/s", "n_gpus": world, "steps": steps, "warmup": args.warmup,
            "ms_per_step": round(1e3 * el / steps, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f64", "data": "synthetic",
            "config": {"workload": f"C5: {q} uniform (s,t) slot pairs per GPU (seed 5 + rank) on the {desc} table",
                       "parallelism": f"{world} replica(s) of the table, each GPU answering its own queries (no communication)"},
            "roofline": {"bound": "hbm", "kernel": "k_lookup", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": pmc_traffic(args, "k_lookup", c5name, pmc_key(c5name, world, 0)),
                         "algorithmic_bytes_per_query": 41,
                         # a uniform query reads one 16-B record at a random location: what bounds it is
                         # the rate of random accesses, measured with the same access alone
                         # (tools/probe_line_fetch.hip, profiles/r06_line_fetch.json): 37.2 G random 16-B
                         # reads/s with an 8-B store each (64-B reads 38.6 G/s, whole 128-B lines 33.8 G/s;
                         # FETCH_SIZE reads 64 B per location for all three, so the streaming x2 does not
                         # apply to this access)
                         "random_access_bound": {"measured_random_16B_reads_per_s": RANDOM_16B_READS_PER_S,
                                                 "source": "profiles/r06_line_fetch.json",
                                                 "frac": round(value / world / RANDOM_16B_READS_PER_S, 4)}},
            "cpu_baseline": cpu, "pmc_key": pmc_key(c5name, world, 0)}
    if cpu:
        line["speedup_vs_cpu_1core"] = round(value / cpu["value"], 1)
    print(json.dumps(line), flush=True)


def cpu_lookup_baseline(A: int, seconds: float, seed: int = 5):
    """The reference's per-packet lookup restated on the host (oracle.c orc_cache:
    IP -> slot hash, then the two-level src -> dst path cache of
    _topology_getPathEntry, shd-topology.c:1952-2075), 1 core, on a bounded
    sample: a cache of 4M uniform pairs of this table, queried for those pairs."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle import LookupCache
    rng = np.random.default_rng(seed)
    npairs = 4_000_000
    pairs = rng.integers(0, A, size=(npairs, 2)).astype(np.int32)
    ips = (0x0A000000 + np.arange(A)).astype(np.uint32)
    c = LookupCache(ips, pairs, rng.uniform(1, 100, npairs), rng.uniform(0.9, 1, npairs))
    sip, dip = ips[pairs[:, 0]], ips[pairs[:, 1]]
    done, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds / 2:
        c.lookup(sip, dip, nthreads=1)
        done += npairs
    el = time.perf_counter() - t0
    nt, quota = host_cores()
    c.lookup(sip, dip, nthreads=nt)   # threads started
    reps, t1 = 0, time.perf_counter()
    while reps < 2 or time.perf_counter() - t1 < seconds / 4:
        c.lookup(sip, dip, nthreads=nt)
        reps += 1
    el_all = time.perf_counter() - t1
    return {"value": round(done / el, 1), "unit": "queries/s", "cores": 1, "kind": "port",
            "sample": f"{done} lookups over a 4M-pair cache (seed {seed}): 2 IP->slot probes + src and (src,dst) "
                      f"cache probes per query, {el:.1f} s",
            "optimistic_all_cores": {"value": round(reps * npairs / el_all, 1), "threads": nt,
                                     "cgroup_cpu_quota": quota, "host_nproc": os.cpu_count()}}


def bench_complete(args):
    """Offline topology completion (compute-topology-paths.py): all
    ordered POI pairs of a 200k-vertex tiered topology (the C4 generator, edge
    jitter U(0, 5)), POIs = the first --pois stub vertices (the reference samples
    CLIENT_SAMPLE_SIZE = 10,000 clients).  Timed: complete_paths end to end (GPU
    rows + the P x P host copy of latency / jitter / hops).  CPU leg: the
    reference tool's per-source worker restated with networkx (its own
    dependency), one core, bounded sample of sources."""
    from shadow_amd import complete, graphs, spe
    top = graphs.gen_tiered()
    rng = np.random.default_rng(7)
    jit = rng.uniform(0.0, 5.0, top.m)
    pois = np.arange(20000, 20000 + args.pois, dtype=np.int32)
    complete.complete_paths(top, pois[:256], jit)   # warm-up (code objects)
    t0 = time.perf_counter()
    r = complete.complete_paths(top, pois, jit)
    el = time.perf_counter() - t0
    assert not np.isnan(r["lat"]).any()
    cpu = None
    if not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import topology_tools as tt
        G = tt.nx_graph(top, jit)
        done, c0 = 0, time.perf_counter()
        while time.perf_counter() - c0 < args.cpu_seconds and done < len(pois):
            tt.source_rows(G, int(pois[done]), pois)
            done += 1
        cel = time.perf_counter() - c0
        cpu = {"value": round(done / cel, 3), "unit": "POI sources/s", "cores": 1, "kind": "port",
               "sample": f"{done} POI sources x {len(pois)} targets: networkx single_source_dijkstra_path + "
                         f"per-target latency sum / jitter mean (compute-topology-paths.py:15-38), {cel:.1f} s"}
    line = {"metric": "topology completion (compute-topology-paths.py): POI source rows/s", "value":
            round(len(pois) / el, 1), "unit": "POI sources/s", "n_gpus": 1, "higher_is_better": True,
            "dtype": "f64", "data": "synthetic",
            "config": {"workload": f"tiered BA core 20k + 180k stubs (C4 graph), {len(pois)} POIs, jitter U(0,5)",
                       "pairs": len(pois) ** 2},
            "seconds": round(el, 3), "cpu_baseline": cpu,
            "speedup_vs_cpu_1core": round(len(pois) / el / cpu["value"], 1) if cpu else None}
    print(json.dumps(line), flush=True)


def bench_shim(args, config: str):
    """bench_shim_in in a scratch directory that is removed whatever happens (the
    GraphML of C4 is ~0.5 GB)."""
    import shutil
    import tempfile
    tmp = tempfile.mkdtemp(prefix="spe-shim-")
    try:
        return bench_shim_in(args, config, tmp)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def bench_shim_in(args, config: str, tmp: str):
    """The drop-in end to end (include/shd_topology_spe.h, libshdtopo): the config's
    topology written once as GraphML (every vertex an "ip"), then what Shadow does
    at start-up -- topology_new (libxml2 ingest + the reference's validation +
    spe_graph_create), topology_attach of every host by exact IP hint, topology_seal
    (slot order + the whole path table + the host mirror) -- each phase timed
    (shd-topology.c:2469-2490 / 2354-2413 / the first query's row runs).  Then C5
    through the drop-in: rounds of uniform (src, dst) host-address pairs answered by
    topology_getPathInfoBatch (per query the reference's path-cache bookkeeping on
    the host, the table read in one device launch), against the reference's
    per-packet lookup restated on one core."""
    from shadow_amd import graphs
    from shadow_amd import topology as T
    top_g, att, desc = workload(config)
    ips = [f"10.{(v >> 16) & 255}.{(v >> 8) & 255}.{v & 255}" for v in range(top_g.n)]
    path = os.path.join(tmp, "topology.graphml")
    t0 = time.perf_counter()
    graphs.write_graphml(top_g, path, ips=ips)
    write_s = time.perf_counter() - t0
    t0 = time.perf_counter()
    top = T.Topology(path)
    new_s = time.perf_counter() - t0
    print(f"[shim] graphml {write_s:.1f} s, topology_new {new_s:.1f} s", file=sys.stderr, flush=True)
    A = int(att.shape[0])
    hosts = np.array([T.ip(f"11.{(i >> 16) & 255}.{(i >> 8) & 255}.{i & 255}") for i in range(A)], np.uint32)
    t0 = time.perf_counter()
    for i in range(A):
        top.attach(int(hosts[i]), ip_hint=ips[int(att[i])])
    attach_s = time.perf_counter() - t0
    print(f"[shim] attach {A} hosts {attach_s:.1f} s", file=sys.stderr, flush=True)
    t0 = time.perf_counter()
    rc = top.seal()
    t_sealed = time.perf_counter()
    seal_s = t_sealed - t0
    print(f"[shim] seal {seal_s:.1f} s", file=sys.stderr, flush=True)
    assert rc == 0, f"topology_seal failed ({rc})"
    q = min(args.queries, 20_000_000)
    rng = np.random.default_rng(5)
    pi = rng.integers(0, A, (q, 2))
    src, dst = hosts[pi[:, 0]], hosts[pi[:, 1]]
    # the answer buffers a worker reuses every round (allocated and touched untimed)
    out = (np.zeros(q, np.uint8), np.zeros(q, np.float64), np.zeros(q, np.float64))
    # untimed warm-up rounds of the same batch: code objects, staging, and the path
    # cache's first stores (the first round of a simulation stores every pair it
    # meets; reported as first_batch_s)
    warm_s = []
    for _ in range(max(1, args.warmup)):
        t0 = time.perf_counter()
        top.path_info_batch(src, dst, out=out)
        warm_s.append(round(time.perf_counter() - t0, 4))
        print(f"[shim] warm-up batch of {q} queries {warm_s[-1]:.3f} s", file=sys.stderr, flush=True)
    steps = args.steps if args.steps > 0 else 3
    t0 = time.perf_counter()
    call_s = []
    for _ in range(steps):
        tc = time.perf_counter()
        ok, lat, rel = top.path_info_batch(src, dst, out=out)
        call_s.append(round(time.perf_counter() - tc, 4))
    el = time.perf_counter() - t0
    print(f"[shim] {steps} batches of {q} queries {el:.1f} s", file=sys.stderr, flush=True)
    assert ok.all(), "every pair of the synthetic topologies is routable"
    # the same pairs one call at a time (topology_getPathInfo), a bounded sample: on C3
    # the whole table is mirrored on the host at seal; on C4 (160 GB of records) a single
    # call outside the mirror reads its 16-B record from HBM, and a source row read
    # repeatedly is mirrored on its third read (uniform pairs: almost every call is a
    # record read)
    # first right after the batches (cold: on C4 the library is still faulting the
    # table's host mapping in), then once that is done (~9.4 s after seal on
    # C4): what a simulation's packets see for the rest of the run
    ns_cold = 50_000
    t1 = time.perf_counter()
    for i in range(ns_cold):
        top.path_info(int(src[-1 - i]), int(dst[-1 - i]))
    cold_rate = ns_cold / (time.perf_counter() - t1)
    settle = 12.0 if A * A * 22 > 50e9 else 0.0
    wait = max(0.0, t_sealed + settle - time.perf_counter())
    if wait > 0:
        time.sleep(wait)
    ns = 200_000
    t1 = time.perf_counter()
    for i in range(ns):
        top.path_info(int(src[i]), int(dst[i]))
    single_s = time.perf_counter() - t1
    print(f"[shim] {ns_cold} cold single calls {ns_cold / cold_rate:.1f} s, then {ns} single calls {single_s:.1f} s "
          f"({settle:.0f} s after seal)", file=sys.stderr, flush=True)
    top.close()
    # the same single calls from C (examples/shd_topology_single_calls.c: no Python in the
    # loop), one worker thread and the job's CPU quota of threads, on its own topology_new /
    # attach / seal of the same file (Shadow's workers call from C, concurrently)
    c_single = None
    exe = os.path.join(ROOT, "shadow_amd", "shd_topology_single_calls")
    if os.path.exists(exe):
        hints = os.path.join(tmp, "hints.txt")
        with open(hints, "w") as f:
            f.write("\n".join(ips[int(v)] for v in att) + "\n")
        nt, _ = host_cores()
        # then again once the library's background pre-fault of the table's host mapping
        # is done (~1 s per 25 GB of records)
        settle = 12 if A * A * 22 > 50e9 else 3
        try:
            r = subprocess.run([exe, path, hints, str(ns), str(nt), "5", str(settle)], capture_output=True, text=True,
                               timeout=240)
            c_single = json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else \
                {"error": f"exit status {r.returncode}", "tail": (r.stdout + r.stderr)[-300:]}
        except (subprocess.TimeoutExpired, ValueError, IndexError) as e:
            c_single = {"error": str(e)[:200]}
        print(f"[shim] C single calls: {c_single}", file=sys.stderr, flush=True)
    value = q * steps / el
    cpu = None if args.no_cpu_baseline else cpu_lookup_baseline(A, args.cpu_seconds)
    line = {"metric": "per-packet lookups through the drop-in (topology_getPathInfoBatch), queries/s",
            "value": round(value, 1), "unit": "queries/s", "n_gpus": 1, "steps": steps,
            "ms_per_step": round(1e3 * el / steps, 3), "higher_is_better": True, "dtype": "f64", "data": "synthetic",
            "config": {"workload": f"{q} uniform (src, dst) host-address pairs per step over the {desc} table, "
                                   f"{A} hosts attached by exact IP hint"},
            "startup_s": {"graphml_write_untimed": round(write_s, 3), "topology_new": round(new_s, 3),
                          "attach_all_hosts": round(attach_s, 3), "seal_table_and_mirror": round(seal_s, 3),
                          "end_to_end": round(new_s + attach_s + seal_s, 3)},
            "single_call_queries_per_s": round(ns / single_s, 1),
            "single_call_queries_per_s_cold": round(cold_rate, 1),
            "single_call_queries_per_s_c": c_single, "batch_call_s": call_s,
            "first_batch_s": warm_s[0], "warmup": len(warm_s),
            "single_call_note": (f"{ns} topology_getPathInfo calls through ctypes (Python call overhead included), "
                                 f"from {settle:.0f} s after seal (C4: once the library's background pre-fault of the "
                                 f"table's host mapping is done); _cold: {ns_cold} calls right after the batches; "
                                 "single_call_queries_per_s_c: the same calls from C on a fresh topology_new / attach "
                                 "/ seal of the same file, one thread and the job's CPU quota of threads (its seal_s "
                                 "includes the driver clearing the VRAM this process just freed), then both again "
                                 "settle_s later (settled_*), when the table's host mapping is faulted in"),
            "cpu_baseline": cpu}
    if cpu:
        line["speedup_vs_cpu_1core"] = round(value / cpu["value"], 1)
    print(json.dumps(line), flush=True)


def bench_fw(args):
    """C2 on the FW engine (SPE_ENGINE_FW): the north star's dense algorithm -- a
    blocked min-plus Floyd-Warshall closure carrying (latency, reliability, first
    edge), then every row re-folded in path order along the first-edge walk --
    timed for the WHOLE bit-exact table (closure + walks + rows, a fresh table per
    step: the closure is not reused), beside the distance-only closure
    (spe_fw_apsp) and the LDS SSSP engine AUTO picks for this graph."""
    import torch
    from shadow_amd import spe
    top, att, desc = workload("c2")
    g = spe.Graph(top, device=0)
    n = g.info()["n_relax_vertices"]
    ld = (n + 63) // 64 * 64
    nb = ld // 64
    relax = float(nb) ** 3 * 64 ** 3
    steps = max(1, args.steps or 2)

    def fw_table():
        t = spe.PathTable(g, att, engine=spe.SPE_ENGINE_FW)
        t.profile(True)
        t0 = time.perf_counter()
        t.build()
        el = time.perf_counter() - t0
        kp = t.kernel_profile()
        t.close()
        return el, kp

    fw_table()   # warm-up (code objects)
    runs = [fw_table() for _ in range(steps)]
    el, kp = min(runs, key=lambda r: r[0])
    fw_ms = kp["fw"]["ms"]
    D = torch.empty(ld * ld, dtype=torch.float64, device="cuda")
    g.fw_apsp(D.data_ptr(), ld)
    dist_only = min(g.fw_apsp(D.data_ptr(), ld) for _ in range(2))
    R = torch.empty(ld * ld, dtype=torch.float64, device="cuda")
    NX = torch.empty(ld * ld, dtype=torch.int32, device="cuda")
    closure = min(g.fw_closure(D.data_ptr(), R.data_ptr(), NX.data_ptr(), ld) for _ in range(2))
    # the (latency, first hop) pair the table build runs (its rows re-fold reliability in path order)
    closure_pair = min(g.fw_closure(D.data_ptr(), 0, NX.data_ptr(), ld) for _ in range(2))
    del D, R, NX
    tl = spe.PathTable(g, att, engine=spe.SPE_ENGINE_LDS)
    tl.build()
    t0 = time.perf_counter()
    tl.build()
    lds_s = time.perf_counter() - t0
    tl.close()
    A = int(att.shape[0])
    line = {"metric": "C2 whole path table by the FW engine (blocked min-plus Floyd-Warshall carrying the "
                      "latency/reliability/next-hop triple, rows re-folded in path order)",
            "value": round(A / el, 1), "unit": "sources/s", "higher_is_better": True, "n_gpus": 1, "steps": steps,
            "dtype": "f64", "data": "synthetic", "full_table_time_s": round(el, 4),
            "config": {"workload": desc, "n_relax": n, "ld": ld, "attached": A},
            "roofline": {"bound": "fp64-valu", "kernel": "k_fw3_rest<false> (the table build's closure: latency + first hop)",
                         "achieved": round(2 * relax / closure_pair / 1e12, 2), "peak": FP64_OP_PEAK_TOPS,
                         "unit": "Tops/s", "frac": round(2 * relax / closure_pair / 1e12 / FP64_OP_PEAK_TOPS, 4),
                         "note": "2 FP64 vector instructions (v_add_f64, v_min_f64) per (min,+) relaxation, ld^3 "
                                 "relaxations, against the FP64 vector instruction peak: 78.6 TFLOP/s counts an FMA "
                                 "as 2 flops, so single-op instructions issue at 39.3 T/s; carrying N adds a select "
                                 "per relaxation, R a multiply and a select more (not counted)",
                         "triple_frac": round(2 * relax / closure / 1e12 / FP64_OP_PEAK_TOPS, 4),
                         "distance_only_frac": round(2 * relax / dist_only / 1e12 / FP64_OP_PEAK_TOPS, 4),
                         "traffic": pmc_traffic(args, "k_fw3_rest", "c2fw", pmc_key("c2fw", 1, 0))},
            "closure_triple_s": round(closure, 4), "closure_pair_s": round(closure_pair, 4),
            "closure_distance_only_s": round(dist_only, 4),
            "fw_kernels_ms_in_table_build": round(fw_ms, 2), "rows_ms": round(kp["rows"]["ms"], 2),
            "lds_engine_table_s": round(lds_s, 4),
            "all_runs_s": [round(r[0], 4) for r in runs], "pmc_key": pmc_key("c2fw", 1, 0)}
    print(json.dumps(line), flush=True)


def relax_bytes(info, A, lds: bool, direct: bool):
    """SURVEY §8d algorithmic bytes per source, priced on the graph the engine
    relaxes (pendants pruned: n_relax_vertices / n_relax_entries) -- the relaxation
    stage B_relax = 12 m + 28 n + 8, the row stage 22 A; the LDS engine's one
    fused kernel does both; a DIRECT (complete) row is 38 B per pair."""
    n, m = info["n_relax_vertices"], info["n_relax_entries"]
    b_relax = 12.0 * m + 28.0 * n + 8.0
    b_rows = 22.0 * A
    if lds:
        b_relax += b_rows
    if direct:
        b_relax = 38.0 * A
    return b_relax, b_rows


def auto_groups(info, nblk: int, A: int, world: int, dev, span_blocks: int = 0) -> int:
    """spe_table_create's default groups per launch (spe.hip): ~10M (group,
    vertex) rows per relaxation round, within the free HBM next to the table
    (state held twice for the rows / relaxation overlap, 4 GB kept free).  At
    N > 1 the chunk is also cut so that every rank runs >= 4 rounds: a round's
    all-gather then overlaps the next round's build, and rounded up to an even
    count (spe_table_create picks 64-source rows for an odd count below 32)."""
    import torch
    n = max(1, info["n_relax_vertices"])
    per_group = 2.0 * (n * 64 * 28.0 + 4.0 * n + 2.0 * info["n_relax_entries"])
    free_b, _ = torch.cuda.mem_get_info(dev)
    table_b = float(span_blocks or nblk) * A * 64 * 22.0
    cap = max(1.0, (free_b - table_b - 4.0e9) / per_group)
    want = max(1.0, min(round(1.0e7 / n), cap))
    if world > 1:
        want = min(want, math.ceil(nblk / (world * 4)))
        if want > 1 and int(want) % 2:
            want = int(want) + 1   # even: the table keeps 128-source rows, e.g. C3 at N = 8: 25 -> 26
    return int(max(1, want))


def calibrate_split(t, lr, blk_elems, nblk, world, rank, dev, dist, span_blocks):
    """N > 1: the inputs of dist.shared_fraction, measured untimed on this job --
    the one-GPU whole-table build time T1 (from a build of this rank's share of a
    pure-sharding schedule, scaled by N) and the all-gather bandwidth B (one
    in-place gather of up to 2 GB per rank) -- agreed over the ranks (max T1,
    min B) so every rank takes the same schedule.  B is measured for both
    gathers, RCCL's all_gather_into_tensor and world - 1 concurrent peer
    exchanges (dist.allgather_span_p2p: every xGMI link at once), and the faster
    one gathers the table (returned as `mode`)."""
    import torch
    share = max(1, nblk // world)
    b0 = min(nblk - 1, rank * share)
    b1 = min(nblk, b0 + share)
    nx = torch.empty((b1 - b0) * blk_elems, dtype=torch.int32, device=dev)
    hp = torch.empty((b1 - b0) * blk_elems, dtype=torch.int16, device=dev)
    t1 = 0.0
    for _ in range(2):   # the second build is timed (the first loads code objects)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        t.build_blocks_into(b0, b1, lr[b0 * blk_elems:].data_ptr(), nx.data_ptr(), hp.data_ptr())
        t1 = (time.perf_counter() - t0) * nblk / max(1, b1 - b0)
    del nx, hp
    from shadow_amd import dist as sd
    per = max(1, min(span_blocks // world, int(2e9 // (blk_elems * 16))))
    recv = (world - 1) * per * blk_elems * 16.0
    rates = []
    # (gloo -- the one-GPU rehearsal -- sends CPU tensors only: the collective alone)
    fns = (sd.allgather_span, sd.allgather_span_p2p) if dist.get_backend() == "nccl" else (sd.allgather_span,)
    for fn in fns:
        fn(lr, 0, per, world, rank, blk_elems, dist)   # warm the communicator / peer connections
        torch.cuda.synchronize(dev)
        dist.barrier()
        t0 = time.perf_counter()
        fn(lr, 0, per, world, rank, blk_elems, dist)
        torch.cuda.synchronize(dev)
        rates.append(-recv / max(time.perf_counter() - t0, 1e-9))
    x = torch.tensor([t1] + rates + [0.0] * (2 - len(rates)), dtype=torch.float64, device=dev)
    dist.all_reduce(x, op=dist.ReduceOp.MAX)
    coll, p2p = float(-x[1].item()), float(-x[2].item())
    mode = "p2p" if p2p > coll else "all_gather"
    return float(x[0].item()), max(coll, p2p), mode, {"all_gather": round(coll / 1e9, 1), "p2p": round(p2p / 1e9, 1)}


def bench_table(args, rank, world, local, dist, config=None, replica_only=False):
    """The default measurement: a step is one WHOLE path table (every source
    row) of the config -- BASELINE's "full path-table time".  At N > 1 (one rank
    per GPU, torchrun) the table is replicated on every GPU at the end of a step,
    and the work is split between sharing and recomputing (DESIGN §6,
    dist.shared_fraction): the first S source blocks are dealt round-robin in
    chunks of one build launch, every chunk's {latency, reliability} records
    all-gathered over RCCL in place (overlapped with the next build), and the
    remaining blocks are built by every rank itself while the gathers run.  Next
    hops / hop counts stay with the rank that built them (its own chunks and the
    local remainder, packed).  The step ends when every rank holds the whole record
    span (strong scaling: the total work per step is fixed)."""
    import torch
    from shadow_amd import spe
    config = config or args.config
    top, att, desc = workload(config)
    t_prep = time.perf_counter()
    g = spe.Graph(top, device=local)   # validation, pendant pruning, degree-3 contraction, heavy plan, upload
    t_prep = time.perf_counter() - t_prep
    t_ord = time.perf_counter()
    att = g.order_sources(att)   # slot numbering is the caller's: clustered sources (host side)
    t_ord = time.perf_counter() - t_ord
    info = g.info()
    A = int(att.shape[0])
    nblk = (A + 63) // 64
    dev = torch.device("cuda", local)
    probe = spe.PathTable(g, att[:64], engine=args.engine)   # the engine AUTO picks for this graph
    lds_engine = probe.layout()["engine"] == spe.SPE_ENGINE_LDS
    probe.close()
    from shadow_amd import dist as sd
    shares = max(world, args.shares)
    emulated = shares != world   # one rank of a `shares`-GPU job: its chunks only, no gather
    gather = world > 1 and not args.no_gather
    # one chunk = one build launch: the LDS engine covers every block in one launch,
    # the batch engine `groups` blocks (auto rule above)
    # (one GPU: the library's own rule, spe_table_create -- shared tables size the batch by their roots)
    gpl = (nblk if lds_engine else args.groups if args.groups > 0 else
           0 if world == 1 and not emulated else auto_groups(info, nblk, A, world, dev))
    blk_elems = A * 64
    pad_blocks = shares * sum(sd.chunk_schedule(nblk, shares, gpl)) if gpl > 0 else nblk   # pure-sharding span
    lr = torch.empty((pad_blocks * blk_elems, 2), dtype=torch.float64, device=dev)
    # the table owns no storage of its own that is ever written: every build goes
    # into the caller's buffers (spe_table_build_blocks_into); lr doubles as its
    # nominal external storage
    # The table's own batch size stays the library's (spe_table_create's rule: a shared
    # table holds every root of a build call in one batch), whatever the chunk size of
    # the gather schedule: a chunk or the local remainder built in batches of `gpl`
    # groups would re-relax the hubs every batch (round 6: the N = 2 rehearsal's local
    # span ran 922 row launches instead of one)
    tgroups = gpl if (lds_engine or args.groups > 0) else 0
    t = spe.PathTable(g, att, blocks=(0, nblk), ext=[lr.data_ptr(), lr.data_ptr(), lr.data_ptr()], groups=tgroups,
                      engine=args.engine, exact_sources=bool(args.exact))
    if gpl == 0:
        gpl = t.layout()["groups_per_launch"]
    calib = None
    gather_fn = sd.allgather_span_p2p if args.gather == "p2p" else sd.allgather_span
    frac = 1.0 if not gather else args.shared_frac
    if gather and frac < 0:   # auto: measure T1 and B on this job, then plan
        print(f"[bench] rank {rank}: calibrating the split", file=sys.stderr, flush=True)
        calib = calibrate_split(t, lr, blk_elems, nblk, world, rank, dev, dist, pad_blocks)
        print(f"[bench] rank {rank}: T1 {calib[0]:.3f} s, gather GB/s {calib[3]}", file=sys.stderr, flush=True)
        frac = sd.shared_fraction(world, calib[0], nblk * blk_elems * 16.0, calib[1])
        if args.gather == "auto":
            gather_fn = sd.allgather_span_p2p if calib[2] == "p2p" else sd.allgather_span
    # one GPU with shared anchor trees: the whole table is one build call,
    # so the library batches by anchor roots (its state holds `gpl` blocks of roots)
    sched_gpl = nblk if (world == 1 and not emulated and t.layout()["shared_sources"]) else gpl
    sizes, S = sd.split_schedule(nblk, shares, sched_gpl, max(0.0, frac) if gather else 1.0)
    slots, nslot = sd.rank_next_hop_slots(nblk, shares, args.share_index if emulated else rank, sizes, S)
    # next hop (i32) and hop count (u16) of this rank's own blocks only, packed
    nx = torch.empty(max(1, nslot) * blk_elems, dtype=torch.int32, device=dev)
    hp = torch.empty(max(1, nslot) * blk_elems, dtype=torch.int16, device=dev)
    nx_base, hp_base = nx.data_ptr(), hp.data_ptr()
    mine = sd.rank_chunks_sched(nblk, shares, args.share_index if emulated else rank, sizes)
    l0, l1 = sd.local_span(nblk, S)
    slot_of = {(b0, b1): s0 for b0, b1, s0 in slots}

    def into(b0, b1):
        s0 = slot_of[(b0, b1)]
        return t.build_blocks_into(b0, b1, lr[b0 * blk_elems:].data_ptr(), nx_base + s0 * blk_elems * 4,
                                   hp_base + s0 * blk_elems * 2)

    lanes_run = [0]   # relaxation lanes (sources, or shared anchor roots) of this rank's builds
    derived_run = [0, 0]   # derived sources (no lane) and fallback blocks of this rank's builds

    def one_table():
        works, tb, tg, its = [], 0.0, 0.0, 0
        for k, off, gk, b0, b1 in mine:
            t0 = time.perf_counter()
            if b1 > b0:
                st = into(b0, b1)
                its += st["iterations"]
                lanes_run[0] += st["relaxed_lanes"]
                derived_run[0] += st["derived_sources"]
                derived_run[1] += st["fallback_blocks"]
            tb += time.perf_counter() - t0
            if gather:   # overlaps the next round's build and the local part (RCCL runs on its own stream)
                w = gather_fn(lr, off, gk, world, rank, blk_elems, dist, async_op=True)
                if w is not None:
                    works.append(w)
        if l1 > l0 and not emulated:   # built by every rank itself: no exchange
            t0 = time.perf_counter()
            st = into(l0, l1)
            its += st["iterations"]
            lanes_run[0] += st["relaxed_lanes"]
            derived_run[0] += st["derived_sources"]
            derived_run[1] += st["fallback_blocks"]
            tb += time.perf_counter() - t0
        t1 = time.perf_counter()
        for w in works:
            w.wait()
        torch.cuda.synchronize(dev)
        tg += time.perf_counter() - t1
        return tb, tg, its

    if replica_only:   # C5 at N > 1: one build of the replicated records, then lookups read them
        one_table()
        return {"graph": g, "attached": att, "lr": lr, "desc": desc, "table": t, "nblk": nblk}

    def barrier():
        if dist is not None:
            dist.barrier()

    for _ in range(args.warmup):
        one_table()
        print(f"[bench] rank {rank}: warm-up table done", file=sys.stderr, flush=True)
    if not args.no_profile:
        t.profile(True)
    steps = args.steps if args.steps > 0 else 3
    torch.cuda.synchronize(dev)
    barrier()
    lanes_run[0] = 0
    derived_run[0] = derived_run[1] = 0
    t0 = time.perf_counter()
    tb_sum = tg_sum = 0.0
    it_total = 0
    step_s = []
    for _ in range(steps):
        ts = time.perf_counter()
        tb, tg, its = one_table()
        step_s.append(time.perf_counter() - ts)
        tb_sum += tb
        tg_sum += tg
        it_total += its
    torch.cuda.synchronize(dev)
    barrier()
    el = time.perf_counter() - t0
    kp = t.kernel_profile() if not args.no_profile else None
    per_rank = None
    if dist is not None:
        mine_t = torch.tensor([[el, tb_sum / steps, tg_sum / steps]], dtype=torch.float64, device=dev)
        allt = [torch.empty_like(mine_t) for _ in range(world)]
        dist.all_gather(allt, mine_t)
        per_rank = [[round(float(v), 4) for v in a[0, 1:].tolist()] for a in allt]
        x = torch.tensor([el, tb_sum, tg_sum], dtype=torch.float64, device=dev)
        dist.all_reduce(x, op=dist.ReduceOp.MAX)
        el, tb_sum, tg_sum = (float(v) for v in x.tolist())
    built = sum(min(A, b1 * 64) - b0 * 64 for _, _, _, b0, b1 in mine if b1 > b0)
    if not emulated and l1 > l0:
        built += min(A, l1 * 64) - l0 * 64
    total = built if emulated else A
    value = total * steps / el
    lds = kp is not None and kp["lds"]["launches"] > 0
    direct = kp is not None and kp["direct"]["launches"] > 0 and kp["relax"]["launches"] == 0 and not lds
    b_relax, b_rows = relax_bytes(info, A, lds, direct)
    key = pmc_key(config, world, gpl, args.exact)
    roof, extra = None, {}
    if kp is not None:
        # the batch engine's relaxation kernel: k_relax (64 sources per row), k_relax_s
        # (128, LDS-ring neighbour rows) or k_relax_m (128, register-staged)
        lay = t.layout()
        relax_k = ("k_relax" if lay["lanes_per_group"] <= 64 else
                   "k_relax_s" if lay["relax_kernel"] == spe.SPE_RELAX_LDS_RING else "k_relax_m")
        kname = "k_sssp_lds" if lds else ("k_rows_direct" if direct else relax_k)
        rl = kp["lds" if lds else ("direct" if direct else "relax")]
        relax_s = rl["ms"] / 1e3
        done = built * steps   # this rank's sources (the profile is this rank's launches)
        # the relaxation's own units: one lane per source, or per shared anchor root
        #  -- the bytes the kernel is priced on are per relaxed lane
        relaxed = lanes_run[0] if (not lds and not direct and lanes_run[0] > 0) else done
        ach = b_relax * relaxed / relax_s / 1e9 if relax_s > 0 else 0.0
        traffic = pmc_traffic(args, kname, config + ("_exact" if args.exact else ""), key)
        roof = {"bound": "hbm", "kernel": kname + (" (SSSP + rows, LDS-resident state)" if lds else
                                                   (" (DIRECT rows)" if direct else " (SSSP stage)")),
                "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "launches": rl["launches"],
                "launch_avg_us": round(1e3 * rl["ms"] / max(1, rl["launches"]), 2),
                "algorithmic_bytes_per_source": b_relax,
                "relaxed_lanes_per_step": round(relaxed / steps),
                "derived_sources_per_step": round(derived_run[0] / steps),
                "fallback_blocks_per_step": round(derived_run[1] / steps, 2),
                "shared_anchor_trees": bool(lay.get("shared_sources", 0)),
                "lanes_per_group": lay["lanes_per_group"],
                "bytes_basis": ("12 m_relax + 28 n_relax + 8 per relaxed lane (SURVEY 8d B_s minus the row stage), "
                                "m_relax / n_relax of the uncontracted relaxation graph (SURVEY's per-source "
                                "definition; the contracted graph the lanes run on keeps fewer state rows)")}
        if traffic and rl["launches"] > 0 and relax_s > 0:
            # the request view: L2-miss reads (raw FETCH_SIZE / 64 B) per second of the kernel
            # against the rate one MI355X sustains for uniformly random reads
            # (tools/probe_line_fetch.hip): a row visit is ~74 scattered line requests
            rq = traffic["fetch_bytes_per_launch"] / 2 / 64 * rl["launches"] / relax_s
            roof["read_request_rate"] = {"l2_miss_reads_per_s": round(rq / 1e9, 2) * 1e9,
                                         "random_read_ceiling_per_s": RANDOM_16B_READS_PER_S,
                                         "frac": round(rq / RANDOM_16B_READS_PER_S, 3),
                                         "source": "PMC summary (traffic) + profiles/r06_line_fetch.json"}
        rw = kp["rows"]
        rows_s = rw["ms"] / 1e3
        # (SPE_ROWS_LM = 1 in kernels_rows.inc: derived sources go through the lane-major pair)
        rows_k = ("k_stage_lanes + k_rows_lm (+ k_rows_self)" if derived_run[0] > 0 else
                  "k_rows_shared_lds" if lay.get("shared_sources", 0) else "k_rows_sssp")
        extra["roofline_rows"] = {"kernel": rows_k, "achieved": round(b_rows * done / rows_s / 1e9, 1)
                                  if rows_s > 0 else 0.0, "unit": "GB/s", "launches": rw["launches"],
                                  "launch_avg_us": round(1e3 * rw["ms"] / max(1, rw["launches"]), 2),
                                  "algorithmic_bytes_per_source": b_rows}
        extra["kernel_ms"] = {k: round(v["ms"], 3) for k, v in kp.items()}
        extra["kernel_launches"] = {k: v["launches"] for k, v in kp.items()}
        extra["engine"] = "lds" if lds else ("direct" if direct else "batch")
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not emulated:
        cpu = cpu_baseline(top, att, args.cpu_seconds, args.cpu_sources)
    if rank == 0:
        gathered = int((world - 1) * sum(sizes) * blk_elems * 16) if gather else None
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "sources/s", "n_gpus": world, "steps": steps,
            "warmup": args.warmup, "ms_per_step": round(1e3 * el / steps, 3), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
            "config": {"workload": desc, "n": info["n_vertices"], "n_relax": info["n_relax_vertices"],
                       "m_relax": info["n_relax_entries"], "attached": A, "slot_order": "spe_order_sources",
                       "slot_order_ms": round(1e3 * t_ord, 1),
                       "build": ("exact_sources=1: every source on its own relaxation lane, latency / reliability "
                                 "the path-order folds bit for bit (what topology_seal builds on non-dyadic "
                                 "latencies)" if args.exact else
                                 "library default: derived / shared-anchor rows (routes exact, latency / "
                                 "reliability within 8.3e-16 relative of the exact build on C3, 7.5e-16 on C4: "
                                 "c3_exact / c4_exact vs_default_build; tests assert 1e-12)"),
                       "step": "one whole path table (every source row)" + (
                           f"; emulated share {args.share_index} of {shares} (no gather)" if emulated else ""),
                       "chunk_blocks": max(sizes) if sizes else 0, "rounds": len(sizes), "chunk_schedule": sizes,
                       "parallelism": (f"{S if S < nblk else nblk} of {nblk} source blocks in round-robin chunks over "
                                       f"{world} GPUs with an RCCL all-gather of the latency/reliability records per "
                                       f"round (overlapped), blocks [{l0}, {l1}) built by every GPU itself"
                                       if gather else f"{world} GPU(s), no collective")},
            "full_table_time_s": round(el / steps, 4) if not emulated else None,
            # the precompute outside the timed step (once per topology, shd-topology.c:356-384 /
            # :1172-1195): spe_graph_create (validation, pruning, contraction, heavy plan, upload)
            # and the clustered slot order
            "graph_prep_s": round(t_prep, 4), "slot_order_s": round(t_ord, 4),
            "precompute_end_to_end_s": round(t_prep + t_ord + el / steps, 4) if not emulated else None,
            "build_s_per_step": round(tb_sum / steps, 4),
            "gather_wait_s_per_step": round(tg_sum / steps, 4) if gather else None,
            "gather_bytes_per_gpu_per_step": gathered,
            "relax_rounds_per_step": round(it_total / max(1, steps), 1),
            "rank0_step_s": [round(x, 4) for x in step_s],
            "roofline": roof, "cpu_baseline": cpu, "pmc_key": key,
        }
        if gather:
            line["split"] = {"shared_fraction": round(frac, 4), "shared_blocks": min(S, nblk), "local_blocks": l1 - l0,
                             "model": "x* = T1 N / ((N - 1) (S / B + T1)) (DESIGN 6)",
                             "gather": "p2p" if gather_fn is sd.allgather_span_p2p else "all_gather",
                             "calibration": None if calib is None else {"t1_s": round(calib[0], 4),
                                                                        "gather_GBps": round(calib[1] / 1e9, 1),
                                                                        "gather_GBps_by_mode": calib[3]},
                             "per_rank_build_gather_s": per_rank}
        line.update(extra)
        if cpu:
            line["speedup_vs_cpu_1core"] = round(value / cpu["value"], 1)
        return line
    return None


def default_vs_exact(config: str, parts: int = 0):
    """Entry-by-entry differences between the default build (derived / shared-anchor
    rows) and the exact build (spe_table_compare on the device): route mismatches
    (must be 0), latency / reliability bit differences, the largest relative
    difference, and ceil(latency * 1e6) flips -- Shadow's packet delay in ns
    (shd-worker.c:244).  C4 in quarters of the source blocks (two 55-GB tables at
    a time)."""
    from shadow_amd import spe
    top, att, desc = workload(config)
    g = spe.Graph(top)
    order = g.order_sources(att)
    nblk = (len(order) + 63) // 64
    parts = parts or (4 if config == "c4" else 1)
    cuts = np.linspace(0, nblk, parts + 1).astype(int)
    tot = {}
    t0 = time.perf_counter()
    for b0, b1 in zip(cuts[:-1], cuts[1:]):
        d = spe.PathTable(g, order, blocks=(int(b0), int(b1)), exact_sources=False)
        d.build()
        x = spe.PathTable(g, order, blocks=(int(b0), int(b1)), exact_sources=True)
        x.build()
        r = d.compare(x, 1e-9)
        d.close()
        x.close()
        for k, v in r.items():
            if k.startswith("max_"):
                tot[k] = max(tot.get(k, 0.0), v)
            elif not k.startswith("first_"):
                tot[k] = tot.get(k, 0) + v
    tot["tolerance"] = 1e-9
    tot["parts"] = parts
    tot["seconds"] = round(time.perf_counter() - t0, 1)
    tot["note"] = ("default build vs exact_sources=1 on every entry (spe_table_compare): routes must match; "
                   "delivery_flips = pairs whose ceil(latency * 1e6) ns packet delay differs (shd-worker.c:244)")
    return tot


# The default run (C3 at N = 1) also measures BASELINE's other configurations
# (and C2 on the FW engine),
# each in a child process of its own once the C3 table is freed (C4's table alone
# is 220 GB), so that every config has a line on the driver's box.  A child that
# fails is recorded with its exit status and the tail of its output; the C3 line
# stands either way.
SIDE_CONFIGS = (
    ("c5", ["--config", "c5", "--steps", "10", "--warmup", "2", "--cpu-seconds", "6"]),
    ("c2", ["--config", "c2", "--cpu-seconds", "6", "--cpu-sources", "0"]),
    ("c4", ["--config", "c4", "--steps", "2", "--cpu-seconds", "6"]),   # 1,000-source 1-core CPU sample (~50 s)
    # the tables topology_seal builds for these graphs (non-dyadic latencies: one lane per
    # source, bit-exact), with their entry-by-entry differences from the default build
    ("c3_exact", ["--config", "c3", "--exact", "--steps", "3", "--no-cpu-baseline"]),
    ("c4_exact", ["--config", "c4", "--exact", "--steps", "2", "--no-cpu-baseline"]),
    ("c1", ["--config", "c1", "--cpu-seconds", "4", "--cpu-sources", "0"]),
    # the drop-in end to end: GraphML -> topology_new -> attach -> seal, then batched
    # lookups.  Each shim line follows a config that frees little device memory: the
    # driver clears the VRAM a finished child released (≈ 50 GB/s), and a seal started
    # right after a 160-GB child waits for it (C3 seal 3.6 s after c5_on_c4, 1.2 s after
    # a small config or alone, MEASUREMENTS.md round 6)
    ("c3_shim", ["--config", "c3shim", "--steps", "3", "--cpu-seconds", "4", "--queries", "20000000"]),
    ("c5_on_c4", ["--config", "c5", "--c5-table", "c4", "--steps", "10", "--warmup", "2", "--cpu-seconds", "6"]),
    ("c2fw", ["--config", "c2fw", "--steps", "1"]),   # the FW engine's whole C2 table
    ("c4_shim", ["--config", "c4shim", "--steps", "2", "--cpu-seconds", "4", "--queries", "20000000"]),
)


RANDOM_16B_READS_PER_S = 37.15e9   # tools/probe_line_fetch.hip on one MI355X (profiles/r06_line_fetch.json)
LINE_MAX_BYTES = 6000   # the driver parses the LAST stdout line from a tail of about 8 KB


def side_summary(v: dict) -> dict:
    """One side config's record cut to what the headline line carries (VERDICT r05
    Next #1): value, unit, its time per step or per table, the dominant kernel's
    roofline fraction, and the default-vs-exact verdict; the full record stays in
    the file named by `full_record`."""
    if "error" in v or "skipped" in v:
        return {k: (str(x)[:160] if isinstance(x, str) else x) for k, x in v.items() if k in ("error", "skipped", "wall_s")}
    if "metric" not in v:   # already a summary (a rank's compacted line passed on by run_multi)
        return v
    s = {"value": v.get("value"), "unit": v.get("unit")}
    for k in ("full_table_time_s", "ms_per_step"):
        if v.get(k) is not None:
            s[k] = v[k]
            break
    roof = v.get("roofline") or {}
    if "frac" in roof:
        s["frac"] = roof["frac"]
        s["kernel"] = roof.get("kernel", "").split(" ")[0]
    vx = v.get("vs_default_build")
    if vx:
        s["vs_default_build"] = {k: vx.get(k) for k in ("route_mismatch", "delivery_flips", "max_latency_rel_err")}
    if "single_call_queries_per_s" in v:
        s["single_call_queries_per_s"] = v["single_call_queries_per_s"]
        if "single_call_queries_per_s_cold" in v:
            s["single_call_queries_per_s_cold"] = v["single_call_queries_per_s_cold"]
        c = v.get("single_call_queries_per_s_c") or {}
        if "single_calls_per_s_1_thread" in c:
            s["single_call_c"] = [c["single_calls_per_s_1_thread"], c["single_calls_per_s_all_threads"], c["threads"]]
            if c.get("settled_calls_per_s_1_thread"):
                s["single_call_c_settled"] = [c["settled_calls_per_s_1_thread"], c["settled_calls_per_s_all_threads"]]
        s["seal_s"] = (v.get("startup_s") or {}).get("seal_table_and_mirror")
    if v.get("cpu_baseline"):
        s["cpu_1core"] = v["cpu_baseline"].get("value")
    s["wall_s"] = v.get("wall_s")
    return s


def compact_line(line: dict, full_path) -> dict:
    """The line rank 0 prints: every headline field, `roofline` and `cpu_baseline`
    in full, side configs as summaries (side_summary); bounded by LINE_MAX_BYTES so
    that the driver's tail of stdout always holds the whole line."""
    out = {k: v for k, v in line.items() if k != "side_configs"}
    if "side_configs" in line:
        out["side_configs"] = {k: side_summary(v) for k, v in line["side_configs"].items()}
    if full_path:
        out["full_record"] = full_path
    # shed optional detail, least useful first, until the line fits
    for k in ("kernel_launches", "rank0_step_s", "precompute_end_to_end_s", "speedup_vs_cpu_1core", "split",
              "kernel_ms", "roofline_rows"):
        if len(json.dumps(out)) <= LINE_MAX_BYTES:
            break
        out.pop(k, None)
    if len(json.dumps(out)) > LINE_MAX_BYTES and "side_configs" in out:
        out["side_configs"] = {k: {"value": v.get("value"), "unit": v.get("unit")} for k, v in out["side_configs"].items()}
    return out


def emit(line: dict, tag: str = "") -> None:
    """Print the line on stdout as the LAST thing this process writes there.  A
    line that carries side configs (or would exceed LINE_MAX_BYTES) is written in
    full to gpurun_out/ and printed compacted; the headline value is echoed on
    stderr as the side configs' are."""
    full_path = None
    if "side_configs" in line or len(json.dumps(line)) > LINE_MAX_BYTES:
        d = os.path.join(ROOT, "gpurun_out")
        try:
            os.makedirs(d, exist_ok=True)
            full_path = os.path.join("gpurun_out", f"bench_full{tag}_n{line.get('n_gpus', 1)}.json")
            with open(os.path.join(ROOT, full_path), "w") as f:
                json.dump(line, f, indent=1)
        except OSError:
            full_path = None
        line = compact_line(line, full_path)
    roof = line.get("roofline") or {}
    print(f"[bench] headline: {line.get('value')} {line.get('unit')} ({line.get('ms_per_step')} ms/step, "
          f"roofline frac {roof.get('frac')} on {roof.get('kernel')}, cpu_baseline "
          f"{(line.get('cpu_baseline') or {}).get('value')})", file=sys.stderr, flush=True)
    sys.stderr.flush()
    print(json.dumps(line), flush=True)


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return int(s.getsockname()[1])


def launch_ranks(n: int, argv, timeout_s: float = 0.0):
    """`python bench.py --gpus N` without torchrun: start N rank processes of this
    script (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, rendezvous on
    127.0.0.1), as torchrun would.  The parent never touches the GPU and never
    execs: it waits for the children, echoes their progress, and returns rank 0's
    JSON line (None when any rank failed: the others are then terminated, since
    they would block in a collective)."""
    import threading
    env = dict(os.environ)
    for k in ("RANK", "LOCAL_RANK", "GROUP_RANK", "TORCHELASTIC_RUN_ID"):
        env.pop(k, None)
    env.update({"WORLD_SIZE": str(n), "LOCAL_WORLD_SIZE": str(n), "MASTER_ADDR": "127.0.0.1",
                "MASTER_PORT": str(_free_port())})
    procs = []
    for r in range(n):
        e = dict(env, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + list(argv), env=e, cwd=ROOT,
                                      stdout=subprocess.PIPE, text=True, start_new_session=True))
    found = [None]

    def pump(p, rank):   # rank 0's JSON line is the result; everything else is progress
        for line in p.stdout:
            if rank == 0 and line.startswith("{"):
                found[0] = line.strip()
            else:
                sys.stderr.write(f"[rank {rank}] {line}")
                sys.stderr.flush()

    th = [threading.Thread(target=pump, args=(p, r), daemon=True) for r, p in enumerate(procs)]
    for x in th:
        x.start()
    t0 = time.perf_counter()
    failed = None
    while True:
        codes = [p.poll() for p in procs]
        bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
        if bad:
            failed = bad
            break
        if all(c == 0 for c in codes):
            break
        if timeout_s > 0 and time.perf_counter() - t0 > timeout_s:
            failed = [("timeout", timeout_s)]
            break
        time.sleep(0.2)
    if failed:
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, 15)
                except OSError:
                    pass
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                try:
                    os.killpg(p.pid, 9)
                except OSError:
                    pass
                p.wait()
        print(f"[bench] rank(s) failed: {failed}", file=sys.stderr, flush=True)
    for x in th:
        x.join(timeout=10)
    return None if failed else found[0]


def bench_inproc(args, n: int, config: str):
    """Shadow's own multi-GPU model (one process, shd-master.c:390-394): ONE path
    table over devices 0..N-1 (spe_table_opts.devices), each device building its
    share on its own host thread and stream, the records broadcast / gathered into
    a replica on every device (the compute-versus-gather split of DESIGN §6).  A
    step is one whole table build (spe_table_build), replicas included."""
    from shadow_amd import spe
    top, att, desc = workload(config)
    t0 = time.perf_counter()
    g = spe.Graph(top, device=0)
    prep_s = time.perf_counter() - t0
    t0 = time.perf_counter()
    att = g.order_sources(att)
    order_s = time.perf_counter() - t0
    rehearse = os.environ.get("SPE_BENCH_REHEARSE_ONE_GPU") == "1"
    devs = [0] * n if rehearse else list(range(n))
    t = spe.PathTable(g, att, devices=devs)
    for _ in range(max(0, args.warmup)):
        t.build()
    steps = args.steps if args.steps > 0 else 2
    runs, stats = [], []
    for _ in range(steps):
        t0 = time.perf_counter()
        st = t.build()
        runs.append(time.perf_counter() - t0)
        stats.append(st)
    el = sum(runs)
    A = int(att.shape[0])
    st = stats[-1]
    line = {"metric": f"{config.upper()} whole path table, one process over {n} devices (spe_table_opts.devices)",
            "value": round(A * steps / el, 1), "unit": "sources/s", "n_gpus": n, "steps": steps,
            "higher_is_better": True, "scaling": "strong", "dtype": "f64", "data": "synthetic",
            "devices": devs, "rehearsal_one_gpu": rehearse,
            "config": {"workload": desc, "attached": A},
            "full_table_time_s": round(el / steps, 4), "all_runs_s": [round(x, 4) for x in runs],
            "graph_prep_s": round(prep_s, 4), "slot_order_s": round(order_s, 4),
            "build_wait_s": round(st.get("build_wait_seconds", 0.0), 4),
            "gather_s": round(st.get("gather_seconds", 0.0), 4),
            "gather_mode": {1: "rccl", 2: "peer"}.get(st.get("gather", 0), st.get("gather", 0)),
            "shared_blocks": st.get("shared_blocks"), "local_blocks": st.get("local_blocks"),
            "nblk": (A + 63) // 64}
    t.close()
    print(json.dumps(line), flush=True)


def side_configs(timeout_s: float = 240.0):
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    out = {}
    for name, argv in SIDE_CONFIGS:
        t0 = time.perf_counter()
        try:
            r = subprocess.run([sys.executable, "-u", os.path.abspath(__file__), "--no-side"] + argv, env=env,
                               cwd=ROOT, capture_output=True, text=True, timeout=timeout_s)
            lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
            if r.returncode == 0 and lines:
                out[name] = json.loads(lines[-1])
            else:
                out[name] = {"error": f"exit status {r.returncode}", "tail": (r.stdout + r.stderr)[-600:]}
        except subprocess.TimeoutExpired:
            out[name] = {"error": f"timed out after {timeout_s:.0f} s"}
        out[name]["wall_s"] = round(time.perf_counter() - t0, 1)
        print(f"[bench] side config {name}: {out[name].get('value', out[name].get('error'))} "
              f"({out[name]['wall_s']} s)", file=sys.stderr, flush=True)
    return out


def run_multi(args, n: int):
    """`python bench.py --gpus N` (N > 1) without torchrun -- the driver's plain
    command line: N rank processes of this script (launch_ranks), then, unless
    --no-inproc, the in-process multi-device table (bench_inproc) for C3 and C4 in
    child processes once the ranks have exited; rank 0's line is printed with
    those under side_configs.  Exits non-zero when a rank fails."""
    argv = [a for a in sys.argv[1:]]
    line = launch_ranks(n, argv)
    if line is None:
        raise SystemExit(1)
    out = json.loads(line)
    dry = os.environ.get("SPE_BENCH_LAUNCH_DRYRUN") == "1"
    if not dry and not args.no_inproc and args.config == "c3":
        env = dict(os.environ)
        for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
            env.pop(k, None)
        rehearse = env.get("SPE_BENCH_REHEARSE_ONE_GPU") == "1"
        side = out.setdefault("side_configs", {})
        # (rehearsal on one GPU: C4's replicated records, 160 GB per replica, do not fit twice)
        for cfg in (("c3",) if rehearse else ("c3", "c4")):
            t0 = time.perf_counter()
            try:
                r = subprocess.run([sys.executable, "-u", os.path.abspath(__file__), "--inproc", str(n), "--config", cfg,
                                    "--steps", "3", "--warmup", "1"], env=env, cwd=ROOT, capture_output=True,
                                   text=True, timeout=300)
                lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
                side[f"inproc_{cfg}"] = (json.loads(lines[-1]) if r.returncode == 0 and lines else
                                         {"error": f"exit status {r.returncode}", "tail": (r.stdout + r.stderr)[-600:]})
            except subprocess.TimeoutExpired:
                side[f"inproc_{cfg}"] = {"error": "timed out after 300 s"}
            side[f"inproc_{cfg}"]["wall_s"] = round(time.perf_counter() - t0, 1)
            print(f"[bench] in-process {cfg} over {n} devices: {side[f'inproc_{cfg}'].get('value', side[f'inproc_{cfg}'].get('error'))}",
                  file=sys.stderr, flush=True)
    emit(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs of this node (default 1).  Without torchrun, N > 1 starts N rank processes itself")
    ap.add_argument("--steps", type=int, default=0, help="whole tables timed (0 = 3)")
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c3")
    ap.add_argument("--groups", type=int, default=0, help="64-source blocks per build launch (0 = auto)")
    ap.add_argument("--engine", type=int, default=0, help="0 auto, 1 batch (64-lane HBM state), 2 LDS-resident rows")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-sources", type=int, default=1000,
                    help="sources the 1-core CPU baseline times (BASELINE.md: 1,000; 0 = --cpu-seconds bound)")
    ap.add_argument("--shared-frac", type=float, default=-1.0,
                    help="N > 1: fraction of source blocks sharded + all-gathered, the rest built by every "
                         "rank (-1 = from the measured build time and gather bandwidth, DESIGN 6)")
    ap.add_argument("--no-north-star", action="store_true",
                    help="N > 1: skip the C4 line measured after the C3 line in the same ranks")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--exact", action="store_true",
                    help="build with spe_table_opts.exact_sources = 1 (the drop-in's table on non-dyadic latencies) "
                         "and report its differences from the default build (spe_table_compare)")
    ap.add_argument("--no-compare", action="store_true",
                    help="--exact: skip the entry-by-entry comparison with the default build (PMC passes)")
    ap.add_argument("--no-profile", action="store_true", help="skip per-launch HIP events")
    ap.add_argument("--no-gather", action="store_true", help="N > 1: skip the all-gather (build only)")
    ap.add_argument("--gather", choices=("auto", "all_gather", "p2p"), default="auto",
                    help="N > 1: RCCL all_gather_into_tensor or world - 1 concurrent peer exchanges; auto = the faster "
                         "one measured by the split calibration (all_gather when the fraction is given)")
    ap.add_argument("--queries", type=int, default=100_000_000, help="c5: lookups per step")
    ap.add_argument("--c5-table", default="c3", choices=("c3", "c4"),
                    help="c5: the table the lookups read (c4: 100k x 100k, 220 GB on one GPU)")
    ap.add_argument("--pois", type=int, default=10000, help="complete: POIs")
    ap.add_argument("--pmc-json", default=None, help="per-dispatch HBM bytes from tools/pmc_to_json.py")
    ap.add_argument("--full-table", action="store_true", help="(the default; kept for old command lines)")
    ap.add_argument("--shares", type=int, default=1, help="emulate one rank of a job with this many GPUs")
    ap.add_argument("--share-index", type=int, default=0, help="--shares: the rank whose chunks this run builds")
    ap.add_argument("--no-side", action="store_true",
                    help="default C3 run at N = 1: skip the C1/C2/C4/C5 lines measured in child processes")
    ap.add_argument("--inproc", type=int, default=0,
                    help="N > 1: one process over devices 0..N-1 (spe_table_opts.devices) instead of N ranks")
    ap.add_argument("--no-inproc", action="store_true",
                    help="N > 1 without torchrun: skip the in-process multi-device lines after the ranks")
    args = ap.parse_args()
    if args.config == "complete":
        return bench_complete(args)
    if args.config == "c2fw":
        return bench_fw(args)
    if args.config in ("c3shim", "c4shim"):
        return bench_shim(args, args.config[:2])
    if args.inproc > 0:
        return bench_inproc(args, args.inproc, args.config)

    gpus = args.gpus if args.gpus is not None else 1
    if "WORLD_SIZE" not in os.environ and gpus > 1:
        return run_multi(args, gpus)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus is not None and world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} (torchrun's --nproc-per-node)")
    if os.environ.get("SPE_BENCH_LAUNCH_DRYRUN") == "1":   # the launcher's CPU test: gloo ranks, no GPU
        import torch
        import torch.distributed as dist
        dist.init_process_group("gloo")
        x = torch.tensor([float(rank + 1)])
        dist.all_reduce(x)
        if rank == 0:
            print(json.dumps({"metric": METRIC, "n_gpus": world, "rank_sum": float(x.item()), "dryrun": True}),
                  flush=True)
        dist.destroy_process_group()
        return
    # rehearsal of the N > 1 path on a one-GPU box: every rank on device 0, gloo
    # instead of RCCL (RCCL refuses two ranks on one device); never for numbers
    rehearse = os.environ.get("SPE_BENCH_REHEARSE_ONE_GPU") == "1"
    if rehearse:
        local = 0
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    if args.config == "c5":
        bench_lookup(args, rank, world, local, dist)
    else:
        line = bench_table(args, rank, world, local, dist)
        import gc
        import torch
        if world > 1 and args.config == "c3" and not args.no_north_star and args.shares == 1:
            # the north star's own target in the same ranks: the whole 200k-vertex /
            # 100k-host table replicated on every GPU (C4), after the C3 table is freed
            # (not in a one-GPU rehearsal: N replicas of its 160-GB records do not fit one GPU)
            if rehearse:
                if line is not None:
                    line["side_configs"] = {"c4": {"skipped": "one-GPU rehearsal: N replicas of the C4 records "
                                                              "do not fit one device"}}
            else:
                gc.collect()
                torch.cuda.empty_cache()
                c4 = bench_table(args, rank, world, local, dist, config="c4")
                if line is not None:
                    line["side_configs"] = {"c4": c4}
        if line is not None and args.exact and world == 1 and args.config in ("c3", "c4") and not args.no_compare:
            gc.collect()
            torch.cuda.empty_cache()
            line["vs_default_build"] = default_vs_exact(args.config)
        if line is not None:
            if world == 1 and args.config == "c3" and not args.no_side and args.shares == 1:
                gc.collect()
                torch.cuda.empty_cache()
                line["side_configs"] = side_configs()
            emit(line, "" if rank == 0 and world == 1 and args.config == "c3" else f"_{args.config}")
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
