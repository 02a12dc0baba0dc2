"""Benchmark: multi-source SSSP path-table rows on MI355X (BASELINE.json metric
"SSSP sources/sec + full path-table time, % HBM roofline, at 1/2/4/8 GPU").

Workload (default, config C3 of BASELINE.json / SURVEY.md §8d): synthetic
Barabasi-Albert n=50,000, m=3, seed 3, latency U(1,100) ms, loss U(0,0.01),
every vertex attached (A = 50,000 sources x 50,000 targets; slots in the
engine's clustered order, spe_order_sources).  A step = one build launch of the
table's groups per launch (48 at C3: 3,072 sources) or `--blocks-per-step`
64-source blocks: full rows (latency, reliability, next hop, hops) written into
the HBM-resident table.  Ranks take disjoint source
blocks (weak scaling: fixed rows per GPU per step, no collective on the data
path).  Rank 0 prints one JSON line.

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


def cpu_baseline(top, att, seconds: float, seed: int = 6):
    """Oracle (C restatement of igraph Dijkstra + Shadow row rules, -O2, 1 core)
    timed on a bounded sample of this workload's sources."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle import Oracle
    o = Oracle(top)
    rng = np.random.default_rng(seed)
    order = rng.permutation(att.shape[0])
    done, t0, dj = 0, time.perf_counter(), 0.0
    chunk = 8
    while time.perf_counter() - t0 < seconds and done < att.shape[0]:
        src = att[order[done:done + chunk]]
        r = o.rows(src, att, nthreads=1, want_dijkstra_time=True)
        dj += r["dijkstra_seconds"]
        done += src.shape[0]
    el = time.perf_counter() - t0
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    # BASELINE.md's "optimistic, all cores" (OpenMP over sources; the reference
    # serialises Dijkstra under graphLock, so this is a bound it cannot reach)
    nt = min(16, os.cpu_count() or 1)
    done_all, t1 = 0, time.perf_counter()
    while time.perf_counter() - t1 < seconds / 4 and done + done_all < att.shape[0]:
        src = att[order[done + done_all:done + done_all + 8 * nt]]
        o.rows(src, att, nthreads=nt)
        done_all += src.shape[0]
    el_all = time.perf_counter() - t1
    return {"value": done / el, "unit": "sources/s", "cores": 1, "kind": "port",
            "sample": f"{done} seeded-random sources (seed {seed}) x {att.shape[0]} targets, full row build, "
                      f"{el:.1f} s; Dijkstra-only {done / max(dj, 1e-9):.1f} sources/s",
            "optimistic_all_cores": {"value": round(done_all / max(el_all, 1e-9), 1), "threads": nt,
                                     "sample": f"{done_all} further sources"},
            "cpu_model": model, "host_nproc": os.cpu_count()}


def pmc_traffic(args, kernel):
    """HBM bytes per dispatch of `kernel` from a committed PMC summary (separate
    rocprofv3 --pmc passes of this same bench command), or None."""
    path = args.pmc_json
    if path is None:
        cand = os.path.join(ROOT, "profiles", f"r01_pmc_{args.config}.json")
        path = cand if os.path.exists(cand) else None
    if not path:
        return None
    try:
        k = json.load(open(path))["kernels"][kernel]
        return {"hbm_bytes_per_launch": round(k["hbm_bytes_per_dispatch"]),
                "fetch_bytes_per_launch": round(k["fetch_bytes_per_dispatch"]),
                "write_bytes_per_launch": round(k["write_bytes_per_dispatch"]),
                "source": os.path.relpath(path, ROOT)}
    except (KeyError, OSError, ValueError):
        return None


def bench_lookup(args):
    """C5: batched per-packet lookups (s_slot, t_slot) -> (latency, reliability, ok)
    against the HBM-resident C3 table; 41 algorithmic bytes per query."""
    import torch
    from shadow_amd import spe
    top, att, desc = workload("c3")
    g = spe.Graph(top, device=0)
    t = spe.PathTable(g, att)
    t.build()
    q = args.queries
    gen = torch.Generator(device="cuda").manual_seed(5)
    pairs = torch.randint(0, t.A, (q, 2), dtype=torch.int32, device="cuda", generator=gen)
    lat = torch.empty(q, dtype=torch.float64, device="cuda")
    rel = torch.empty(q, dtype=torch.float64, device="cuda")
    ok = torch.empty(q, dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    steps = args.steps if args.steps > 0 else 10
    for _ in range(args.warmup):
        t.lookup_batch(pairs.data_ptr(), q, lat.data_ptr(), rel.data_ptr(), ok.data_ptr(), stream)
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    for _ in range(steps):
        t.lookup_batch(pairs.data_ptr(), q, lat.data_ptr(), rel.data_ptr(), ok.data_ptr(), stream)
    ev1.record()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    kern_s = ev0.elapsed_time(ev1) / 1e3 / steps
    assert bool(ok.all().item())
    value = q * steps / el
    ach = 41.0 * q / kern_s / 1e9
    cpu = None
    if not args.no_cpu_baseline:
        cpu = cpu_lookup_baseline(t.A, args.cpu_seconds)
    line = {"metric": "per-packet lookup queries/s against the GPU-resident path table (config C5)",
            "value": round(value, 1), "unit": "queries/s", "n_gpus": 1, "steps": steps, "warmup": args.warmup,
            "ms_per_step": round(1e3 * el / steps, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f64", "data": "synthetic",
            "config": {"workload": f"C5: {q} uniform (s,t) slot pairs (seed 5) on the {desc} table"},
            "roofline": {"bound": "hbm", "kernel": "k_lookup", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": pmc_traffic(args, "k_lookup"),
                         "algorithmic_bytes_per_query": 41},
            "cpu_baseline": cpu}
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
    nt = min(16, os.cpu_count() or 1)
    t1 = time.perf_counter()
    c.lookup(sip, dip, nthreads=nt)
    c.lookup(sip, dip, nthreads=nt)
    el_all = time.perf_counter() - t1
    return {"value": round(done / el, 1), "unit": "queries/s", "cores": 1, "kind": "port",
            "sample": f"{done} lookups over a 4M-pair cache (seed {seed}): 2 IP->slot probes + src and (src,dst) "
                      f"cache probes per query, {el:.1f} s",
            "optimistic_all_cores": {"value": round(2 * npairs / el_all, 1), "threads": nt}}


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


def bench_fw(args):
    """C2 on the blocked min-plus Floyd-Warshall comparison engine (spe_fw_apsp):
    the north star's dense algorithm, timed for distances only (FW association,
    not the bit-exact table) against the LDS SSSP engine's full exact table."""
    import torch
    from shadow_amd import spe
    top, att, desc = workload("c2")
    g = spe.Graph(top, device=0)
    n = g.info()["n_relax_vertices"]
    ld = (n + 63) // 64 * 64
    D = torch.empty(ld * ld, dtype=torch.float64, device="cuda")
    g.fw_apsp(D.data_ptr(), ld)   # warm-up
    secs = [g.fw_apsp(D.data_ptr(), ld) for _ in range(max(1, args.steps or 3))]
    sec = min(secs)
    nb = ld // 64
    relax = float(nb) ** 3 * 64 ** 3
    line = {"metric": "C2 all-pairs distances by blocked min-plus Floyd-Warshall (comparison engine)",
            "value": round(sec, 4), "unit": "s", "higher_is_better": False, "n_gpus": 1, "dtype": "f64",
            "data": "synthetic", "config": {"workload": desc, "n_relax": n, "ld": ld},
            "roofline": {"bound": "fp64-valu", "achieved": round(2 * relax / sec / 1e12, 2),
                         "peak": 78.6, "unit": "TFLOP/s", "frac": round(2 * relax / sec / 1e12 / 78.6, 4),
                         "note": "2 FP64 ops (add, min) per (min,+) relaxation, ld^3 relaxations"},
            "all_runs_s": [round(x, 4) for x in secs]}
    print(json.dumps(line), flush=True)


def bench_full_table(args, rank, world, local, dist):
    """Whole path-table precompute (BASELINE north star: C4 on 8 GPUs in < 10 s).
    Rank r owns the contiguous source-block range r of `shares` (= world, or more to
    emulate one rank of a larger job on fewer GPUs); with --gather and world > 1 the
    latency/reliability records are then all-gathered over RCCL into a full
    replicated table on every GPU (one contiguous SB64 span per rank)."""
    import torch
    from shadow_amd import spe
    top, att, desc = workload(args.config)
    g = spe.Graph(top, device=local)
    t_ord = time.perf_counter()
    att = g.order_sources(att)   # slot numbering is the caller's: clustered sources (host side)
    t_ord = time.perf_counter() - t_ord
    info = g.info()
    A = int(att.shape[0])
    nblk = (A + 63) // 64
    shares = max(world, args.shares)
    share = rank if shares == world else args.share_index
    cb = (nblk + shares - 1) // shares
    b0, b1 = min(nblk, share * cb), min(nblk, (share + 1) * cb)
    elems = cb * A * 64
    dev = torch.device("cuda", local)
    bufs = [torch.empty((elems, 2), dtype=torch.float64, device=dev),   # {latency, reliability}
            torch.empty(elems, dtype=torch.int32, device=dev), torch.empty(elems, dtype=torch.int16, device=dev)]
    t = None
    if b1 > b0:   # (a rank past the last block owns nothing but still joins the gather)
        t = spe.PathTable(g, att, blocks=(b0, b1), ext=[b.data_ptr() for b in bufs], groups=args.groups)
    if t is not None:   # warm-up: one batch (kernel code objects, first-touch of the state)
        t.build_blocks(b0, min(b1, b0 + 1))
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    if t is not None:
        t.build()
    torch.cuda.synchronize(dev)
    t_build = time.perf_counter() - t0
    if dist is not None:
        dist.barrier()
    t_all = time.perf_counter() - t0
    gather = None
    if args.gather and dist is not None:
        full_lr = torch.empty((world * elems, 2), dtype=torch.float64, device=dev)
        torch.cuda.synchronize(dev)
        dist.barrier()
        tg = time.perf_counter()
        dist.all_gather_into_tensor(full_lr, bufs[0])
        torch.cuda.synchronize(dev)
        dist.barrier()
        t_gather = time.perf_counter() - tg
        t_all = time.perf_counter() - t0
        gather = {"bytes_per_gpu_received": int(2 * (world - 1) * elems * 8), "seconds": round(t_gather, 3),
                  "GBps_per_gpu": round(2 * (world - 1) * elems * 8 / t_gather / 1e9, 1)}
    x = torch.tensor([t_build, t_all], dtype=torch.float64, device=dev)
    if dist is not None:
        dist.all_reduce(x, op=dist.ReduceOp.MAX)
    t_build, t_all = float(x[0]), float(x[1])
    if rank == 0:
        srcs = min(A, b1 * 64) - b0 * 64 if shares != world else A
        # SURVEY §8d per-source algorithmic bytes on the FULL graph (the reference's
        # Dijkstra scans every vertex and edge; pendant pruning is this engine's saving)
        m_dir_full = int(np.count_nonzero(top.esrc != top.edst)) * (1 if top.directed else 2)
        b_s = 12.0 * m_dir_full + 28.0 * top.n + 22.0 * A + 8.0
        per_gpu_s = t_build
        ach = b_s * srcs / (1 if shares != world else world) / max(per_gpu_s, 1e-9) / 1e9
        roof_full = {"bound": "hbm", "kernel": "whole build (relax + rows), per GPU", "achieved": round(ach, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                     "algorithmic_bytes_per_source": b_s, "traffic": None,
                     "note": "SURVEY 8d B_s = 12 m_dir + 28 n + 22 A + 8 over the full graph"}
        line = {"metric": "full path-table precompute time (north star: C4 on 8 GPUs < 10 s)",
                "value": round(t_all, 3), "unit": "s", "higher_is_better": False, "n_gpus": world,
                "dtype": "f64", "data": "synthetic",
                "config": {"workload": desc, "n": info["n_vertices"], "relax_vertices": info["n_relax_vertices"],
                           "m_dir_relax": info["n_relax_entries"], "attached": A, "slot_order": "spe_order_sources", "slot_order_ms": round(1e3 * t_ord, 1),
                           "shares": shares, "share_built": [b0, b1] if shares != world else "all",
                           "table_bytes_per_gpu": int(elems * 22)},
                "build_s": round(t_build, 3), "sources_per_s_per_gpu": round(srcs / max(t_build, 1e-9) / (1 if shares != world else world), 1),
                "roofline": roof_full,
                "gather": gather,
                "note": ("emulated: this run built ONE share of a %d-way split (weak-scaling equivalent of one rank); "
                         "no all-gather measured" % shares) if shares != world else None}
        print(json.dumps(line), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=0, help="0 = one full table at N=1")
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c3")
    ap.add_argument("--blocks-per-step", type=int, default=0,
                    help="64-source blocks per step; 0 = one build launch (the table's groups per launch)")
    ap.add_argument("--groups", type=int, default=0)
    ap.add_argument("--engine", type=int, default=0, help="0 auto, 1 batch (64-lane HBM state), 2 LDS-resident rows")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true", help="skip per-launch HIP events")
    ap.add_argument("--queries", type=int, default=100_000_000, help="c5: lookups per step")
    ap.add_argument("--pois", type=int, default=10000, help="complete: POIs")
    ap.add_argument("--pmc-json", default=None, help="per-dispatch HBM bytes from tools/pmc_to_json.py")
    ap.add_argument("--full-table", action="store_true", help="time one whole path-table precompute")
    ap.add_argument("--gather", action="store_true", help="--full-table: RCCL all-gather of latency/reliability")
    ap.add_argument("--shares", type=int, default=1, help="--full-table: split into this many source shares")
    ap.add_argument("--share-index", type=int, default=0, help="--full-table: the share this run builds")
    args = ap.parse_args()
    if args.config == "c5":
        return bench_lookup(args)
    if args.config == "complete":
        return bench_complete(args)
    if args.config == "c2fw":
        return bench_fw(args)

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
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

    if args.full_table:
        bench_full_table(args, rank, world, local, dist)
        if dist is not None:
            dist.destroy_process_group()
        return

    from shadow_amd import spe
    top, att, desc = workload(args.config)
    g = spe.Graph(top, device=local)
    t_ord = time.perf_counter()
    att = g.order_sources(att)   # slot numbering is the caller's: clustered sources (host side)
    t_ord = time.perf_counter() - t_ord
    info = g.info()
    t = spe.PathTable(g, att, groups=args.groups, engine=args.engine)
    A = t.A
    nblk = t.nblocks
    lay = t.layout()
    bps = args.blocks_per_step if args.blocks_per_step > 0 else (
        lay["groups_per_launch"] if lay["engine"] == spe.SPE_ENGINE_BATCH else 16)
    nwin = math.ceil(nblk / bps)
    steps = args.steps if args.steps > 0 else nwin

    def window(k: int):
        w = (k * world + rank) % nwin
        return w * bps, min(nblk, (w + 1) * bps)

    def sources_in(b0, b1):
        return min(A, b1 * 64) - b0 * 64

    def barrier():
        if dist is not None:
            dist.barrier()

    for k in range(args.warmup):
        t.build_blocks(*window(k))
    if not args.no_profile:
        t.profile(True)
    it_total, fr_total, done = 0, 0, 0
    barrier()
    t0 = time.perf_counter()
    for k in range(steps):
        b0, b1 = window(args.warmup + k)
        st = t.build_blocks(b0, b1)
        it_total += st["iterations"]
        fr_total += st["active_rounds"]
        done += sources_in(b0, b1)
    barrier()
    el = time.perf_counter() - t0
    kp = t.kernel_profile() if not args.no_profile else None

    total_sources = done
    if dist is not None:
        import torch
        x = torch.tensor([el], dtype=torch.float64, device="cuda")
        dist.all_reduce(x, op=dist.ReduceOp.MAX)
        el = float(x.item())
        y = torch.tensor([done], dtype=torch.float64, device="cuda")
        dist.all_reduce(y)
        total_sources = int(y.item())

    value = total_sources / el
    n, m_dir = info["n_vertices"], info["n_relax_entries"]
    # SURVEY §8d per-source algorithmic bytes, split by stage
    b_relax = 12.0 * m_dir + 28.0 * n + 8.0
    b_rows = 22.0 * A
    roof = None
    extra = {}
    lds = kp is not None and kp["lds"]["launches"] > 0
    direct = kp is not None and kp["direct"]["launches"] > 0 and kp["relax"]["launches"] == 0 and not lds
    if lds:   # one fused kernel: relaxation in LDS + row writes
        b_relax += b_rows
    if direct:   # complete graph: every row is DIRECT, 38 B per pair
        b_relax = 38.0 * A
    if kp is not None:
        kname = "k_sssp_lds" if lds else ("k_rows_direct" if direct else "k_relax")
        rl = kp["lds" if lds else ("direct" if direct else "relax")]
        relax_s = rl["ms"] / 1e3
        ach = b_relax * done / relax_s / 1e9 if relax_s > 0 else 0.0
        traffic = pmc_traffic(args, kname)
        roof = {"bound": "hbm", "kernel": kname + (" (SSSP + rows, LDS-resident state)" if lds else
                                                   (" (DIRECT rows)" if direct else " (SSSP stage)")),
                "achieved": round(ach, 1),
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic,
                "launches": rl["launches"], "launch_avg_us": round(1e3 * rl["ms"] / max(1, rl["launches"]), 2),
                "algorithmic_bytes_per_source": b_relax}
        rw = kp["rows"]
        rows_s = rw["ms"] / 1e3
        extra["roofline_rows"] = {"kernel": "k_rows_sssp", "achieved": round(b_rows * done / rows_s / 1e9, 1)
                                  if rows_s > 0 else 0.0, "unit": "GB/s", "launches": rw["launches"],
                                  "launch_avg_us": round(1e3 * rw["ms"] / max(1, rw["launches"]), 2),
                                  "algorithmic_bytes_per_source": b_rows}
        extra["kernel_ms"] = {k: round(v["ms"], 3) for k, v in kp.items()}
        extra["kernel_launches"] = {k: v["launches"] for k, v in kp.items()}
        extra["pipeline_frac_of_hbm"] = round((b_relax + (0 if lds else b_rows)) * value / 1e9 / HBM_PEAK_GBS, 4)
        extra["engine"] = "lds" if lds else ("direct" if direct else "batch")
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(top, att, args.cpu_seconds)
    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "sources/s", "n_gpus": world, "steps": steps,
            "warmup": args.warmup, "ms_per_step": round(1e3 * el / steps, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
            "config": {"workload": desc, "n": n, "m_dir": m_dir, "attached": A, "slot_order": "spe_order_sources", "slot_order_ms": round(1e3 * t_ord, 1),
                       "sources_per_step_per_gpu": bps * 64, "groups_per_launch": lay["groups_per_launch"],
                       "parallelism": f"source blocks sharded over {world} GPU(s), no data-path collective"},
            "full_table_time_s": round(A / value, 3),
            "relax_rounds_per_step": round(it_total / max(1, steps), 1),
            "active_rounds_per_step": round(fr_total / max(1, steps), 1),
            "roofline": roof, "cpu_baseline": cpu,
        }
        line.update(extra)
        if cpu:
            line["speedup_vs_cpu_1core"] = round(value / cpu["value"], 1)
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
