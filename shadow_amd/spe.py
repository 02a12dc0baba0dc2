"""Python mirror of the path-engine C ABI (include/spe.h) over ctypes.

This is plumbing for tests and the benchmark: every computation runs in
libspe.so's gfx950 kernels.  There is no CPU fallback -- if the library or a
gfx950 device is missing, construction raises SpeError.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional

import numpy as np

from .graphs import Topology

_HERE = os.path.dirname(os.path.abspath(__file__))
# SPE_LIB: an alternative build of the library (e.g. a -DSPE_DIAGNOSTICS build for ablations)
LIB_PATH = os.environ.get("SPE_LIB") or os.path.join(_HERE, "libspe.so")

SPE_OK = 0
SPE_SELF_ROW = 0
SPE_SELF_RULE = 1
SPE_ENGINE_AUTO, SPE_ENGINE_BATCH, SPE_ENGINE_LDS, SPE_ENGINE_FW = 0, 1, 2, 3
SPE_GATHER_AUTO, SPE_GATHER_RCCL, SPE_GATHER_PEER = 0, 1, 2
SPE_RELAX_AUTO, SPE_RELAX_REGISTER, SPE_RELAX_LDS_RING = 0, 1, 2
SPE_EUNSUPPORTED = -4
WAVE = 64

# Test / experiment hooks of this mirror (libspe itself reads no environment):
#   SPE_ENGINE=1|2|3   engine for tables that leave it AUTO (falls back to batch when
#                      the graph does not fit the asked engine)
#   SPE_LANES=64|128, SPE_RELAX=1|2, SPE_INFL=<rows per trip>, SPE_OCC=<waves/SIMD>, SPE_NO_CONTRACT=1,
#   SPE_EXACT_SOURCES=1 (every pendant source on its own lane: bit-exact path-order latencies),
#   SPE_DELTA=<ms>, SPE_NO_OVERLAP=1, SPE_TRACE=1   batch-engine tuning (spe_table_opts)
#   SPE_NO_PRUNE=1     graphs keep their pendant vertices (spe_graph_desc.keep_pendants)


def _env_int(name: str, default: int = 0) -> int:
    v = os.environ.get(name)
    return int(v) if v not in (None, "") else default


class SpeError(RuntimeError):
    pass


class _Sized(C.Structure):
    """A spe.h struct that starts with struct_size (the ABI guard): set on creation."""

    def __init__(self, *args, **kw):
        super().__init__(C.sizeof(type(self)), *args, **kw)


class GraphDesc(_Sized):
    _fields_ = [("struct_size", C.c_uint32), ("n_vertices", C.c_int32), ("n_edges", C.c_int64),
                ("edge_source", C.c_void_p), ("edge_target", C.c_void_p),
                ("edge_latency", C.c_void_p), ("edge_packetloss", C.c_void_p),
                ("vertex_packetloss", C.c_void_p), ("directed", C.c_int32), ("prefer_direct", C.c_int32),
                ("keep_pendants", C.c_int32)]


class GraphInfo(_Sized):
    _fields_ = [("struct_size", C.c_uint32), ("n_vertices", C.c_int32), ("n_edges", C.c_int64), ("n_relax_entries", C.c_int64),
                ("directed", C.c_int32), ("prefer_direct", C.c_int32), ("complete", C.c_int32),
                ("parallel_latency_differs", C.c_int32), ("weight_floor_ok", C.c_int32), ("device", C.c_int32),
                ("n_relax_vertices", C.c_int32), ("sums_exact", C.c_int32),
                ("shared_rows_exact", C.c_int32)]


class TableOpts(_Sized):
    _fields_ = [("struct_size", C.c_uint32), ("self_mode", C.c_int32), ("force_sssp", C.c_int32), ("groups_per_launch", C.c_int32),
                ("block_begin", C.c_int32), ("block_end", C.c_int32),
                ("ext_latrel", C.c_void_p),
                ("ext_next_hop", C.c_void_p), ("ext_hops", C.c_void_p), ("ext_filled", C.c_int32),
                ("owner_rank", C.c_void_p), ("engine", C.c_int32), ("lanes_per_group", C.c_int32),
                ("want_aux", C.c_int32), ("devices", C.c_void_p), ("n_devices", C.c_int32),
                ("gather", C.c_int32), ("relax_kernel", C.c_int32), ("rows_in_flight", C.c_int32),
                ("waves_per_simd", C.c_int32), ("no_overlap", C.c_int32), ("delta_ms", C.c_double),
                ("trace", C.c_int32), ("shared_fraction", C.c_double), ("gather_gbps", C.c_double),
                ("build_seconds_hint", C.c_double), ("no_contract", C.c_int32), ("exact_sources", C.c_int32)]


class TableLayout(_Sized):
    _fields_ = [("struct_size", C.c_uint32), ("n_attached", C.c_int32), ("block_begin", C.c_int32), ("block_end", C.c_int32),
                ("elems", C.c_int64), ("latrel", C.c_void_p),
                ("next_hop", C.c_void_p), ("hops", C.c_void_p), ("groups_per_launch", C.c_int32),
                ("engine", C.c_int32), ("n_devices", C.c_int32), ("device", C.c_int32),
                ("lanes_per_group", C.c_int32), ("relax_kernel", C.c_int32), ("contracted_vertices", C.c_int32),
                ("shared_sources", C.c_int32), ("host_reads", C.c_int32),
                ("host_prefault", C.c_int32), ("reserved0", C.c_int32), ("host_prefault_s", C.c_double)]


class Entry(C.Structure):
    _fields_ = [("latency", C.c_double), ("reliability", C.c_double), ("next_hop", C.c_int32),
                ("hops", C.c_int32)]


KERNELS = ["init", "seed", "heavy", "relax", "rows", "direct", "lds", "fw", "routes"]


class CheckReport(C.Structure):
    _fields_ = [("pairs", C.c_int64), ("unroutable", C.c_int64), ("bad_values", C.c_int64),
                ("next_not_adjacent", C.c_int64), ("hop_checked", C.c_int64), ("hop_mismatch", C.c_int64),
                ("sym_checked", C.c_int64), ("sym_mismatch", C.c_int64), ("max_sym_rel_err", C.c_double),
                ("first_bad_s", C.c_int32), ("first_bad_t", C.c_int32)]


class CompareReport(_Sized):
    _fields_ = [("struct_size", C.c_uint32), ("pairs", C.c_int64), ("routable", C.c_int64),
                ("route_mismatch", C.c_int64), ("latency_differs", C.c_int64), ("reliability_differs", C.c_int64),
                ("beyond_tolerance", C.c_int64), ("delivery_flips", C.c_int64),
                ("max_latency_rel_err", C.c_double), ("max_reliability_rel_err", C.c_double),
                ("first_bad_s", C.c_int32), ("first_bad_t", C.c_int32)]


class KernelProfile(C.Structure):
    _fields_ = [("ms", C.c_double * 9), ("launches", C.c_int64 * 9)]


class BuildStats(_Sized):
    _fields_ = [("struct_size", C.c_uint32), ("iterations", C.c_int64), ("active_rounds", C.c_int64), ("launches", C.c_int64),
                ("seconds", C.c_double), ("gather_seconds", C.c_double), ("n_devices", C.c_int32),
                ("gather", C.c_int32), ("shared_blocks", C.c_int32), ("local_blocks", C.c_int32),
                ("build_wait_seconds", C.c_double), ("relaxed_lanes", C.c_int64), ("fallback_blocks", C.c_int32),
                ("derived_sources", C.c_int64)]


# every symbol include/spe.h declares (tests/test_abi.py checks the export table)
EXPORTS = ["spe_last_error", "spe_device_count", "spe_graph_create", "spe_graph_info_get", "spe_graph_free",
           "spe_order_sources",
           "spe_table_create", "spe_table_build", "spe_table_build_blocks", "spe_table_build_blocks_into",
           "spe_table_profile_enable",
           "spe_table_profile_get", "spe_table_build_stats", "spe_table_layout_get",
           "spe_table_get", "spe_table_download", "spe_lookup_batch", "spe_table_min_latency",
           "spe_table_key", "spe_table_save", "spe_table_load", "spe_table_free",
           "spe_graph_set_edge_aux", "spe_table_download_aux", "spe_fw_apsp", "spe_fw_closure", "spe_graph_self_path",
           "spe_graph_adjacent", "spe_device_shares", "spe_graph_edge", "spe_table_source_tree",
           "spe_device_split", "spe_lookup_batch_replica", "spe_table_replica_device", "spe_table_check",
           "spe_lookup_batch_host", "spe_table_compare", "spe_table_get_latrel",
           "spe_table_get_row_latrel"]

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise SpeError(f"{LIB_PATH} missing: run __graft_entry__.build() (no CPU fallback exists)")
        # One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64 (soname
        # libamdhip64.so.7, NEEDED as "libamdhip64.so" via $ORIGIN).  Loading torch first
        # lets libspe's libamdhip64.so.7 dependency bind to that same copy; the other order
        # would map two runtimes and torch would see no GPU.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = C.CDLL(LIB_PATH)
        P = C.c_void_p
        L.spe_last_error.restype = C.c_char_p
        L.spe_device_count.argtypes = [P]
        L.spe_graph_create.argtypes = [P, C.c_int32, P]
        L.spe_graph_info_get.argtypes = [P, P]
        L.spe_order_sources.argtypes = [P, P, C.c_int32, P]
        L.spe_graph_free.argtypes = [P]
        L.spe_graph_free.restype = None
        L.spe_table_create.argtypes = [P, P, C.c_int32, P, P]
        L.spe_table_build.argtypes = [P, P]
        L.spe_table_build_blocks.argtypes = [P, C.c_int32, C.c_int32, P]
        L.spe_table_build_blocks_into.argtypes = [P, C.c_int32, C.c_int32, P, P, P, P]
        L.spe_table_profile_enable.argtypes = [P, C.c_int32]
        L.spe_table_profile_get.argtypes = [P, P]
        L.spe_table_build_stats.argtypes = [P, P]
        L.spe_table_layout_get.argtypes = [P, P]
        L.spe_table_get.argtypes = [P, C.c_int32, C.c_int32, P]
        L.spe_table_get_latrel.argtypes = [P, C.c_int32, C.c_int32, P, P]
        L.spe_table_download.argtypes = [P, C.c_int32, C.c_int32, P, P, P, P]
        L.spe_lookup_batch.argtypes = [P, P, C.c_int64, P, P, P, P]
        L.spe_lookup_batch_replica.argtypes = [P, C.c_int32, P, C.c_int64, P, P, P, P]
        L.spe_table_replica_device.argtypes = [P, C.c_int32, P]
        L.spe_lookup_batch_host.argtypes = [P, P, C.c_int64, P, P, P]
        L.spe_table_check.argtypes = [P, P]
        L.spe_table_compare.argtypes = [P, P, C.c_double, P]
        L.spe_device_split.argtypes = [C.c_int32, C.c_int32, C.c_double, P, P, P]
        L.spe_table_min_latency.argtypes = [P, P]
        L.spe_table_key.argtypes = [P, P]
        L.spe_table_save.argtypes = [P, C.c_char_p]
        L.spe_table_load.argtypes = [P, C.c_char_p]
        L.spe_graph_set_edge_aux.argtypes = [P, P]
        L.spe_table_download_aux.argtypes = [P, C.c_int32, C.c_int32, P]
        L.spe_fw_apsp.argtypes = [P, P, C.c_int64, P, P, P]
        L.spe_fw_closure.argtypes = [P, P, P, P, C.c_int64, P, P]
        L.spe_table_free.argtypes = [P]
        L.spe_table_free.restype = None
        L.spe_device_shares.argtypes = [C.c_int32, C.c_int32, P, P]
        L.spe_graph_self_path.argtypes = [P, C.c_int32, P]
        L.spe_graph_adjacent.argtypes = [P, C.c_int32, C.c_int32, P]
        L.spe_graph_edge.argtypes = [P, C.c_int32, C.c_int32, P, P]
        L.spe_table_source_tree.argtypes = [P, C.c_int32, P]
        _lib = L
    return _lib


def _check(rc: int, what: str):
    if rc != SPE_OK:
        msg = lib().spe_last_error().decode(errors="replace")
        raise SpeError(f"{what} failed ({rc}): {msg}")


def _p(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def device_shares(n_attached: int, n_devices: int):
    """spe_device_shares: the [begin, end) 64-source block range of each device of
    a multi-device table (host-only)."""
    b0 = np.empty(n_devices, np.int32)
    b1 = np.empty(n_devices, np.int32)
    _check(lib().spe_device_shares(int(n_attached), int(n_devices), _p(b0), _p(b1)), "spe_device_shares")
    return list(zip(b0.tolist(), b1.tolist()))


def device_split(n_attached: int, n_devices: int, shared_fraction: float):
    """spe_device_split: ([(begin, end)] shares of the sharded blocks, first block of
    the local remainder every device builds) (host-only)."""
    b0 = np.empty(n_devices, np.int32)
    b1 = np.empty(n_devices, np.int32)
    lb = C.c_int32(0)
    _check(lib().spe_device_split(int(n_attached), int(n_devices), float(shared_fraction), _p(b0), _p(b1),
                                  C.byref(lb)), "spe_device_split")
    return list(zip(b0.tolist(), b1.tolist())), int(lb.value)


def device_count() -> int:
    c = C.c_int32(0)
    lib().spe_device_count(C.byref(c))
    return int(c.value)


class Graph:
    """spe_graph: the topology uploaded to one device (topology_new's role)."""

    def __init__(self, top: Topology, device: int = 0, keep_pendants: Optional[bool] = None):
        self.top = top
        if keep_pendants is None:
            keep_pendants = _env_int("SPE_NO_PRUNE") != 0
        keep = [np.ascontiguousarray(top.esrc, np.int32), np.ascontiguousarray(top.edst, np.int32),
                np.ascontiguousarray(top.elat, np.float64), np.ascontiguousarray(top.eloss, np.float64),
                np.ascontiguousarray(top.vloss, np.float64)]
        d = GraphDesc(int(top.n), int(keep[0].shape[0]), _p(keep[0]), _p(keep[1]), _p(keep[2]), _p(keep[3]),
                      _p(keep[4]), int(bool(top.directed)), int(bool(top.prefer_direct)), int(bool(keep_pendants)))
        h = C.c_void_p()
        _check(lib().spe_graph_create(C.byref(d), int(device), C.byref(h)), "spe_graph_create")
        self.h = h
        self.device = device

    def set_edge_aux(self, edge_aux) -> None:
        """Per-edge auxiliary attribute (GraphML jitter) folded by want_aux tables."""
        self._aux = np.ascontiguousarray(edge_aux, np.float64)
        if self._aux.shape != (self.top.m,):
            raise ValueError("edge_aux needs one value per edge")
        _check(lib().spe_graph_set_edge_aux(self.h, _p(self._aux)), "spe_graph_set_edge_aux")

    def fw_apsp(self, d_dist: int, ld: int, d_next: int = 0, stream: int = 0) -> float:
        """Blocked min-plus Floyd-Warshall into caller device buffers; returns device seconds."""
        sec = C.c_double(0)
        _check(lib().spe_fw_apsp(self.h, C.c_void_p(d_dist), int(ld), C.c_void_p(d_next or None),
                                 C.c_void_p(stream or None), C.byref(sec)), "spe_fw_apsp")
        return float(sec.value)

    def fw_closure(self, d_dist: int, d_rel: int, d_next: int, ld: int, stream: int = 0) -> float:
        """Blocked min-plus FW carrying (latency, reliability, first hop) into caller
        device buffers of ld x ld elements; returns device seconds of the closure."""
        sec = C.c_double(0)
        _check(lib().spe_fw_closure(self.h, C.c_void_p(d_dist), C.c_void_p(d_rel), C.c_void_p(d_next), int(ld),
                                    C.c_void_p(stream or None), C.byref(sec)), "spe_fw_closure")
        return float(sec.value)

    def edge(self, u: int, v: int):
        """spe_graph_edge: (latency, reliability) of the get_eid edge u -> v."""
        w, a = C.c_double(0), C.c_double(0)
        _check(lib().spe_graph_edge(self.h, int(u), int(v), C.byref(w), C.byref(a)), "spe_graph_edge")
        return float(w.value), float(a.value)

    def order_sources(self, attached) -> np.ndarray:
        """spe_order_sources: a slot order clustering sources by relaxation anchor."""
        a = np.ascontiguousarray(attached, dtype=np.int32)
        out = np.empty_like(a)
        _check(lib().spe_order_sources(self.h, a.ctypes.data, int(a.shape[0]), out.ctypes.data), "spe_order_sources")
        return out

    def info(self) -> dict:
        i = GraphInfo()
        _check(lib().spe_graph_info_get(self.h, C.byref(i)), "spe_graph_info_get")
        return {f: getattr(i, f) for f, _ in GraphInfo._fields_}

    def close(self):
        if getattr(self, "h", None):
            lib().spe_graph_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except (TypeError, AttributeError):   # interpreter shutdown: module globals already cleared
            pass


class PathTable:
    """spe_table: the per-(source, target) path table for attached vertices."""

    def __init__(self, graph: Graph, attached, self_mode: int = SPE_SELF_ROW, force_sssp: bool = False,
                 groups: int = 0, blocks=None, ext=None, ext_filled: bool = False, lanes: int = 0,
                 owner_order=None, engine: int = 0, want_aux: bool = False, devices=None,
                 gather: int = SPE_GATHER_AUTO, relax_kernel: int = 0, rows_in_flight: int = 0,
                 waves_per_simd: int = 0, no_overlap: Optional[bool] = None, delta_ms: Optional[float] = None,
                 shared_fraction: float = 0.0, gather_gbps: float = 0.0, build_seconds_hint: float = 0.0,
                 no_contract: Optional[bool] = None, exact_sources: Optional[bool] = None):
        self.graph = graph
        self.attached = np.ascontiguousarray(attached, np.int32)
        self.A = int(self.attached.shape[0])
        o = TableOpts()
        o.self_mode = int(self_mode)
        o.force_sssp = int(bool(force_sssp))
        o.groups_per_launch = int(groups)
        o.lanes_per_group = int(lanes) or _env_int("SPE_LANES")
        o.engine = int(engine)
        o.want_aux = int(bool(want_aux))
        o.relax_kernel = int(relax_kernel) or _env_int("SPE_RELAX")
        o.rows_in_flight = int(rows_in_flight) or _env_int("SPE_INFL")
        o.waves_per_simd = int(waves_per_simd) or _env_int("SPE_OCC")
        o.no_overlap = int(bool(no_overlap if no_overlap is not None else _env_int("SPE_NO_OVERLAP")))
        o.delta_ms = float(delta_ms if delta_ms is not None else (os.environ.get("SPE_DELTA") or 0.0))
        o.trace = _env_int("SPE_TRACE")
        o.no_contract = int(bool(no_contract if no_contract is not None else _env_int("SPE_NO_CONTRACT")))
        o.exact_sources = int(bool(exact_sources if exact_sources is not None else _env_int("SPE_EXACT_SOURCES")))
        env_engine = engine == SPE_ENGINE_AUTO and not want_aux and _env_int("SPE_ENGINE") != 0
        if env_engine:
            o.engine = _env_int("SPE_ENGINE")
        if owner_order is not None:   # source-run order (slots) -> rank of each slot
            self._rank = np.empty(self.A, np.int32)
            self._rank[np.asarray(owner_order, np.int64)] = np.arange(self.A, dtype=np.int32)
            o.owner_rank = self._rank.ctypes.data
        if blocks is not None:
            o.block_begin, o.block_end = int(blocks[0]), int(blocks[1])
        if devices is not None:   # one process, several devices: shares + all-gather (spe_multi.cpp)
            self._devs = np.ascontiguousarray(devices, np.int32)
            o.devices = self._devs.ctypes.data
            o.n_devices = int(self._devs.shape[0])
            o.gather = int(gather)
            o.shared_fraction = float(shared_fraction)
            o.gather_gbps = float(gather_gbps)
            o.build_seconds_hint = float(build_seconds_hint)
        if ext is not None:  # three device pointers (ints): latrel (2 x f64), next_hop (i32), hops (u16)
            o.ext_latrel, o.ext_next_hop, o.ext_hops = [int(x) for x in ext]
            o.ext_filled = int(bool(ext_filled))
        h = C.c_void_p()
        rc = lib().spe_table_create(graph.h, _p(self.attached), self.A, C.byref(o), C.byref(h))
        if rc == SPE_EUNSUPPORTED and env_engine and o.engine != SPE_ENGINE_BATCH:
            o.engine = SPE_ENGINE_BATCH   # SPE_ENGINE asked for an engine the graph does not fit
            rc = lib().spe_table_create(graph.h, _p(self.attached), self.A, C.byref(o), C.byref(h))
        _check(rc, "spe_table_create")
        self.h = h

    @property
    def nblocks(self) -> int:
        return (self.A + WAVE - 1) // WAVE

    def build(self, stream: Optional[int] = None) -> dict:
        _check(lib().spe_table_build(self.h, C.c_void_p(stream) if stream else None), "spe_table_build")
        return self.stats()

    def build_blocks(self, b0: int, b1: int, stream: Optional[int] = None) -> dict:
        _check(lib().spe_table_build_blocks(self.h, int(b0), int(b1), C.c_void_p(stream) if stream else None),
               "spe_table_build_blocks")
        return self.stats()

    def build_blocks_into(self, b0: int, b1: int, latrel: int, next_hop: int, hops: int,
                          stream: Optional[int] = None) -> dict:
        """spe_table_build_blocks_into: rows of blocks [b0, b1) into caller device
        buffers (pointers to where block b0's elements go)."""
        _check(lib().spe_table_build_blocks_into(self.h, int(b0), int(b1), C.c_void_p(latrel), C.c_void_p(next_hop),
                                                 C.c_void_p(hops), C.c_void_p(stream) if stream else None),
               "spe_table_build_blocks_into")
        return self.stats()

    def profile(self, enable: bool = True):
        _check(lib().spe_table_profile_enable(self.h, int(bool(enable))), "spe_table_profile_enable")

    def kernel_profile(self) -> dict:
        k = KernelProfile()
        _check(lib().spe_table_profile_get(self.h, C.byref(k)), "spe_table_profile_get")
        return {name: {"ms": k.ms[i], "launches": k.launches[i]} for i, name in enumerate(KERNELS)}

    def stats(self) -> dict:
        s = BuildStats()
        _check(lib().spe_table_build_stats(self.h, C.byref(s)), "spe_table_build_stats")
        return {f: getattr(s, f) for f, _ in BuildStats._fields_}

    def layout(self) -> dict:
        l = TableLayout()
        _check(lib().spe_table_layout_get(self.h, C.byref(l)), "spe_table_layout_get")
        return {f: getattr(l, f) for f, _ in TableLayout._fields_}

    def get(self, s_slot: int, t_slot: int) -> dict:
        e = Entry()
        _check(lib().spe_table_get(self.h, int(s_slot), int(t_slot), C.byref(e)), "spe_table_get")
        return {"latency": e.latency, "reliability": e.reliability, "next_hop": e.next_hop, "hops": e.hops}

    def get_latrel(self, s_slot: int, t_slot: int):
        lat, rel = C.c_double(), C.c_double()
        _check(lib().spe_table_get_latrel(self.h, int(s_slot), int(t_slot), C.byref(lat), C.byref(rel)),
               "spe_table_get_latrel")
        return lat.value, rel.value

    def download(self, row_begin: int = 0, row_end: Optional[int] = None,
                 fields=("lat", "rel", "next", "hops")) -> dict:
        row_end = self.A if row_end is None else row_end
        nr = row_end - row_begin
        types = {"lat": np.float64, "rel": np.float64, "next": np.int32, "hops": np.int32}
        out = {f: np.empty((nr, self.A), types[f]) for f in fields}
        _check(lib().spe_table_download(self.h, int(row_begin), int(row_end), _p(out.get("lat")), _p(out.get("rel")),
                                        _p(out.get("next")), _p(out.get("hops"))), "spe_table_download")
        if "lat" in out:
            out["ok"] = out["lat"] > -1.0
        return out

    def source_tree(self, s_slot: int) -> np.ndarray:
        """spe_table_source_tree: parent[v] on the row of source slot s_slot (-1: root / unreachable)."""
        out = np.empty(self.graph.top.n, np.int32)
        _check(lib().spe_table_source_tree(self.h, int(s_slot), _p(out)), "spe_table_source_tree")
        return out

    def download_aux(self, row_begin: int = 0, row_end: Optional[int] = None) -> np.ndarray:
        row_end = self.A if row_end is None else row_end
        out = np.empty((row_end - row_begin, self.A), np.float64)
        _check(lib().spe_table_download_aux(self.h, int(row_begin), int(row_end), _p(out)), "spe_table_download_aux")
        return out

    def lookup_batch(self, d_pairs: int, q: int, d_lat: int, d_rel: int, d_ok: int, stream: Optional[int] = None):
        _check(lib().spe_lookup_batch(self.h, C.c_void_p(d_pairs), int(q), C.c_void_p(d_lat), C.c_void_p(d_rel),
                                      C.c_void_p(d_ok), C.c_void_p(stream) if stream else None),
               "spe_lookup_batch")

    def lookup_batch_replica(self, replica: int, d_pairs: int, q: int, d_lat: int, d_rel: int, d_ok: int,
                             stream: Optional[int] = None):
        """spe_lookup_batch_replica: queries on replica `replica`'s device, answered from its records."""
        _check(lib().spe_lookup_batch_replica(self.h, int(replica), C.c_void_p(d_pairs), int(q), C.c_void_p(d_lat),
                                              C.c_void_p(d_rel), C.c_void_p(d_ok),
                                              C.c_void_p(stream) if stream else None), "spe_lookup_batch_replica")

    def lookup_batch_host(self, pairs):
        """spe_lookup_batch_host: (q, 2) int32 slot pairs (host) -> (lat, rel, ok) host arrays."""
        pairs = np.ascontiguousarray(pairs, np.int32)
        q = int(pairs.shape[0])
        lat = np.empty(q, np.float64)
        rel = np.empty(q, np.float64)
        ok = np.empty(q, np.uint8)
        _check(lib().spe_lookup_batch_host(self.h, _p(pairs), q, _p(lat), _p(rel), _p(ok)), "spe_lookup_batch_host")
        return lat, rel, ok

    def check(self) -> dict:
        """spe_table_check: whole-table invariants counted on the device."""
        r = CheckReport()
        _check(lib().spe_table_check(self.h, C.byref(r)), "spe_table_check")
        return {f: getattr(r, f) for f, _ in CheckReport._fields_}

    def compare(self, other: "PathTable", rel_tol: float = 1e-12) -> dict:
        """spe_table_compare(self, other): entry-by-entry differences on the device
        (route mismatches, latency / reliability bit differences, entries beyond
        rel_tol relative to `other`, ceil(latency * 1e6) delivery-time flips)."""
        r = CompareReport()
        _check(lib().spe_table_compare(self.h, other.h, float(rel_tol), C.byref(r)), "spe_table_compare")
        return {f: getattr(r, f) for f, _ in CompareReport._fields_ if f != "struct_size"}

    def replica_device(self, replica: int) -> int:
        d = C.c_int32(0)
        _check(lib().spe_table_replica_device(self.h, int(replica), C.byref(d)), "spe_table_replica_device")
        return int(d.value)

    def key(self) -> int:
        k = C.c_uint64(0)
        _check(lib().spe_table_key(self.h, C.byref(k)), "spe_table_key")
        return int(k.value)

    def save(self, path: str):
        _check(lib().spe_table_save(self.h, os.fsencode(path)), "spe_table_save")

    def load(self, path: str):
        _check(lib().spe_table_load(self.h, os.fsencode(path)), "spe_table_load")

    def min_latency(self) -> float:
        v = C.c_double(0)
        _check(lib().spe_table_min_latency(self.h, C.byref(v)), "spe_table_min_latency")
        return float(v.value)

    def close(self):
        if getattr(self, "h", None):
            lib().spe_table_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except (TypeError, AttributeError):   # interpreter shutdown: module globals already cleared
            pass
