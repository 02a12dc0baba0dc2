"""ctypes front-end for the CPU oracle (oracle/oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg -- never by shadow_amd/.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")
_lib = None

KIND_FAIL, KIND_DIRECT, KIND_SSSP, KIND_SELF = 0, 1, 2, 3


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        P = C.c_void_p
        L.orc_graph_new.restype = P
        L.orc_graph_new.argtypes = [C.c_int32, C.c_int64, P, P, P, P, P, C.c_int32, C.c_int32]
        L.orc_graph_free.argtypes = [P]
        L.orc_is_complete.argtypes = [P]
        L.orc_is_complete.restype = C.c_int32
        L.orc_get_eid.argtypes = [P, C.c_int32, C.c_int32]
        L.orc_get_eid.restype = C.c_int64
        L.orc_dijkstra.argtypes = [P, C.c_int32, P, C.c_int32, C.c_int32, P, P, P]
        L.orc_dijkstra.restype = C.c_int32
        L.orc_rows.argtypes = [P, P, P, C.c_int32, P, C.c_int32, P, P, P, P, P, P, P, C.c_int32]
        L.orc_rows.restype = C.c_int32
        L.orc_rows2.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_int32] + [C.c_void_p] * 8 \
            + [C.c_int32]
        L.orc_rows2.restype = C.c_int32
        _lib = L
    return _lib


class _Opts(C.Structure):
    _fields_ = [("self_mode", C.c_int32), ("tie_mode", C.c_int32), ("force_sssp", C.c_int32)]


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


class Oracle:
    """igraph-faithful Dijkstra + Shadow row rules on one topology."""

    def __init__(self, top):
        L = lib()
        self.top = top
        self._keep = [np.ascontiguousarray(top.esrc, dtype=np.int32),
                      np.ascontiguousarray(top.edst, dtype=np.int32),
                      np.ascontiguousarray(top.elat, dtype=np.float64),
                      np.ascontiguousarray(top.eloss, dtype=np.float64),
                      np.ascontiguousarray(top.vloss, dtype=np.float64)]
        k = self._keep
        self.g = L.orc_graph_new(int(top.n), int(k[0].shape[0]), _ptr(k[0]), _ptr(k[1]), _ptr(k[2]),
                                 _ptr(k[3]), _ptr(k[4]), int(bool(top.directed)),
                                 int(bool(top.prefer_direct)))
        if not self.g:
            raise RuntimeError("orc_graph_new failed")

    def __del__(self):
        if getattr(self, "g", None):
            lib().orc_graph_free(self.g)
            self.g = None

    @property
    def complete(self) -> bool:
        return bool(lib().orc_is_complete(self.g))

    def get_eid(self, a: int, b: int) -> int:
        return int(lib().orc_get_eid(self.g, int(a), int(b)))

    def dijkstra(self, src: int, targets=None, stop_early: bool = False):
        n = self.top.n
        tg = np.arange(n, dtype=np.int32) if targets is None else np.ascontiguousarray(targets, np.int32)
        dist = np.empty(n, np.float64)
        peid = np.empty(n, np.int64)
        rank = np.empty(n, np.int32)
        lib().orc_dijkstra(self.g, int(src), _ptr(tg), int(tg.shape[0]), int(stop_early),
                           _ptr(dist), _ptr(peid), _ptr(rank))
        return dist, peid, rank

    def rows(self, sources, targets, self_mode: int = 0, tie_mode: int = 0, nthreads: int = 1, force_sssp: bool = False,
             want_ties: bool = False, want_dijkstra_time: bool = False, want_prev: bool = False):
        src = np.ascontiguousarray(sources, dtype=np.int32)
        tg = np.ascontiguousarray(targets, dtype=np.int32)
        ns, A = src.shape[0], tg.shape[0]
        out = {
            "lat": np.empty((ns, A), np.float64),
            "rel": np.empty((ns, A), np.float64),
            "next": np.empty((ns, A), np.int32),
            "hops": np.empty((ns, A), np.int32),
            "kind": np.empty((ns, A), np.uint8),
        }
        if want_prev:
            out["prev"] = np.empty((ns, A), np.int32)
        ties = np.zeros(1, np.int64)
        djs = np.zeros(1, np.float64)
        opts = _Opts(int(self_mode), int(tie_mode), int(force_sssp))
        r = lib().orc_rows2(self.g, C.byref(opts), _ptr(src), ns, _ptr(tg), A,
                            _ptr(out["lat"]), _ptr(out["rel"]), _ptr(out["next"]), _ptr(out["hops"]),
                            _ptr(out["kind"]), _ptr(out["prev"]) if want_prev else None,
                            _ptr(ties) if want_ties else None,
                            _ptr(djs) if want_dijkstra_time else None, int(nthreads))
        if r != 0:
            raise RuntimeError(f"orc_rows failed: {r}")
        out["ok"] = out["kind"] != KIND_FAIL
        out["double_ties"] = int(ties[0])
        out["dijkstra_seconds"] = float(djs[0])
        return out

    def rows_owner(self, attached, order, self_mode: int = 0, tie_mode: int = 0):
        """The reference's answers when every attached source has run its Dijkstra
        in `order` (slot indices), replaying the path cache: a computed path (s, t)
        is stored only if neither (s, t) nor (t, s) is cached yet
        (_topology_shouldStorePath, shd-topology.c:1292-1321); DIRECT pairs are
        never stored from a Dijkstra row (:1305-1316) and are recomputed on lookup;
        a lookup tries (s, t) then (t, s) whatever the direction (:1970-1973,
        :2017-2020).  Pure-Python cache simulation: small graphs only.
        Next hop of an entry answered by the reverse path: the vertex before s on
        the owner's path t -> s when undirected, -1 when directed (the reference's
        Path has no next hop; ours is the first hop of the path it returns)."""
        A_ = np.ascontiguousarray(attached, np.int32)
        r = self.rows(A_, A_, self_mode=self_mode, tie_mode=tie_mode, want_prev=True)
        A = A_.shape[0]
        cache = {}
        for s in order:
            for t in range(A):
                if r["kind"][s, t] != KIND_SSSP or s == t:
                    continue
                if (s, t) in cache or (t, s) in cache:
                    continue
                cache[(s, t)] = s
        out = {k: r[k].copy() for k in ("lat", "rel", "next", "hops", "kind")}
        for s in range(A):
            for t in range(A):
                if s == t or r["kind"][s, t] in (KIND_DIRECT,):
                    continue
                if (s, t) in cache:
                    continue
                if (t, s) in cache:
                    out["lat"][s, t] = r["lat"][t, s]
                    out["rel"][s, t] = r["rel"][t, s]
                    out["hops"][s, t] = r["hops"][t, s]
                    out["next"][s, t] = -1 if self.top.directed else r["prev"][t, s]
                    out["kind"][s, t] = KIND_SSSP
                else:   # neither direction stored: the lookup fails
                    out["lat"][s, t] = out["rel"][s, t] = -1.0
                    out["next"][s, t] = -1
                    out["hops"][s, t] = 0
                    out["kind"][s, t] = KIND_FAIL
        out["ok"] = out["kind"] != KIND_FAIL
        return out


class LookupCache:
    """CPU restatement of the per-packet lookup (IP -> slot hash, two-level path
    cache; oracle.c orc_cache_*), for the C5 CPU baseline and its tests."""

    def __init__(self, ips, pairs, lat, rel):
        L = lib()
        L.orc_cache_new.restype = C.c_void_p
        L.orc_cache_new.argtypes = [C.c_int32, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p]
        L.orc_cache_free.argtypes = [C.c_void_p]
        L.orc_cache_lookup.restype = C.c_int64
        L.orc_cache_lookup.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p,
                                       C.c_void_p, C.c_int32]
        self._keep = [np.ascontiguousarray(ips, np.uint32), np.ascontiguousarray(pairs, np.int32),
                      np.ascontiguousarray(lat, np.float64), np.ascontiguousarray(rel, np.float64)]
        k = self._keep
        self.h = L.orc_cache_new(int(k[0].shape[0]), _ptr(k[0]), int(k[1].shape[0]), _ptr(k[1]), _ptr(k[2]),
                                 _ptr(k[3]))
        if not self.h:
            raise RuntimeError("orc_cache_new failed")

    def lookup(self, sip, dip, nthreads: int = 1):
        sip = np.ascontiguousarray(sip, np.uint32)
        dip = np.ascontiguousarray(dip, np.uint32)
        q = sip.shape[0]
        lat, rel, ok = np.empty(q), np.empty(q), np.empty(q, np.uint8)
        hits = lib().orc_cache_lookup(self.h, _ptr(sip), _ptr(dip), q, _ptr(lat), _ptr(rel), _ptr(ok), int(nthreads))
        return lat, rel, ok, int(hits)

    def __del__(self):
        if getattr(self, "h", None):
            try:
                lib().orc_cache_free(self.h)
            except (TypeError, AttributeError):
                pass
            self.h = None
