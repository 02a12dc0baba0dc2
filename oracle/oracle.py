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
             want_ties: bool = False, want_dijkstra_time: bool = False):
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
        ties = np.zeros(1, np.int64)
        djs = np.zeros(1, np.float64)
        opts = _Opts(int(self_mode), int(tie_mode), int(force_sssp))
        r = lib().orc_rows(self.g, C.byref(opts), _ptr(src), ns, _ptr(tg), A,
                           _ptr(out["lat"]), _ptr(out["rel"]), _ptr(out["next"]), _ptr(out["hops"]),
                           _ptr(out["kind"]), _ptr(ties) if want_ties else None,
                           _ptr(djs) if want_dijkstra_time else None, int(nthreads))
        if r != 0:
            raise RuntimeError(f"orc_rows failed: {r}")
        out["ok"] = out["kind"] != KIND_FAIL
        out["double_ties"] = int(ties[0])
        out["dijkstra_seconds"] = float(djs[0])
        return out
