"""ctypes mirror of the drop-in topology API (include/shd_topology_spe.h,
libshdtopo.so) -- the same entry points, argument meanings and error
conventions as the reference's shd-topology.h; used by the tests."""
from __future__ import annotations

import ctypes as C
import os
import socket
import struct

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libshdtopo.so")
EXPORTS = ["topology_new", "topology_new_on_device", "topology_free", "topology_attach", "topology_detach",
           "topology_isRoutable", "topology_getLatency", "topology_getReliability",
           "topology_incrementPathPacketCounter", "topology_set_log_callback",
           "topology_set_min_latency_callback", "topology_seal", "topology_vertex_count",
           "topology_attached_vertex", "topology_path_packet_count", "topology_min_path_latency",
           "topology_getPathInfo", "topology_set_log_level", "topology_set_answer_mode",
           "topology_cached_path_count", "topology_check_graphml", "topology_getPathInfoBatch",
           "topology_incrementPathPacketCounterBatch"]
ANSWER_ROWS, ANSWER_REFERENCE = 0, 1

RANDOM_FN = C.CFUNCTYPE(C.c_double, C.c_void_p)
MINLAT_FN = C.CFUNCTYPE(None, C.c_double, C.c_void_p)
LOG_FN = C.CFUNCTYPE(None, C.c_int, C.c_char_p, C.c_void_p)
_lib = None


def lib():
    global _lib
    if _lib is None:
        from . import spe
        spe.lib()   # one HIP runtime per process (see spe.lib)
        L = C.CDLL(LIB_PATH)
        P, U = C.c_void_p, C.c_uint32
        L.topology_new.restype = P
        L.topology_new.argtypes = [C.c_char_p]
        L.topology_new_on_device.restype = P
        L.topology_new_on_device.argtypes = [C.c_char_p, C.c_int32]
        L.topology_free.argtypes = [P]
        L.topology_attach.argtypes = [P, U, RANDOM_FN, P, C.c_char_p, C.c_char_p, C.c_char_p, C.c_char_p,
                                      C.c_char_p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        L.topology_detach.argtypes = [P, U]
        for f in ("topology_getLatency", "topology_getReliability"):
            getattr(L, f).argtypes = [P, U, U]
            getattr(L, f).restype = C.c_double
        L.topology_isRoutable.argtypes = [P, U, U]
        L.topology_isRoutable.restype = C.c_int32
        L.topology_incrementPathPacketCounter.argtypes = [P, U, U]
        L.topology_getPathInfo.argtypes = [P, U, U, C.POINTER(C.c_double), C.POINTER(C.c_double)]
        L.topology_getPathInfo.restype = C.c_int32
        L.topology_set_log_callback.argtypes = [P, LOG_FN, P]
        L.topology_set_min_latency_callback.argtypes = [P, MINLAT_FN, P]
        L.topology_seal.argtypes = [P]
        L.topology_seal.restype = C.c_int32
        L.topology_vertex_count.argtypes = [P]
        L.topology_vertex_count.restype = C.c_int32
        L.topology_attached_vertex.argtypes = [P, U]
        L.topology_attached_vertex.restype = C.c_int32
        L.topology_path_packet_count.argtypes = [P, U, U]
        L.topology_path_packet_count.restype = C.c_uint64
        L.topology_min_path_latency.argtypes = [P]
        L.topology_min_path_latency.restype = C.c_double
        L.topology_set_log_level.argtypes = [P, C.c_int32]
        L.topology_set_answer_mode.argtypes = [P, C.c_int32]
        L.topology_set_answer_mode.restype = C.c_int32
        L.topology_check_graphml.argtypes = [C.c_char_p]
        L.topology_check_graphml.restype = C.c_int32
        L.topology_getPathInfoBatch.argtypes = [P, C.c_int64, P, P, P, P, P]
        L.topology_getPathInfoBatch.restype = C.c_int64
        L.topology_incrementPathPacketCounterBatch.argtypes = [P, C.c_int64, P, P]
        L.topology_cached_path_count.argtypes = [P]
        L.topology_cached_path_count.restype = C.c_int64
        _lib = L
    return _lib


def check_graphml(path: str) -> bool:
    """topology_check_graphml: would topology_new accept this file (no GPU needed)."""
    return bool(lib().topology_check_graphml(path.encode()))


def ip(s: str) -> int:
    """dotted quad -> in_addr_t value (network byte order, as address_toNetworkIP)."""
    return struct.unpack("=I", socket.inet_aton(s))[0]


class Topology:
    def __init__(self, graph_path: str, device: int = 0):
        self.h = lib().topology_new_on_device(graph_path.encode(), int(device))
        if not self.h:
            raise ValueError(f"topology_new failed for {graph_path}")
        self._keep = []

    def attach(self, address: int, rand=None, ip_hint=None, citycode=None, countrycode=None, geocode=None,
               type_hint=None):
        seq = list(rand) if rand is not None else [0.0]
        state = {"i": 0}

        def nxt(_ctx):
            v = seq[state["i"] % len(seq)]
            state["i"] += 1
            return v

        cb = RANDOM_FN(nxt)
        self._keep.append(cb)
        down, up = C.c_uint64(0), C.c_uint64(0)
        enc = lambda x: x.encode() if x else None
        lib().topology_attach(self.h, address, cb, None, enc(ip_hint), enc(citycode), enc(countrycode),
                              enc(geocode), enc(type_hint), C.byref(down), C.byref(up))
        return down.value, up.value

    def detach(self, address: int):
        lib().topology_detach(self.h, address)

    def latency(self, a: int, b: int) -> float:
        return lib().topology_getLatency(self.h, a, b)

    def reliability(self, a: int, b: int) -> float:
        return lib().topology_getReliability(self.h, a, b)

    def routable(self, a: int, b: int) -> bool:
        return bool(lib().topology_isRoutable(self.h, a, b))

    def path_info(self, a: int, b: int):
        """(routable, latency, reliability) in one lookup (topology_getPathInfo)."""
        lat, rel = C.c_double(0), C.c_double(0)
        ok = lib().topology_getPathInfo(self.h, a, b, C.byref(lat), C.byref(rel))
        return bool(ok), lat.value, rel.value

    def path_info_batch(self, src, dst, out=None):
        """topology_getPathInfoBatch: (routable u8, latency, reliability) arrays for
        address arrays src / dst (in_addr_t values).  `out` = (ok, lat, rel) arrays
        of the batch's length to fill instead of fresh ones (a worker reuses its
        buffers every round; fresh 20M-entry arrays cost their page faults)."""
        import numpy as np
        s = np.ascontiguousarray(src, np.uint32)
        d = np.ascontiguousarray(dst, np.uint32)
        if s.ndim != 1 or s.shape != d.shape:
            raise ValueError("path_info_batch: src and dst must be 1-D arrays of equal length")
        n = int(s.shape[0])
        if out is None:
            lat = np.empty(n, np.float64)
            rel = np.empty(n, np.float64)
            ok = np.empty(n, np.uint8)
        else:
            ok, lat, rel = out
            for a, dt in ((ok, np.uint8), (lat, np.float64), (rel, np.float64)):
                if a.dtype != dt or a.shape != (n,) or not a.flags.c_contiguous or not a.flags.writeable:
                    raise ValueError("path_info_batch: out = (ok u8, lat f64, rel f64) contiguous arrays of the batch's length")
        r = lib().topology_getPathInfoBatch(self.h, n, s.ctypes.data, d.ctypes.data, lat.ctypes.data,
                                            rel.ctypes.data, ok.ctypes.data)
        if r < 0:
            raise ValueError("topology_getPathInfoBatch: bad arguments")
        return ok, lat, rel

    def count_packets_batch(self, src, dst):
        import numpy as np
        s = np.ascontiguousarray(src, np.uint32)
        d = np.ascontiguousarray(dst, np.uint32)
        if s.ndim != 1 or s.shape != d.shape:
            raise ValueError("count_packets_batch: src and dst must be 1-D arrays of equal length")
        lib().topology_incrementPathPacketCounterBatch(self.h, int(s.shape[0]), s.ctypes.data, d.ctypes.data)

    def count_packet(self, a: int, b: int):
        lib().topology_incrementPathPacketCounter(self.h, a, b)

    def packets(self, a: int, b: int) -> int:
        return int(lib().topology_path_packet_count(self.h, a, b))

    def vertex_of(self, a: int) -> int:
        return int(lib().topology_attached_vertex(self.h, a))

    def min_latency(self) -> float:
        return float(lib().topology_min_path_latency(self.h))

    def seal(self) -> int:
        return int(lib().topology_seal(self.h))

    def set_answer_mode(self, mode: int):
        assert lib().topology_set_answer_mode(self.h, int(mode)) == 0

    def cached_paths(self) -> int:
        return int(lib().topology_cached_path_count(self.h))

    def capture_logs(self, level: int = 4):
        """Route the topology's log lines (level <= `level`) into self.logs."""
        self.logs = []

        def cb(lvl, text, _ctx):
            self.logs.append((lvl, text.decode()))

        self._log_cb = LOG_FN(cb)
        lib().topology_set_log_callback(self.h, self._log_cb, None)
        lib().topology_set_log_level(self.h, int(level))

    def close(self):
        if getattr(self, "h", None):
            lib().topology_free(self.h)
            self.h = None

    def __del__(self):
        self.close()
