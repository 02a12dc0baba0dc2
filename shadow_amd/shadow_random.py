"""Host-side mirror of Shadow's random streams as they reach topology_attach:
shd-random.c (a rand_r state per stream) and the seed chain master -> slave ->
host that decides which topology vertex an un-hinted host attaches to.

  master = Random(options seed, default 1)           shd-master.c:80, shd-options.c:75
  slave  = Random(master.nextUInt())                 shd-master.c:393, shd-slave.c:161
  slave.nextUInt()  -> scheduler seed                shd-slave.c:176
  per host, in configuration order (quantity expanded in place, shd-master.c:280-297):
      host = Random(slave.nextUInt())                shd-slave.c:279, shd-host.c:135
      topology_attach(..., host, ...)                shd-host.c:140
  an un-hinted attach draws once: index round((k - 1) * host.nextDouble()) over
  the k candidate vertices                           shd-topology.c:2310-2316

rand_r is glibc's, called through ctypes, so the streams are the reference's
bit for bit on this libc."""
from __future__ import annotations

import ctypes as C
import math
from typing import Iterable, List, Tuple

_libc = C.CDLL(None)
_rand_r = _libc.rand_r
_rand_r.argtypes = [C.POINTER(C.c_uint)]
_rand_r.restype = C.c_int
RAND_MAX = 2147483647
UINT_MAX = 4294967295


class Random:
    """shd-random.c: random_new / random_nextDouble / random_nextUInt."""

    def __init__(self, seed: int):
        self.state = C.c_uint(seed & 0xFFFFFFFF)

    def rand(self) -> int:
        return int(_rand_r(C.byref(self.state)))

    def next_double(self) -> float:
        return float(self.rand()) / float(RAND_MAX)

    def next_uint(self) -> int:
        return int(self.next_double() * float(UINT_MAX))   # C (uint) cast truncates


def host_streams(hosts: Iterable[Tuple[str, int]], seed: int = 1) -> List[Tuple[str, Random]]:
    """[(hostname, host Random)] for configuration hosts [(id, quantity)], in the
    order the master registers them (names id1..idN when quantity > 1)."""
    master = Random(seed)
    slave = Random(master.next_uint())
    slave.next_uint()   # scheduler seed
    out = []
    for hid, q in hosts:
        for i in range(q):
            name = f"{hid}{i + 1}" if q > 1 else hid
            out.append((name, Random(slave.next_uint())))
    return out


def unhinted_vertex(host: Random, n_candidates: int) -> int:
    """The candidate index an un-hinted attach picks (shd-topology.c:2310-2316)."""
    x = (n_candidates - 1) * host.next_double()
    r = math.floor(x)
    return int(r + 1 if x - r >= 0.5 else r)   # C round(): halves away from zero (Python's round() is to even)
