"""The CMake target a Shadow build adds next to FindIGRAPH (CMakeLists.txt,
cmake/FindSPE.cmake; reference src/main/CMakeLists.txt:6 and :123-125), and
examples/shd_topology_demo.c, a Shadow-worker-shaped C user of the drop-in
topology API (topology_new -> attach -> concurrent per-packet queries ->
free, shd-master.c:209 / shd-host.c:140 / shd-worker.c:235-247).

CPU: the CMake project configures and builds (hipcc cross-compiles gfx950),
the libraries export what the headers declare, a consumer project finds them
with find_package(SPE); the demo rejects an invalid graph before any GPU work.
GPU: the demo on the shipped topology (complete: DIRECT) and on a sparse
synthetic graph (SSSP rows), 4 worker threads, getPathInfo vs the three
separate getters bit for bit."""
import json
import os
import re
import shutil
import subprocess

import numpy as np
import pytest

from shadow_amd import graphs

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEMO = os.path.join(ROOT, "shadow_amd", "shd_topology_demo")


def _declared(header, prefix):
    txt = re.sub(r"/\*.*?\*/", "", open(os.path.join(ROOT, "include", header)).read(), flags=re.S)
    txt = re.sub(r"SHD_TOPO\((\w+)\)", r"\1", txt)   # shd_topology_spe.h's name macro (unprefixed build)
    return set(re.findall(r"\b(" + prefix + r"[A-Za-z0-9_]+)\s*\(", txt))


def _exports(so):
    out = subprocess.run(["nm", "-D", "--defined-only", so], capture_output=True, text=True, check=True).stdout
    return {l.split()[-1] for l in out.splitlines() if " T " in l}


@pytest.mark.skipif(shutil.which("cmake") is None or shutil.which("ninja") is None, reason="cmake/ninja absent")
def test_cmake_target_builds_engine_shim_and_demo(tmp_path):
    b = tmp_path / "build"
    subprocess.run(["cmake", "-S", ROOT, "-B", str(b), "-G", "Ninja"], check=True, capture_output=True, timeout=300)
    subprocess.run(["cmake", "--build", str(b)], check=True, capture_output=True, timeout=600)
    ninja = (b / "build.ninja").read_text()
    assert "--offload-arch=gfx950" in ninja and "-ffp-contract=off" in ninja
    spe, topo = str(b / "libspe.so"), str(b / "libshdtopo.so")
    assert _declared("spe.h", "spe_") <= _exports(spe)
    assert _declared("shd_topology_spe.h", "topology_") <= _exports(topo)
    assert (b / "shd_topology_demo").exists()


@pytest.mark.skipif(shutil.which("cmake") is None, reason="cmake absent")
def test_find_package_spe_from_a_consumer_project(tmp_path):
    """What Shadow's src/main/CMakeLists.txt would do: find_package(SPE) with
    SPE_ROOT at this repository (in-tree build) and link a C program."""
    (tmp_path / "main.c").write_text(
        '#include "shd_topology_spe.h"\n#include "spe.h"\n'
        "int main(void) { return topology_new(\"/nonexistent.graphml\") == 0 ? 0 : 1; }\n")
    (tmp_path / "CMakeLists.txt").write_text(
        "cmake_minimum_required(VERSION 3.21)\nproject(consumer C)\n"
        f"list(APPEND CMAKE_MODULE_PATH {ROOT}/cmake)\nset(SPE_ROOT {ROOT})\n"
        "find_package(SPE REQUIRED)\ninclude_directories(${SPE_INCLUDES})\n"
        "add_executable(consumer main.c)\ntarget_link_libraries(consumer ${SHDTOPO_LIBRARIES} ${SPE_LIBRARIES})\n")
    b = tmp_path / "b"
    subprocess.run(["cmake", "-S", str(tmp_path), "-B", str(b)], check=True, capture_output=True, timeout=120)
    cache = (b / "CMakeCache.txt").read_text()
    assert f"SPE_LIBRARIES:FILEPATH={ROOT}/shadow_amd/libspe.so" in cache
    subprocess.run(["cmake", "--build", str(b)], check=True, capture_output=True, timeout=120)
    # a missing graph file is a validation failure (NULL), no GPU involved
    assert subprocess.run([str(b / "consumer")], timeout=60).returncode == 0


def test_demo_rejects_invalid_graph(tmp_path):
    t = graphs.gen_random_small(20, 30, 1)
    t.elat[0] = 0.0   # latency must be > 0 (shd-topology.c:1026-1109)
    p = tmp_path / "bad.graphml"
    graphs.write_graphml(t, str(p))
    r = subprocess.run([DEMO, str(p), "10", "100"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 2 and "topology_new failed" in r.stderr


def _run_demo(path, hosts, packets, threads=4, seed=1, late=0, batch=0):
    r = subprocess.run([DEMO, str(path), str(hosts), str(packets), str(threads), str(seed), str(late), str(batch)],
                       capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout + r.stderr
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.gpu
@pytest.mark.engine_fixed
def test_demo_on_shipped_topology(tmp_path, golden_dir):
    """C1's graph (complete => DIRECT): 150 hosts, 200k packets on 4 threads."""
    z = np.load(os.path.join(golden_dir, "shipped_topology.npz"))
    top = graphs.Topology(n=int(z["n"]), esrc=z["esrc"], edst=z["edst"], elat=z["elat"], eloss=z["eloss"],
                          vloss=z["vloss"])
    p = tmp_path / "shipped.graphml"
    graphs.write_graphml(top, str(p))
    d = _run_demo(p, 150, 200_000)
    assert d["mismatches"] == 0 and d["routable"] == 200_000 and d["vertices"] == 183
    assert 90 < d["attached_vertices"] <= 150
    # min over the attached pairs' table entries, so at least the graph's min edge latency
    assert d["min_path_latency"] >= float(np.min(z["elat"])) > 0


@pytest.mark.gpu
@pytest.mark.engine_fixed
@pytest.mark.parametrize("engine", ["1", "2"], ids=["batch", "lds"])
def test_demo_on_sparse_graph(tmp_path, monkeypatch, engine):
    """Not complete, no preferdirectpaths => every query is an SSSP row."""
    monkeypatch.setenv("SHADOW_SPE_ENGINE", engine)
    t = graphs.gen_random_small(1500, 4500, 11)
    p = tmp_path / "sparse.graphml"
    graphs.write_graphml(t, str(p))
    d = _run_demo(p, 400, 400_000)
    assert d["mismatches"] == 0 and d["routable"] == 400_000 and d["vertices"] == 1500
    assert d["count_pair_0_0"] >= 0 and d["min_path_latency"] > 0


@pytest.mark.gpu
@pytest.mark.engine_fixed
def test_demo_attach_after_seal_under_concurrent_readers(tmp_path):
    """4 worker threads query while the main thread attaches 200 more hosts to a
    sealed topology: each new vertex makes the next query that needs it build a
    replacement table that is swapped in under the readers.  Getters agree with
    getPathInfo, and the packet counters of all cached paths add up exactly to the
    packets counted (no count lost across the swaps)."""
    t = graphs.gen_random_small(2000, 6000, 12)
    p = tmp_path / "late.graphml"
    graphs.write_graphml(t, str(p))
    d = _run_demo(p, 100, 300_000, threads=4, late=200)
    assert d["mismatches"] == 0 and d["late_hosts"] == 200
    assert d["counted"] == d["routable"] > 0


@pytest.mark.gpu
@pytest.mark.engine_fixed
def test_demo_batched_rounds_with_late_hosts(tmp_path):
    """Workers answer rounds of 80k packets with topology_getPathInfoBatch (the
    threaded path) and count them with topology_incrementPathPacketCounterBatch,
    while the main thread attaches hosts after sealing: every 64th packet of a
    round agrees bit for bit with topology_getPathInfo, and the counters of all
    cached paths add up to the packets counted."""
    t = graphs.gen_random_small(2000, 6000, 13)
    p = tmp_path / "batch.graphml"
    graphs.write_graphml(t, str(p))
    d = _run_demo(p, 300, 640_000, threads=4, late=100, batch=80_000)
    assert d["mismatches"] == 0 and d["batch"] == 80_000
    assert d["counted"] == d["routable"] > 0
