"""Generate the committed golden fixtures under tests/golden/.

Inputs come from the reference's own data files (read here, where
/root/reference exists); expected outputs for the DIRECT regime follow from
those data directly (edge attributes), and the oracle's outputs are stored
alongside so the GPU box (which has no /root/reference) can check against
them.  Run:  python tools/gen_golden.py
"""
import json
import os
import re
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
from shadow_amd import graphs  # noqa: E402
from oracle import Oracle  # noqa: E402

REF = "/root/reference"
OUT = os.path.join(ROOT, "tests", "golden")


def cdata_topology(config_path):
    txt = open(config_path).read()
    m = re.search(r"<!\[CDATA\[(.*?)\]\]>", txt, re.S)
    return m.group(1)


def main():
    os.makedirs(OUT, exist_ok=True)
    # --- K4: shipped topology (resource/topology.graphml.xml.xz)
    top = graphs.load_graphml(os.path.join(REF, "resource", "topology.graphml.xml.xz"))
    o = Oracle(top)
    A = np.arange(top.n, dtype=np.int32)
    direct = o.rows(A, A)
    diag_ig = o.rows(A, A, force_sssp=True, tie_mode=0, want_ties=True)
    diag_cn = o.rows(A, A, force_sssp=True, tie_mode=1)
    np.savez_compressed(
        os.path.join(OUT, "shipped_topology.npz"),
        n=top.n, esrc=top.esrc, edst=top.edst, elat=top.elat, eloss=top.eloss, vloss=top.vloss,
        directed=int(top.directed), prefer_direct=int(top.prefer_direct),
        direct_lat=direct["lat"], direct_rel=direct["rel"], direct_kind=direct["kind"],
        sssp_lat=diag_ig["lat"], sssp_rel=diag_ig["rel"], sssp_next=diag_ig["next"], sssp_hops=diag_ig["hops"],
        sssp_canon_next=diag_cn["next"], sssp_canon_hops=diag_cn["hops"], sssp_canon_rel=diag_cn["rel"],
        sssp_double_ties=diag_ig["double_ties"],
    )
    # --- completion tool (compute-topology-paths.py) on the shipped topology, every
    # vertex a POI: networkx restatement (oracle/topology_tools.py) of its worker()
    import topology_tools as tt
    jit = top.eattrs["jitter"]
    pois = np.arange(top.n, dtype=np.int32)
    clat, cjit, chops = tt.all_rows(top, jit, pois)
    np.savez_compressed(os.path.join(OUT, "completion_shipped.npz"), ejitter=jit, pois=pois,
                        lat=clat, jitter=cjit, hops=chops)
    # --- K1/K2: the 1-vertex topologies embedded in the reference's configs
    kats = {}
    for name, rel in [("examples", "resource/examples/shadow.config.xml"),
                      ("tcp_lossy", "src/test/tcp/tcp-blocking-lossy.test.shadow.config.xml"),
                      ("tcp_lossless", "src/test/tcp/tcp-blocking-lossless.test.shadow.config.xml")]:
        gml = cdata_topology(os.path.join(REF, rel))
        t = graphs.load_graphml(gml, is_text=True)
        r = Oracle(t).rows([0], [0])
        kats[name] = {"source": rel, "graphml": gml, "complete": bool(Oracle(t).complete),
                      "lat": float(r["lat"][0, 0]), "rel": float(r["rel"][0, 0]), "kind": int(r["kind"][0, 0])}
    with open(os.path.join(OUT, "kat_1vertex.json"), "w") as f:
        json.dump(kats, f, indent=1)
    print("shipped topology:", top.n, "vertices", top.m, "edges; double ties (SSSP diag):",
          diag_ig["double_ties"])
    print(json.dumps({k: (v["lat"], v["rel"], v["kind"]) for k, v in kats.items()}))


if __name__ == "__main__":
    main()
