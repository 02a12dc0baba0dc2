"""GPU check of the blocked min-plus Floyd-Warshall comparison engine
(spe_fw_apsp): its closure agrees with the oracle's distances to rounding (FW
associates path segments differently), and its derived next hop equals the
table's on tie-free graphs."""
import numpy as np
import pytest
import torch

from oracle import Oracle
from shadow_amd import graphs, spe

pytestmark = [pytest.mark.gpu, pytest.mark.engine_fixed]


@pytest.mark.parametrize("n,extra,seed,directed", [(70, 150, 1, False), (300, 900, 2, False), (700, 1500, 3, False),
                                                   (200, 700, 5, True)])
def test_fw_distances_and_next_hop(n, extra, seed, directed, monkeypatch):
    monkeypatch.setenv("SPE_NO_PRUNE", "1")   # FW runs over relaxation ids: keep them = vertex ids
    top = graphs.gen_random_small(n, extra, seed, directed=directed)
    g = spe.Graph(top)
    ld = (n + 63) // 64 * 64
    D = torch.empty(ld * ld, dtype=torch.float64, device="cuda")
    NX = torch.empty(n * n, dtype=torch.int32, device="cuda")
    sec = g.fw_apsp(D.data_ptr(), ld, NX.data_ptr())
    assert sec > 0
    d = D.view(ld, ld)[:n, :n].cpu().numpy()
    nx = NX.view(n, n).cpu().numpy()
    A = np.arange(n, dtype=np.int32)
    ref = Oracle(top).rows(A, A, force_sssp=True, tie_mode=1)
    off = ~np.eye(n, dtype=bool)
    assert np.allclose(d[off], ref["lat"][off], rtol=1e-12, atol=0)
    assert np.all(np.diag(d) == 0.0)
    assert np.array_equal(nx[off], ref["next"][off])
    assert np.array_equal(np.diag(nx), np.arange(n))


def test_fw_rejects_bad_ld():
    top = graphs.gen_random_small(100, 200, 4)
    g = spe.Graph(top)
    D = torch.empty(64 * 64, dtype=torch.float64, device="cuda")
    with pytest.raises(spe.SpeError):
        g.fw_apsp(D.data_ptr(), 64)
