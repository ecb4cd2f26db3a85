"""Topology probe (mp4x/utils/topology.py, csrc/runtime/topo.hip)."""
import pytest

from mp4x.utils.topology import LINK_NAMES, XGMI, summarize


def _mesh(n, link=XGMI, hops=1):
    m = {k: [[0] * n for _ in range(n)] for k in ("link", "hops", "access", "perf_rank", "atomics")}
    for a in range(n):
        for b in range(n):
            if a == b:
                m["link"][a][b] = -1
                m["access"][a][b] = 1
            else:
                m["link"][a][b] = link
                m["hops"][a][b] = hops
                m["access"][a][b] = 1
    return m


def test_full_xgmi_mesh():
    s = summarize(_mesh(8))
    assert s["devices"] == 8 and s["xgmi_mesh"] is True
    assert s["pairs"] == {"xgmi": 56} and s["max_hops"] == 1 and s["no_peer_access"] == []


def test_subset_and_pcie_and_no_access():
    m = _mesh(8)
    m["link"][2][5] = 2          # one PCIe pair
    assert summarize(m, [0, 1, 3])["xgmi_mesh"] is True      # the PCIe pair is outside the subset
    s = summarize(m, [2, 5])
    assert s["xgmi_mesh"] is False and s["pairs"] == {"pcie": 1, "xgmi": 1}
    m["access"][0][1] = 0
    s = summarize(m, [0, 1])
    assert s["xgmi_mesh"] is False and s["no_peer_access"] == [(0, 1)]
    assert summarize(_mesh(8, hops=2))["xgmi_mesh"] is False


def test_single_device_and_duplicates():
    s = summarize(_mesh(8), [3, 3])      # ranks sharing one GPU
    assert s["devices"] == 1 and s["xgmi_mesh"] is None and s["pairs"] == {}


@pytest.mark.gpu
def test_probe_on_device():
    import torch
    from mp4x.utils.topology import local_summary, probe
    m = probe()
    assert m is not None, "native topology probe unavailable on a GPU box"
    n = torch.cuda.device_count()
    assert len(m["link"]) == n and all(len(r) == n for r in m["link"])
    for a in range(n):
        assert m["access"][a][a] == 1 and m["hops"][a][a] == 0
        for b in range(n):
            if a != b:   # a known link type, at least one hop (an MI355X node: xGMI, 1 hop)
                assert m["link"][a][b] in LINK_NAMES and m["hops"][a][b] >= 1, (a, b, m["link"][a][b])
    s = local_summary()
    assert s["devices"] == n
