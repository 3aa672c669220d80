"""Edge-list ingest, pinned by EdgeListDataSourceTest.scala:39-45,78-82 (4 nodes, 4 relationships)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

EDGE_LIST = "\n0 1\n0 2\n1 2\n1 3\n"


def test_edge_list_graph(session, tmp_path):
    from capsmi import graph, io
    p = tmp_path / "caps_edgelist"
    p.write_text(EDGE_LIST)
    nodes, rels = io.edge_list_graph(session, str(p), " ")
    assert nodes.size == 4
    assert rels.size == 4
    assert sorted(nodes.column("id").values.tolist()) == [0, 1, 2, 3]
    assert rels.column("id").values.tolist() == [0, 1, 2, 3]
    # the graph answers pattern queries through the fused path as well
    bm = graph.NodeBitmap(session, 0, 4).add_scan(nodes)
    assert graph.two_hop_count(session, [rels], bm, bm, bm) == 2        # 0->1->2, 0->1->3
    assert graph.two_hop_count_distinct(session, [rels], bm, bm, bm) == 2


def test_read_edge_list_parsing(tmp_path):
    from capsmi.io import read_edge_list
    p = tmp_path / "e.csv"
    p.write_text("# comment\n5,7\n7,5\n")
    s, d = read_edge_list(str(p), ",")
    np.testing.assert_array_equal(s, [5, 7])
    np.testing.assert_array_equal(d, [7, 5])
