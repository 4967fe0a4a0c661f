"""CPU suite for SURVEY.md §8f row 3 (aclswarm_amd/formations.py): the
formations.yaml loader (operator.py semantics), the ROS1 encodings of
aclswarm_msgs/Formation and CBAA, and final bids rebuilt from the engine's
who tables + alignments against the CPU restatement's own bid tables."""
import os
import struct

import numpy as np
import pytest

import helpers as H
import pyoracle as O
from aclswarm_amd import formations as FM

REF_YAML = "/root/reference/aclswarm/param/formations.yaml"


@pytest.mark.skipif(not os.path.exists(REF_YAML), reason="reference tree not mounted")
def test_loader_reads_reference_formations_yaml_like_the_operator():
    g = FM.load_formation_group(REF_YAML, "swarm6_3d")
    fx = H.load_json("swarm6_3d.json")
    assert g["agents"] == fx["n"] == 6
    for f, ref in zip(g["formations"], fx["formations"]):
        assert f["name"] == ref["name"]
        # the operator sends float32 points (operator.py:156-157)
        assert (f["points"] == np.array(ref["points"], np.float32).astype(np.float64)).all()
        # the group-level `adjmat: fc` (formations.yaml:143) overrides the
        # per-formation lists (manageAdjmat, operator.py:96-110)
        assert (f["adjmat"] == 1 - np.eye(6, dtype=np.uint8)).all()
        assert (f["gains"] == np.array(ref["gains"])).all()
    sq = FM.load_formation_group(REF_YAML, "swarm4")      # adjmat: fc (group level)
    assert (sq["formations"][0]["adjmat"] == 1 - np.eye(4, dtype=np.uint8)).all()


def test_loader_adjmat_rules_and_scale(tmp_path):
    y = tmp_path / "f.yaml"
    y.write_text("""
grp:
  agents: 3
  formations:
    - name: "a"
      scale: 2.0
      points: [[0.1, 0, 0], [1, 0, 0], [0, 1, 0.5]]
    - name: "b"
      adjmat: [[0, 1, 0], [1, 0, 1], [0, 1, 0]]
      points: [[0, 0, 0], [1, 0, 0], [0, 1, 0]]
glob:
  agents: 3
  adjmat: [[0, 1, 1], [1, 0, 0], [1, 0, 0]]
  formations:
    - name: "c"
      adjmat: fc
      points: [[0, 0, 0], [1, 0, 0], [0, 1, 0]]
""")
    g = FM.load_formation_group(str(y), "grp")
    a, b = g["formations"]
    assert (a["adjmat"] == 1 - np.eye(3, dtype=np.uint8)).all()          # missing -> fc
    assert a["points"][0, 0] == float(np.float32(2.0) * np.float32(0.1))  # float32 scale
    assert (b["adjmat"] == np.array([[0, 1, 0], [1, 0, 1], [0, 1, 0]])).all()
    c = FM.load_formation_group(str(y), "glob")["formations"][0]
    assert (c["adjmat"] == np.array([[0, 1, 1], [1, 0, 0], [1, 0, 0]])).all()  # global wins
    with pytest.raises(KeyError):
        FM.load_formation_group(str(y), "nope")


def test_cbaa_message_bytes_and_round_trip():
    b = FM.encode_cbaa(7, 3, [0.5, 0.0], [1, -1], seq=2, stamp=(10, 20), frame_id="v1")
    want = (struct.pack("<III", 2, 10, 20) + struct.pack("<I", 2) + b"v1"
            + struct.pack("<II", 7, 3) + struct.pack("<I", 2) + struct.pack("<ff", 0.5, 0.0)
            + struct.pack("<I", 2) + struct.pack("<ii", 1, -1))
    assert b == want
    d = FM.decode_cbaa(b)
    assert d["auctionId"] == 7 and d["iter"] == 3 and d["header"]["frame_id"] == "v1"
    assert list(d["price"]) == [0.5, 0.0] and list(d["who"]) == [1, -1]


def test_formation_message_round_trip():
    pts, adj, gains, _ = H.swarm6()
    b = FM.encode_formation("Pentagonal Pyramid", pts[0], adj[0], gains[0], seq=1)
    d = FM.decode_formation(b)
    assert d["name"] == "Pentagonal Pyramid"
    assert (d["points"] == pts[0]).all() and (d["adjmat"] == adj[0]).all()
    assert (d["gains"] == np.asarray(gains[0], np.float32).astype(np.float64)).all()
    d2 = FM.decode_formation(FM.encode_formation("x", pts[0], adj[0], None))
    assert d2["gains"] is None          # gains used only with a 2-D layout


def test_bids_from_who_tables_and_alignments_equal_the_oracle_bids():
    P20, A20 = H.simform("simform20_nc")
    rng = np.random.RandomState(4)
    for k in range(6):
        p, adj = P20[k, 0], A20[k]
        q = H.random_positions(rng, 20, 20.0)
        P = H.random_perm(rng, 20)
        C, Rt = O.prices(q, p, adj, P)
        who, pr, _ = O.cbaa(C, adj, P)
        w16 = np.where(who < 0, 0xFFFF, who).astype(np.uint16)
        price, who2 = FM.bids_from_solve(q, p, w16, Rt)
        assert (who2 == who).all()
        assert (price.view(np.uint32) == pr.view(np.uint32)).all()
