"""Formation files and wire formats around the decision loop (SURVEY.md §8f
row 3): the formations.yaml loader, and the ROS1 encodings of
aclswarm_msgs/Formation and aclswarm_msgs/CBAA, so formation groups and
per-vehicle bids can move between this engine and a reference deployment
without ROS installed.

* load_formation_group(path, group) follows the operator's reading of
  aclswarm/param/formations.yaml (aclswarm/nodes/operator.py):
  manageAdjmat (:87-110) -- a group-level `adjmat` overrides every
  formation's, a missing or non-list adjmat ("fc") is ones - eye;
  getPoints (:156-157) -- points scaled by the optional `scale` in float32,
  which is what the vehicles receive (buildFormationMessage :159-174 packs
  them into geometry_msgs/Point); optional `gains` as given (the debugging
  path of :184-206), or float32-rounded as decodeGainMat
  (aclswarm/include/aclswarm/utils.h:110-126) would see them.
* encode_formation / decode_formation: ROS1 serialization of
  aclswarm_msgs/Formation.msg (Header, string name, geometry_msgs/Point[],
  std_msgs/UInt8MultiArray adjmat, std_msgs/Float32MultiArray gains);
  decode follows CoordinationROS::formationCb (coordination_ros.cpp:210-232)
  with utils::decodeAdjMat / decodeGainMat (utils.h:83-126): gains are used
  only when their layout has two dimensions.
* encode_cbaa / decode_cbaa: aclswarm_msgs/CBAA.msg (Header, uint32
  auctionId, uint32 iter, float32[] price, int32[] who), the bid
  sendBidCb publishes (coordination_ros.cpp:308-318).
* bids_from_solve: a vehicle's final bid (price and who per task) rebuilt
  from acl_solve_batch's `who` tables and `align_Rt` (price = C[who][j],
  getPrice auctioneer.cpp:546-549, from who's own alignment).

ROS1 wire format: little-endian; uint32 length before strings and
variable-length arrays; Header = uint32 seq, time stamp (uint32 sec, uint32
nsec), string frame_id.
"""
import struct

import numpy as np
import yaml


def load_formation_group(path, group):
    """-> dict(name, agents, formations=[dict(name, points [n][3] f64,
    adjmat [n][n] u8, gains [3n][3n] f64 or None, gains_f32 or None)])."""
    with open(path) as f:
        doc = yaml.safe_load(f)
    if group not in doc:
        raise KeyError(f"formation group {group!r} not in {path}")
    g = doc[group]
    n = int(g["agents"])
    has_global = "adjmat" in g
    out = []
    for fm in g["formations"]:
        adj = g["adjmat"] if has_global else fm.get("adjmat")
        if not isinstance(adj, list):
            A = (np.ones((n, n)) - np.eye(n)).astype(np.uint8)
        else:
            A = np.array(adj, dtype=np.uint8)
        scale = float(fm["scale"]) if "scale" in fm else 1.0
        pts = scale * np.array(fm["points"], dtype=np.float32)  # float32 (NEP 50)
        gains = np.array(fm["gains"], dtype=np.float64) if "gains" in fm else None
        if A.shape != (n, n) or pts.shape != (n, 3):
            raise ValueError(f"formation {fm.get('name')!r}: shapes do not match agents={n}")
        out.append({"name": fm["name"], "points": pts.astype(np.float64), "adjmat": A,
                    "gains": gains,
                    "gains_f32": None if gains is None else
                    gains.astype(np.float32).astype(np.float64)})
    return {"name": group, "agents": n, "formations": out}


def formation_table(group, device="cuda", use_f32_gains=False):
    """An engine.FormationTable over every formation of a loaded group (gains
    required)."""
    from . import engine
    key = "gains_f32" if use_f32_gains else "gains"
    fms = group["formations"]
    if any(f[key] is None for f in fms):
        raise ValueError("formation_table: every formation needs gains (run ADMM first)")
    return engine.FormationTable.from_host([f["points"] for f in fms],
                                           [f["adjmat"] for f in fms],
                                           [f[key] for f in fms], device=device)


# ---- ROS1 serialization ---------------------------------------------------

def _header(seq=0, stamp=(0, 0), frame_id=""):
    fid = frame_id.encode()
    return struct.pack("<III", seq, stamp[0], stamp[1]) + struct.pack("<I", len(fid)) + fid


def _read_header(buf, o):
    seq, sec, nsec, ln = struct.unpack_from("<IIII", buf, o)
    o += 16
    fid = bytes(buf[o:o + ln]).decode()
    return {"seq": seq, "stamp": (sec, nsec), "frame_id": fid}, o + ln


def _multiarray(data, dtype, dims):
    """std_msgs/*MultiArray: MultiArrayLayout (dim[] of {string label, uint32
    size, uint32 stride}, uint32 data_offset) then data[]."""
    b = struct.pack("<I", len(dims))
    for label, size, stride in dims:
        lb = label.encode()
        b += struct.pack("<I", len(lb)) + lb + struct.pack("<II", size, stride)
    b += struct.pack("<I", 0)
    arr = np.ascontiguousarray(data, dtype=dtype).ravel()
    return b + struct.pack("<I", arr.size) + arr.astype(np.dtype(dtype).newbyteorder("<")).tobytes()


def _read_multiarray(buf, o, dtype):
    (nd,) = struct.unpack_from("<I", buf, o)
    o += 4
    dims = []
    for _ in range(nd):
        (ln,) = struct.unpack_from("<I", buf, o)
        label = bytes(buf[o + 4:o + 4 + ln]).decode()
        o += 4 + ln
        size, stride = struct.unpack_from("<II", buf, o)
        o += 8
        dims.append((label, size, stride))
    (off, cnt) = struct.unpack_from("<II", buf, o)
    o += 8
    dt = np.dtype(dtype).newbyteorder("<")
    data = np.frombuffer(bytes(buf[o:o + cnt * dt.itemsize]), dtype=dt).astype(dtype)
    return {"dims": dims, "data_offset": off, "data": data}, o + cnt * dt.itemsize


def _matrix_dims(rows, cols):
    # operator.py:175-182: dim[0] rows (stride rows*cols), dim[1] cols (stride cols)
    return [("rows", rows, rows * cols), ("cols", cols, cols)]


def encode_formation(name, points, adjmat, gains=None, seq=0, stamp=(0, 0), frame_id=""):
    """aclswarm_msgs/Formation (buildFormationMessage, operator.py:159-206;
    gains as the Float32MultiArray the message declares)."""
    pts = np.asarray(points, dtype=np.float64)
    A = np.asarray(adjmat, dtype=np.uint8)
    nm = name.encode()
    b = _header(seq, stamp, frame_id) + struct.pack("<I", len(nm)) + nm
    b += struct.pack("<I", pts.shape[0]) + pts.astype("<f8").tobytes()
    b += _multiarray(A, np.uint8, _matrix_dims(*A.shape))
    if gains is None:
        b += _multiarray(np.zeros(0, np.float32), np.float32, [])
    else:
        G = np.asarray(gains, dtype=np.float32)
        b += _multiarray(G, np.float32, _matrix_dims(*G.shape))
    return b


def decode_formation(buf):
    """-> dict(header, name, points [n][3] f64, adjmat [n][n] u8, gains
    [3n][3n] f64 or None) as CoordinationROS::formationCb reads it."""
    hdr, o = _read_header(buf, 0)
    (ln,) = struct.unpack_from("<I", buf, o)
    name = bytes(buf[o + 4:o + 4 + ln]).decode()
    o += 4 + ln
    (npts,) = struct.unpack_from("<I", buf, o)
    o += 4
    pts = np.frombuffer(bytes(buf[o:o + 24 * npts]), dtype="<f8").reshape(npts, 3).astype(np.float64)
    o += 24 * npts
    am, o = _read_multiarray(buf, o, np.uint8)
    gm, o = _read_multiarray(buf, o, np.float32)

    def decode(m, dtype):  # utils::decodeAdjMat / decodeGainMat (utils.h:83-126)
        rows, cols = m["dims"][0][1], m["dims"][1][1]
        stride = m["dims"][1][2]
        out = np.zeros((rows, cols), dtype)
        for i in range(rows):
            out[i] = m["data"][m["data_offset"] + stride * i: m["data_offset"] + stride * i + cols]
        return out

    A = decode(am, np.uint8)
    G = decode(gm, np.float64) if len(gm["dims"]) == 2 else None
    return {"header": hdr, "name": name, "points": pts, "adjmat": A, "gains": G}


def encode_cbaa(auction_id, iteration, price, who, seq=0, stamp=(0, 0), frame_id=""):
    """aclswarm_msgs/CBAA (sendBidCb, coordination_ros.cpp:308-318)."""
    p = np.asarray(price, dtype="<f4")
    w = np.asarray(who, dtype="<i4")
    return (_header(seq, stamp, frame_id) + struct.pack("<II", auction_id, iteration)
            + struct.pack("<I", p.size) + p.tobytes() + struct.pack("<I", w.size) + w.tobytes())


def decode_cbaa(buf):
    hdr, o = _read_header(buf, 0)
    auction_id, iteration, npr = struct.unpack_from("<III", buf, o)
    o += 12
    price = np.frombuffer(bytes(buf[o:o + 4 * npr]), dtype="<f4").astype(np.float32)
    o += 4 * npr
    (nw,) = struct.unpack_from("<I", buf, o)
    o += 4
    who = np.frombuffer(bytes(buf[o:o + 4 * nw]), dtype="<i4").astype(np.int32)
    return {"header": hdr, "auctionId": auction_id, "iter": iteration, "price": price, "who": who}


def bids_from_solve(q, p, who_rows, align_Rt):
    """Final bids of one swarm's vehicles from acl_solve_batch outputs:
    q [n][3] vehicle positions, p [n][3] formation points, who_rows [n][n]
    (uint16, 0xFFFF = -1; row v = vehicle v's table), align_Rt [n][6] (R, t
    per vehicle, acl_solve_args_t::align_Rt). Returns (price
    [n][n] f32, who [n][n] i32) with price[v][j] = getPrice of who's bid,
    i.e. C[who][j] (auctioneer.cpp:546-549), 0 where who == -1."""
    q = np.asarray(q, np.float64)
    p = np.asarray(p, np.float64)
    n = q.shape[0]
    W = np.asarray(who_rows).astype(np.int64)
    Rt = np.asarray(align_Rt, np.float64)
    # C[u][j]: vehicle u's price for task j, from u's own alignment
    px, py, pz = p[:, 0][None, :], p[:, 1][None, :], p[:, 2][None, :]
    R0, R1, R2, R3, t0, t1 = (Rt[:, k][:, None] for k in range(6))
    ax = ((R0 * px + R1 * py) + 0.0 * pz) + t0
    ay = ((R2 * px + R3 * py) + 0.0 * pz) + t1
    az = ((0.0 * px + 0.0 * py) + 1.0 * pz) + 0.0
    dx, dy, dz = q[:, 0][:, None] - ax, q[:, 1][:, None] - ay, q[:, 2][:, None] - az
    C = (1.0 / (np.sqrt((dx * dx + dy * dy) + dz * dz) + 1e-8)).astype(np.float32)
    who = np.where(W == 0xFFFF, -1, W).astype(np.int32)
    price = np.zeros((n, n), np.float32)
    jj = np.arange(n)[None, :].repeat(n, 0)
    ok = who >= 0
    price[ok] = C[who[ok], jj[ok]]
    return price, who
