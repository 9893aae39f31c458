"""The reference's parameter snapshot format: `Variable::save` / `Variable::load` (express/Expr.cpp:833-965).

`Variable::save(model->parameters(), file)` writes one MNN `Net` flatbuffer
(schema/default/MNN.fbs:496-513) whose `oplists` hold one op per parameter: type TrainableParam
(a trainable VARP, Expr.cpp:886-888), `main` = Blob {dims, dataFormat, dataType DT_INT8, int8s}
(Tensor.fbs:20-35; Expr.cpp:860-885), `outputIndexes` = [its tensor index], and the name
`EnumNameOpType(type) + index` when the variable has none (Expr.cpp:897-899).  The NITI modules
register only the int8 weight as a parameter (tools/train/source/nn/NN.cpp:1163-1176, the wscale
line is commented out), so the weight scales live in a JSON side-car next to the snapshot.

`flatbuffers` is not importable here, so this module carries its own minimal encoder and decoder
of the flatbuffers binary layout for exactly these tables; the decoder also walks any MNN model
file (tests read the reference's benchmark models through it).
"""
import json
import struct

import numpy as np

# enum values of schema/default/MNN.fbs, Tensor.fbs, Type.fbs
OP_TRAINABLE_PARAM = 266   # OpType::TrainableParam
OP_CONST = 11              # OpType::Const
OP_PARAM_BLOB = 7          # OpParameter union index of Blob (1-based; 0 = NONE)
DT_INT8 = 6                # DataType::DT_INT8
DT_FLOAT = 1
DT_INT32 = 3
DT_UINT8 = 4
FMT_NCHW = 0               # MNN_DATA_FORMAT::NCHW

# field ids (declaration order; a union takes two: <name>_type, then <name>)
_OP = {"inputIndexes": 0, "main_type": 1, "main": 2, "name": 3, "outputIndexes": 4, "type": 5,
       "defaultDimentionFormat": 6}
_NET = {"bizCode": 0, "extraTensorDescribe": 1, "gpulibrary": 2, "oplists": 3, "outputName": 4,
        "preferForwardType": 5, "sourceType": 6, "tensorName": 7, "tensorNumber": 8, "usage": 9,
        "subgraphs": 10, "mnn_uuid": 11}
_BLOB = {"dims": 0, "dataFormat": 1, "dataType": 2, "uint8s": 3, "int8s": 4, "int32s": 5, "int64s": 6,
         "float32s": 7, "strings": 8}


# ---------------------------------------------------------------------------------- encoder
class _Table:
    def __init__(self, fields):
        self.fields = fields  # [(field id, kind, value)], kind: 'b' 'B' 'i' 'I' scalar, 'ref' node


class _Vec:
    def __init__(self, fmt, values):
        self.fmt, self.values = fmt, values  # struct format char of one element


class _RefVec:
    def __init__(self, nodes):
        self.nodes = nodes


class _Str:
    def __init__(self, s):
        self.s = s.encode()


class _Writer:
    """Front-to-back flatbuffer writer: every object is appended after the fields that point at
    it, so each uoffset (target - field position) is positive as the format requires."""

    def __init__(self):
        self.b = bytearray(4)  # root uoffset, patched at the end

    def _align(self, n, extra=0):
        while (len(self.b) + extra) % n:
            self.b.append(0)

    def _patch_u32(self, at, target):
        struct.pack_into("<I", self.b, at, target - at)

    def write(self, node):
        if isinstance(node, _Str):
            self._align(4)
            pos = len(self.b)
            self.b += struct.pack("<I", len(node.s)) + node.s + b"\0"
            return pos
        if isinstance(node, _Vec):
            size = struct.calcsize("<" + node.fmt)
            self._align(max(4, size), extra=4 if size > 4 else 0)
            pos = len(self.b)
            self.b += struct.pack("<I", len(node.values))
            if len(node.values):
                dt = {"b": "i1", "B": "u1", "i": "<i4", "I": "<u4", "q": "<i8", "f": "<f4"}[node.fmt]
                self.b += np.asarray(node.values).astype(dt).tobytes()
            return pos
        if isinstance(node, _RefVec):
            self._align(4)
            pos = len(self.b)
            self.b += struct.pack("<I", len(node.nodes)) + bytes(4 * len(node.nodes))
            for k, child in enumerate(node.nodes):
                self._patch_u32(pos + 4 + 4 * k, self.write(child))
            return pos
        # table: vtable, then the table (soffset to the vtable first), then its children
        fields = sorted(node.fields, key=lambda f: f[0])
        nslots = (fields[-1][0] + 1) if fields else 0
        self._align(2)
        vt = len(self.b)
        self.b += bytes(4 + 2 * nslots)
        self._align(4)
        tbl = len(self.b)
        self.b += struct.pack("<i", tbl - vt)
        refs = []
        offs = {}
        for fid, kind, value in fields:
            size = 4 if kind == "ref" else struct.calcsize("<" + kind)
            self._align(size)
            offs[fid] = len(self.b) - tbl
            if kind == "ref":
                refs.append((len(self.b), value))
                self.b += bytes(4)
            else:
                self.b += struct.pack("<" + kind, value)
        struct.pack_into("<HH", self.b, vt, 4 + 2 * nslots, len(self.b) - tbl)
        for fid, o in offs.items():
            struct.pack_into("<H", self.b, vt + 4 + 2 * fid, o)
        for at, child in refs:
            self._patch_u32(at, self.write(child))
        return tbl

    def finish(self, root):
        pos = self.write(root)
        struct.pack_into("<I", self.b, 0, pos)
        return bytes(self.b)


def encode_params(params, names=None) -> bytes:
    """Net flatbuffer of `Variable::save(params, ...)` for int8 NCHW parameters (the order is kept:
    `Module::loadParameters` assigns them in order)."""
    ops, tnames = [], []
    for i, w in enumerate(params):
        w = np.ascontiguousarray(w, dtype=np.int8)
        name = (names[i] if names else "") or f"TrainableParam{i + 1}"  # Expr.cpp:897-899
        blob = _Table([(_BLOB["dims"], "ref", _Vec("i", [int(d) for d in w.shape])),
                       (_BLOB["dataFormat"], "b", FMT_NCHW),
                       (_BLOB["dataType"], "i", DT_INT8),
                       (_BLOB["int8s"], "ref", _Vec("b", w.reshape(-1)))])
        ops.append(_Table([(_OP["inputIndexes"], "ref", _Vec("i", [])),
                           (_OP["main_type"], "B", OP_PARAM_BLOB),
                           (_OP["main"], "ref", blob),
                           (_OP["name"], "ref", _Str(name)),
                           (_OP["outputIndexes"], "ref", _Vec("i", [i])),
                           (_OP["type"], "i", OP_TRAINABLE_PARAM)]))
        tnames.append(name)  # Expr.cpp:906-923: an unnamed output takes its op's name
    net = _Table([(_NET["oplists"], "ref", _RefVec(ops)),
                  (_NET["tensorName"], "ref", _RefVec([_Str(n) for n in tnames]))])
    return _Writer().finish(net)


# ---------------------------------------------------------------------------------- decoder
class _Reader:
    def __init__(self, buf: bytes):
        self.b = memoryview(buf)
        if len(buf) < 8:
            raise ValueError("not a flatbuffer: too short")

    def u32(self, at):
        if at < 0 or at + 4 > len(self.b):
            raise ValueError(f"offset {at} out of range")
        return struct.unpack_from("<I", self.b, at)[0]

    def root(self):
        return self.u32(0)

    def _vtable(self, tbl):
        vt = tbl - struct.unpack_from("<i", self.b, tbl)[0]
        if vt < 0 or vt + 4 > len(self.b):
            raise ValueError("bad vtable")
        vsize, _ = struct.unpack_from("<HH", self.b, vt)
        return vt, vsize

    def field_pos(self, tbl, fid):
        vt, vsize = self._vtable(tbl)
        if 4 + 2 * fid >= vsize:
            return None
        o = struct.unpack_from("<H", self.b, vt + 4 + 2 * fid)[0]
        return tbl + o if o else None

    def scalar(self, tbl, fid, fmt, default=0):
        p = self.field_pos(tbl, fid)
        return default if p is None else struct.unpack_from("<" + fmt, self.b, p)[0]

    def ref(self, tbl, fid):
        p = self.field_pos(tbl, fid)
        return None if p is None else p + self.u32(p)

    def _str_at(self, p):
        n = self.u32(p)
        if p + 4 + n + 1 > len(self.b) or self.b[p + 4 + n] != 0:
            raise ValueError("string past the buffer or not terminated")
        return bytes(self.b[p + 4:p + 4 + n]).decode()

    def string(self, tbl, fid):
        p = self.ref(tbl, fid)
        return None if p is None else self._str_at(p)

    def vec(self, tbl, fid, dtype):
        p = self.ref(tbl, fid)
        if p is None:
            return None
        n = self.u32(p)
        dt = np.dtype(dtype)
        end = p + 4 + n * dt.itemsize
        if end > len(self.b):
            raise ValueError("vector past the buffer")
        return np.frombuffer(self.b[p + 4:end], dtype=dt).copy()

    def tables(self, tbl, fid):
        p = self.ref(tbl, fid)
        if p is None:
            return []
        n = self.u32(p)
        return [p + 4 + 4 * k + self.u32(p + 4 + 4 * k) for k in range(n)]

    def strings(self, tbl, fid):
        return [self._str_at(s) for s in self.tables(tbl, fid)]


def decode_net(buf: bytes) -> dict:
    """{'ops': [{name, type, main_type, inputIndexes, outputIndexes, blob?}], 'tensorName': [...]}
    for any MNN Net flatbuffer; `blob` (dims, dataFormat, dataType, data) for Blob-parameter ops."""
    r = _Reader(buf)
    net = r.root()
    ops = []
    for t in r.tables(net, _NET["oplists"]):
        op = {"name": r.string(t, _OP["name"]), "type": r.scalar(t, _OP["type"], "i"),
              "main_type": r.scalar(t, _OP["main_type"], "B"),
              "inputIndexes": r.vec(t, _OP["inputIndexes"], "<i4"),
              "outputIndexes": r.vec(t, _OP["outputIndexes"], "<i4")}
        if op["main_type"] == OP_PARAM_BLOB:
            b = r.ref(t, _OP["main"])
            dims = r.vec(b, _BLOB["dims"], "<i4")
            dt = r.scalar(b, _BLOB["dataType"], "i", DT_FLOAT)
            field, npt = {DT_INT8: ("int8s", np.int8), DT_UINT8: ("uint8s", np.uint8), DT_INT32: ("int32s", "<i4"),
                          DT_FLOAT: ("float32s", "<f4")}.get(dt, (None, None))
            data = r.vec(b, _BLOB[field], npt) if field else None
            op["blob"] = {"dims": [] if dims is None else dims.tolist(),
                          "dataFormat": r.scalar(b, _BLOB["dataFormat"], "b"), "dataType": dt, "data": data}
        ops.append(op)
    return {"ops": ops, "tensorName": r.strings(net, _NET["tensorName"])}


# ---------------------------------------------------------------------------------- files
def save(path: str, weights, wscales, names=None, meta=None):
    """`Variable::save(model->parameters(), path)` + `path.wscale.json` (the scales the NITI
    modules keep outside their parameters)."""
    with open(path, "wb") as f:
        f.write(encode_params(weights, names))
    side = {"format": "niti-mnn-snapshot-wscale", "wscale": [int(s) for s in wscales]}
    if meta:
        side.update(meta)
    with open(path + ".wscale.json", "w") as f:
        json.dump(side, f)


def load(path: str):
    """`Variable::load(path)`: the int8 parameters in file order, their wscales (None without a
    side-car) and the side-car metadata.  ValueError on anything that is not such a snapshot."""
    with open(path, "rb") as f:
        buf = f.read()
    try:
        net = decode_net(buf)
    except (struct.error, ValueError, UnicodeDecodeError) as e:
        raise ValueError(f"{path}: not an MNN Net flatbuffer ({e})") from None
    weights = []
    for op in net["ops"]:
        b = op.get("blob")
        if op["type"] not in (OP_TRAINABLE_PARAM, OP_CONST) or b is None:
            raise ValueError(f"{path}: op {op['name']!r} is not a parameter blob")
        if b["dataType"] != DT_INT8 or b["data"] is None:
            raise ValueError(f"{path}: parameter {op['name']!r} is not int8")
        n = int(np.prod(b["dims"])) if b["dims"] else 1
        if b["data"].size != n:
            raise ValueError(f"{path}: parameter {op['name']!r} holds {b['data'].size} values for dims {b['dims']}")
        weights.append(b["data"].reshape(b["dims"]))
    wscales, meta = None, {}
    try:
        with open(path + ".wscale.json") as f:
            meta = json.load(f)
        wscales = [int(v) for v in meta["wscale"]]
    except FileNotFoundError:
        pass
    except (ValueError, KeyError, TypeError) as e:
        raise ValueError(f"{path}.wscale.json: malformed ({e})") from None
    if wscales is not None and len(wscales) != len(weights):
        raise ValueError(f"{path}: {len(weights)} parameters but {len(wscales)} wscales")
    return weights, wscales, meta
