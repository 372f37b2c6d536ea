"""Go encoding/gob, the wire format of the reference's net/rpc transport (DistSys/main.go:10-11,
900-907,1191-1204; every Peer.* RPC argument and reply travels as gob over TCP).

A gob stream is a sequence of messages ``uint(len) + payload``; a payload is ``int(type id)`` then
either a type definition (negative id: a ``wireType`` struct) or a value (positive id; a non-struct
top-level value is preceded by a 0 "singleton field" byte).  Type ids 1-7 are the builtins bool, int,
uint, float, []byte, string, complex; user types are numbered from 65 as each encoder first meets
them, depth-first, a struct taking its id before its fields' types.  Integers are zig-zag coded
uints; uints < 128 are one byte, larger ones a negated byte count and big-endian bytes; floats are
the byte-reversed IEEE-754 bits as a uint; structs send only their non-zero fields as
(field-number delta, value) pairs ended by 0.

This module encodes and decodes exactly the schema language the reference's messages need: the
basic types, slices, maps, structs (pointers are transparent in gob).  `Encoder` / `Decoder` keep
the per-stream type state, like Go's, so a net/rpc connection (parallel/netrpc.py) can interleave
headers and bodies.  The block hash preimage (gob of BlockData, blockData.go:31-41) produced here
is byte-identical to the C++ ledger's encoder and to the hand-derived Go vector
(tests/test_protocol.py::test_gob_blockdata_hand_derived_vector).
"""
from __future__ import annotations

import io
import struct
from dataclasses import dataclass, field


# ---------------------------------------------------------------------------- schema
@dataclass(frozen=True)
class Basic:
    name: str
    id: int


BOOL, INT, UINT, FLOAT, BYTES, STRING = (Basic("bool", 1), Basic("int", 2), Basic("uint", 3), Basic("float", 4),
                                         Basic("[]byte", 5), Basic("string", 6))
_BASIC_BY_ID = {b.id: b for b in (BOOL, INT, UINT, FLOAT, BYTES, STRING)}


@dataclass(frozen=True)
class Slice:
    elem: object
    name: str = ""


@dataclass(frozen=True)
class Map:
    key: object
    elem: object
    name: str = ""


@dataclass(frozen=True, eq=False)
class Struct:
    name: str
    fields: tuple = field(default_factory=tuple)   # ((field name, schema), ...) in declaration order


def type_name(t) -> str:
    if isinstance(t, Basic):
        return {"[]byte": "[]uint8"}.get(t.name, t.name if t.name != "float" else "float64")
    if isinstance(t, Struct):
        return t.name
    if isinstance(t, Slice):
        return t.name or "[]" + _elem_name(t.elem)
    if isinstance(t, Map):
        return t.name or f"map[{_elem_name(t.key)}]{_elem_name(t.elem)}"
    raise TypeError(t)


def _elem_name(t) -> str:
    if isinstance(t, Struct):
        return "main." + t.name
    return type_name(t)


# ---------------------------------------------------------------------------- primitive coding
def enc_uint(out: bytearray, v: int) -> None:
    if v < 0:
        raise ValueError("negative uint")
    if v < 128:
        out.append(v)
        return
    b = v.to_bytes((v.bit_length() + 7) // 8, "big")
    out.append((256 - len(b)) & 0xFF)
    out += b


def enc_int(out: bytearray, v: int) -> None:
    enc_uint(out, ((~v) << 1) | 1 if v < 0 else v << 1)


def enc_float(out: bytearray, v: float) -> None:
    bits = struct.unpack("<Q", struct.pack("<d", v))[0]
    enc_uint(out, int.from_bytes(bits.to_bytes(8, "little"), "big"))


def enc_bytes(out: bytearray, b: bytes) -> None:
    enc_uint(out, len(b))
    out += b


class _Reader:
    def __init__(self, buf: bytes):
        self.b, self.i = buf, 0

    def byte(self) -> int:
        v = self.b[self.i]
        self.i += 1
        return v

    def take(self, n: int) -> bytes:
        v = self.b[self.i:self.i + n]
        if len(v) != n:
            raise EOFError("truncated gob value")
        self.i += n
        return v

    def uint(self) -> int:
        c = self.byte()
        if c < 128:
            return c
        n = 256 - c
        if n > 8:   # Go's decoder: a uint has at most 8 bytes
            raise ValueError("gob: uint with more than 8 bytes")
        return int.from_bytes(self.take(n), "big")

    def count(self) -> int:
        """An element count: every element takes at least one byte, so a count beyond the bytes left in
        the message is malformed (never allocate or loop on what a peer merely declares)."""
        n = self.uint()
        if n > len(self.b) - self.i:
            raise ValueError("gob: element count exceeds the message")
        return n

    def int(self) -> int:
        u = self.uint()
        return ~(u >> 1) if u & 1 else u >> 1

    def float(self) -> float:
        u = self.uint()
        return struct.unpack("<d", struct.pack("<Q", int.from_bytes(u.to_bytes(8, "big"), "little")))[0]

    def bytes_(self) -> bytes:
        return bytes(self.take(self.count()))


# ---------------------------------------------------------------------------- encoder
def _is_zero(t, v) -> bool:
    if v is None:
        return True
    if isinstance(t, Basic):
        return v in (0, 0.0, False, b"", "") and not (t is FLOAT and str(v) == "-0.0")
    if isinstance(t, (Slice, Map)):
        return len(v) == 0
    return False   # structs are always sent (gob sends a nested struct even when all fields are zero)


class Encoder:
    """One direction of a gob stream (Go's gob.Encoder): type definitions are sent once per stream.
    Ids are allocated like Go's type builder (a struct takes its id before its fields' types, a slice or
    map after its element types) and definitions go out in Go's sendType order (a type, then the types
    of its fields / element, depth-first)."""

    def __init__(self):
        self.ids: dict = {}
        self.sent: set = set()
        self.next_id = 65

    @staticmethod
    def _k(t):
        return t if isinstance(t, Struct) else (type(t), _key(t))

    def _alloc(self, t) -> int:
        if isinstance(t, Basic):
            return t.id
        k = self._k(t)
        if k in self.ids:
            return self.ids[k]
        if isinstance(t, Struct):
            self.ids[k] = tid = self.next_id
            self.next_id += 1
            for _, ft in t.fields:
                self._alloc(ft)
            return tid
        if isinstance(t, Slice):
            self._alloc(t.elem)
        elif isinstance(t, Map):
            self._alloc(t.key)
            self._alloc(t.elem)
        else:
            raise TypeError(t)
        self.ids[k] = tid = self.next_id
        self.next_id += 1
        return tid

    def _send(self, t, out: bytearray) -> None:
        if isinstance(t, Basic):
            return
        k = self._k(t)
        if k in self.sent:
            return
        self.sent.add(k)
        tid = self.ids[k]
        body = bytearray()
        # wireType: field 0 ArrayT, 1 SliceT, 2 StructT, 3 MapT
        if isinstance(t, Struct):
            enc_uint(body, 3)                        # StructT
            enc_uint(body, 1)                        # structType.CommonType
            self._common(body, type_name(t), tid)
            enc_uint(body, 1)                        # structType.Field
            enc_uint(body, len(t.fields))
            for name, ft in t.fields:
                enc_uint(body, 1)
                enc_bytes(body, name.encode())
                enc_uint(body, 1)
                enc_int(body, self.ids[self._k(ft)] if not isinstance(ft, Basic) else ft.id)
                enc_uint(body, 0)
            enc_uint(body, 0)                        # end structType
            children = [ft for _, ft in t.fields]
        elif isinstance(t, Slice):
            enc_uint(body, 2)                        # SliceT
            enc_uint(body, 1)
            self._common(body, type_name(t), tid)
            enc_uint(body, 1)
            enc_int(body, self._alloc(t.elem))
            enc_uint(body, 0)
            children = [t.elem]
        else:
            enc_uint(body, 4)                        # MapT
            enc_uint(body, 1)
            self._common(body, type_name(t), tid)
            enc_uint(body, 1)
            enc_int(body, self._alloc(t.key))
            enc_uint(body, 1)
            enc_int(body, self._alloc(t.elem))
            enc_uint(body, 0)
            children = [t.key, t.elem]
        enc_uint(body, 0)                            # end wireType
        msg = bytearray()
        enc_int(msg, -tid)
        msg += body
        enc_uint(out, len(msg))
        out += msg
        for c in children:
            self._send(c, out)

    @staticmethod
    def _common(body: bytearray, name: str, tid: int) -> None:
        enc_uint(body, 1)
        enc_bytes(body, name.encode())
        enc_uint(body, 1)
        enc_int(body, tid)
        enc_uint(body, 0)

    def encode(self, t, value) -> bytes:
        """Messages for one top-level value of schema t (type definitions first, if new)."""
        tid = self._alloc(t)
        out = bytearray()
        self._send(t, out)
        body = bytearray()
        enc_int(body, tid)
        if not isinstance(t, Struct):
            enc_uint(body, 0)   # singleton field
        self._value(body, t, value)
        enc_uint(out, len(body))
        out += body
        return bytes(out)

    def _value(self, out: bytearray, t, v) -> None:
        if t is BOOL:
            enc_uint(out, 1 if v else 0)
        elif t is INT:
            enc_int(out, int(v))
        elif t is UINT:
            enc_uint(out, int(v))
        elif t is FLOAT:
            enc_float(out, float(v))
        elif t is BYTES:
            enc_bytes(out, bytes(v))
        elif t is STRING:
            enc_bytes(out, v.encode())
        elif isinstance(t, Slice):
            enc_uint(out, len(v))
            for x in v:
                self._value(out, t.elem, x)
        elif isinstance(t, Map):
            enc_uint(out, len(v))
            for k, x in v.items():
                self._value(out, t.key, k)
                self._value(out, t.elem, x)
        elif isinstance(t, Struct):
            last = -1
            for i, (name, ft) in enumerate(t.fields):
                x = v.get(name) if isinstance(v, dict) else getattr(v, name, None)
                if _is_zero(ft, x):
                    continue
                enc_uint(out, i - last)
                last = i
                self._value(out, ft, x)
            enc_uint(out, 0)
        else:
            raise TypeError(t)


def _key(t):
    if isinstance(t, Basic):
        return t.id
    if isinstance(t, Struct):
        return id(t)
    if isinstance(t, Slice):
        return ("s", _key(t.elem))
    return ("m", _key(t.key), _key(t.elem))


# ---------------------------------------------------------------------------- decoder
@dataclass
class _Wire:
    kind: str                      # struct | slice | map
    name: str
    fields: list = field(default_factory=list)   # [(name, tid)]
    elem: int = 0
    key: int = 0


class Decoder:
    """One direction of a gob stream: learns the sender's type definitions, decodes values into plain
    Python objects (dict for structs, list for slices, dict for maps, bytes for []byte)."""

    def __init__(self):
        self.types: dict[int, _Wire] = {}

    def feed_message(self, payload: bytes):
        """Decode one message payload; returns None for a type definition, else the value."""
        r = _Reader(payload)
        tid = r.int()
        if tid < 0:
            self.types[-tid] = self._wire(r)
            return None
        if tid not in _BASIC_BY_ID and tid in self.types and self.types[tid].kind == "struct":
            return self._value(r, tid)
        if r.uint() != 0:
            raise ValueError("gob: bad singleton field")
        return self._value(r, tid)

    def _common(self, r: _Reader):
        name, tid = "", 0
        f = -1
        while True:
            d = r.uint()
            if d == 0:
                return name, tid
            f += d
            if f == 0:
                name = r.bytes_().decode()
            elif f == 1:
                tid = r.int()

    def _wire(self, r: _Reader) -> _Wire:
        f = -1
        w = None
        while True:
            d = r.uint()
            if d == 0:
                break
            f += d
            sub = -1
            if f == 1:      # SliceT
                w = _Wire("slice", "")
                while True:
                    dd = r.uint()
                    if dd == 0:
                        break
                    sub += dd
                    if sub == 0:
                        w.name, _ = self._common(r)
                    elif sub == 1:
                        w.elem = r.int()
            elif f == 2:    # StructT
                w = _Wire("struct", "")
                while True:
                    dd = r.uint()
                    if dd == 0:
                        break
                    sub += dd
                    if sub == 0:
                        w.name, _ = self._common(r)
                    elif sub == 1:
                        for _ in range(r.count()):
                            fname, fid, ff = "", 0, -1
                            while True:
                                d3 = r.uint()
                                if d3 == 0:
                                    break
                                ff += d3
                                if ff == 0:
                                    fname = r.bytes_().decode()
                                elif ff == 1:
                                    fid = r.int()
                            w.fields.append((fname, fid))
            elif f == 3:    # MapT
                w = _Wire("map", "")
                while True:
                    dd = r.uint()
                    if dd == 0:
                        break
                    sub += dd
                    if sub == 0:
                        w.name, _ = self._common(r)
                    elif sub == 1:
                        w.key = r.int()
                    elif sub == 2:
                        w.elem = r.int()
            else:
                raise ValueError(f"gob: unsupported wire type field {f}")
        if w is None:
            raise ValueError("gob: empty wire type")
        return w

    def _value(self, r: _Reader, tid: int):
        if tid == 1:
            return r.uint() != 0
        if tid == 2:
            return r.int()
        if tid == 3:
            return r.uint()
        if tid == 4:
            return r.float()
        if tid == 5:
            return r.bytes_()
        if tid == 6:
            return r.bytes_().decode()
        w = self.types[tid]
        if w.kind == "slice":
            n = r.count()
            if w.elem == 4:   # []float64 fast path
                return [r.float() for _ in range(n)]
            return [self._value(r, w.elem) for _ in range(n)]
        if w.kind == "map":
            n = r.count()
            out = {}
            for _ in range(n):
                k = self._value(r, w.key)
                out[k] = self._value(r, w.elem)
            return out
        out = {name: None for name, _ in w.fields}
        f = -1
        while True:
            d = r.uint()
            if d == 0:
                return out
            f += d
            name, ftid = w.fields[f]
            out[name] = self._value(r, ftid)


MAX_MESSAGE = 1 << 30   # Go's decoder refuses messages over 1 GB (tooBig)


def read_message(stream, limit: int = MAX_MESSAGE) -> bytes:
    """One message payload from a binary stream (socket file), or EOFError; messages longer than `limit`
    bytes (or with a length field over 8 bytes) are refused before anything is allocated."""
    first = stream.read(1)
    if not first:
        raise EOFError
    c = first[0]
    if c < 128:
        n = c
    else:
        k = 256 - c
        if k > 8:
            raise ValueError("gob: message length with more than 8 bytes")
        n = int.from_bytes(_read_exact(stream, k), "big")
    if n > limit:
        raise ValueError(f"gob: message of {n} bytes exceeds the {limit}-byte limit")
    return _read_exact(stream, n)


def _read_exact(stream, n: int) -> bytes:
    """n bytes, read in pieces of at most 1 MB: a declared length is only a claim, so memory grows with the
    bytes that actually arrive instead of being reserved up front (a buffered socket file's read(n) allocates
    n bytes at once)."""
    buf = bytearray()
    while len(buf) < n:
        chunk = stream.read(min(n - len(buf), 1 << 20))
        if not chunk:
            raise EOFError("gob: stream ended inside a message")
        buf += chunk
    return bytes(buf)


def split_messages(data: bytes) -> list[bytes]:
    s = io.BytesIO(data)
    out = []
    while True:
        try:
            out.append(read_message(s))
        except EOFError:
            return out


# ---------------------------------------------------------------------------- the reference's types
Share = Struct("Share", (("X", INT), ("Y", INT)))
Update = Struct("Update", (("SourceID", INT), ("Iteration", INT), ("Delta", Slice(FLOAT)), ("Commitment", BYTES),
                           ("Noise", Slice(FLOAT)), ("NoisedDelta", Slice(FLOAT)), ("Accepted", BOOL),
                           ("SignatureList", Slice(BYTES))))
BlockData = Struct("BlockData", (("Iteration", INT), ("GlobalW", Slice(FLOAT)), ("Deltas", Slice(Update))))
Block = Struct("Block", (("Timestamp", INT), ("Data", BlockData), ("PrevBlockHash", BYTES), ("Hash", BYTES),
                         ("StakeMap", Map(INT, INT))))
Blockchain = Struct("Blockchain", (("Blocks", Slice(Block, "[]*main.Block")),))
TCPAddr = Struct("TCPAddr", (("IP", BYTES), ("Port", INT), ("Zone", STRING)))
PolynomialPartRPC = Struct("PolynomialPartRPC", (("Polynomial", Slice(INT, "[]int64")), ("Commitment", BYTES),
                                                 ("Secrets", Slice(Share)), ("Witnesses", Slice(BYTES))))
MinerPartRPC = Struct("MinerPartRPC", (("CommitmentUpdate", BYTES), ("Iteration", INT), ("NodeID", INT),
                                       ("SignatureList", Slice(BYTES)),
                                       ("PolyMap", Map(INT, PolynomialPartRPC, "PolynomialMapRPC"))))
Request = Struct("Request", (("ServiceMethod", STRING), ("Seq", UINT)))
Response = Struct("Response", (("ServiceMethod", STRING), ("Seq", UINT), ("Error", STRING)))
InvalidRequest = Struct("invalidRequest", ())
