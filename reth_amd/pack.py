"""The reth_buffer wire format, and the ingest of an append message into an HBM replay.

Reference: reth_buffer/reth_buffer/utils/pack.py:60-164 (serialize / deserialize /
read_header), client/client.py:21-35 (Client.append's message) and
server/main_loop.py:21-61 (append_loop, which stores each row message in LMDB).

A message is
    [4-byte big-endian header length][msgpack header][body]
with header = {"meta": ..., "body_len": n, "time": t} (plus KEY_COMPRESS when the body is
an LZ4 frame: csrc/lz4frame.cpp restates the frame format, no lz4 library is in the image).  `meta` mirrors the serialized object: lists / dicts recurse; an ndarray
becomes {KEY_NUMPY: True, "header": numpy .npy header dict, "raw_size", "offset",
"length"} pointing into the body; bytes-like objects become {KEY_BYTES: True, ...}.

Client.append sends serialize([rows, weights]) where every row is itself a message of the
row's column slices.  `ingest_append` below puts such a message into an HbmReplay without
materialising rows on the host: the body goes to the device in one copy and every column
is appended straight out of it (rows are equally spaced in the body when their headers
have equal length -- always, for fixed-shape columns), float32 frames are narrowed to the
replay's uint8 storage by the copy kernel.
"""
import ctypes
import time

import msgpack
import numpy as np
import torch

KEY_COMPRESS = "reth_compress_953531b51ab8"
KEY_NUMPY = "reth_numpy_356b759ef2b3"
KEY_BYTES = "reth_bytes_a32b00c47e72"


def _walk_out(obj, chunks, pos):
    """meta for obj; appends body chunks; pos = [current body offset]"""
    if isinstance(obj, (list, tuple)):
        return [_walk_out(x, chunks, pos) for x in obj]
    if isinstance(obj, dict):
        return {k: _walk_out(v, chunks, pos) for k, v in obj.items()}
    if isinstance(obj, np.ndarray):
        # the body carries the elements in C order even for a Fortran-ordered array whose
        # header says fortran_order=True -- what the reference writes (its bytearray copy of
        # the array's buffer), so its deserialize returns such arrays transposed-scrambled;
        # kept byte-for-byte
        c = np.ascontiguousarray(obj)
        mv = memoryview(c).cast("B") if c.ndim else memoryview(c.tobytes())
        entry = {KEY_NUMPY: True, "header": np.lib.format.header_data_from_array_1_0(obj), "raw_size": obj.nbytes}
        entry["offset"], entry["length"] = pos[0], mv.nbytes
        chunks.append(mv)
        pos[0] += mv.nbytes
        return entry
    if isinstance(obj, (bytes, bytearray, memoryview)):
        mv = memoryview(obj)
        entry = {KEY_BYTES: True, "raw_size": mv.nbytes, "offset": pos[0], "length": mv.nbytes}
        chunks.append(mv.cast("B") if mv.ndim != 1 or mv.format != "B" else mv)
        pos[0] += mv.nbytes
        return entry
    return obj


def _u8(buf):
    """a uint8 ndarray over a host buffer (bytes / bytearray / memoryview), no copy"""
    return np.frombuffer(buf, dtype=np.uint8)


def lz4_compress(data):
    """lz4.frame.compress (pack.py:67): an LZ4 frame of `data` (csrc/lz4frame.cpp)"""
    from ._lib import call, lib

    src = _u8(data)
    out = np.empty(lib().rth_lz4_frame_compress_bound(src.size), dtype=np.uint8)
    m = ctypes.c_int64()
    call("rth_lz4_frame_compress", src.ctypes.data if src.size else None, src.size, out.ctypes.data, out.size,
         ctypes.byref(m))
    return bytearray(out[:m.value])


def lz4_decompress(frame):
    """lz4.frame.decompress (pack.py:157): the content of an LZ4 frame, as a bytearray"""
    from ._lib import call

    src = _u8(frame)
    bound = ctypes.c_int64()
    call("rth_lz4_frame_bound", src.ctypes.data, src.size, ctypes.byref(bound))
    out = bytearray(bound.value)
    view = _u8(out)
    m = ctypes.c_int64()
    call("rth_lz4_frame_decompress", src.ctypes.data, src.size, view.ctypes.data if view.size else None, view.size,
         ctypes.byref(m))
    del view  # release the export before trimming
    del out[m.value:]
    return out


def serialize(data, compress=False):
    """pack.py:60-98; compress=True puts the body into an LZ4 frame and marks the header
    (the frame bytes differ from python-lz4's encoder -- any LZ4 decoder reads both)"""
    chunks, pos = [], [0]
    meta = _walk_out(data, chunks, pos)
    if compress:
        raw = bytearray(pos[0])
        o = 0
        for c in chunks:
            raw[o:o + c.nbytes] = c
            o += c.nbytes
        body = lz4_compress(raw)
        header = msgpack.packb({KEY_COMPRESS: True, "meta": meta, "body_len": len(body), "time": time.time()})
        chunks, pos = [memoryview(body)], [len(body)]
    else:
        header = msgpack.packb({"meta": meta, "body_len": pos[0], "time": time.time()})
    out = bytearray(4 + len(header) + pos[0])
    out[:4] = len(header).to_bytes(4, "big")
    out[4:4 + len(header)] = header
    o = 4 + len(header)
    for c in chunks:
        out[o:o + c.nbytes] = c
        o += c.nbytes
    return out


def read_header(data):
    """pack.py:140-144: (header dict, header length)"""
    view = memoryview(data)
    hlen = int.from_bytes(view[:4], "big")
    return msgpack.unpackb(view[4:4 + hlen]), hlen


def _array_from(body, entry):
    h = entry["header"]
    dt = np.lib.format.descr_to_dtype(h["descr"])
    shape = tuple(h["shape"])
    arr = np.frombuffer(body[entry["offset"]:entry["offset"] + entry["length"]], dtype=dt)
    if h["fortran_order"]:
        arr = arr.reshape(shape[::-1]).transpose()
    else:
        arr = arr.reshape(shape)
    assert arr.nbytes == entry["raw_size"]
    return arr


def _walk_in(meta, body):
    if isinstance(meta, (list, tuple)):
        return [_walk_in(x, body) for x in meta]
    if isinstance(meta, dict):
        if KEY_NUMPY in meta:
            return _array_from(body, meta)
        if KEY_BYTES in meta:
            part = body[meta["offset"]:meta["offset"] + meta["length"]]
            assert part.nbytes == meta["raw_size"]
            return part
        return {k: _walk_in(v, body) for k, v in meta.items()}
    return meta


def deserialize(data):
    """pack.py:147-164 (views into `data`, like the reference; a compressed body is
    decompressed first and the views point into that copy)"""
    header, hlen = read_header(data)
    body = memoryview(data)[4 + hlen:]
    assert body.nbytes == header["body_len"]
    if header.get(KEY_COMPRESS):
        body = memoryview(lz4_decompress(body))
    return _walk_in(header["meta"], body)


def _row_layout(body, rows_meta):
    """(first row's column entries, byte offset of row 0's body, row stride) when every row
    message has the same layout; None otherwise"""
    offs, first, stride = [], None, None
    for k, r in enumerate(rows_meta):
        if not (isinstance(r, dict) and KEY_BYTES in r):
            return None
        offs.append(r["offset"])
        if k == 0:
            msg = body[r["offset"]:r["offset"] + r["length"]]
            hdr, hlen = read_header(msg)
            first = (hdr["meta"], r["offset"] + 4 + hlen, r["length"])
    if len(offs) > 1:
        d = np.diff(np.asarray(offs))
        if not np.all(d == d[0]) or d[0] != first[2]:
            return None
        stride = int(d[0])
    else:
        stride = first[2]
    # equal header length for every row: check the last one too
    last = rows_meta[-1]
    _, hlen_last = read_header(body[last["offset"]:last["offset"] + last["length"]])
    if 4 + hlen_last != first[1] - rows_meta[0]["offset"]:
        return None
    return first[0], first[1], stride


def ingest_append(replay, message, staging=None):
    """append_loop for one Client.append message: rows into `replay` (an HbmReplay whose
    columns match the row columns; float32 columns may land in uint8 storage), priorities =
    the message's weights.  Returns the number of rows."""
    header, hlen = read_header(message)
    body = memoryview(message)[4 + hlen:]
    if header.get(KEY_COMPRESS):  # worker.py:60 sends compress=True: decompress on the host first
        body = memoryview(lz4_decompress(body))
        staging = None
    rows_meta, w_meta = header["meta"]
    weights = _array_from(body, w_meta)
    n = len(rows_meta)
    assert n == len(weights)
    if n == 0:
        return 0
    dev = replay.device
    layout = _row_layout(body, rows_meta)
    if layout is None:  # unequal rows: rebuild columns on the host
        rows = [deserialize(body[r["offset"]:r["offset"] + r["length"]]) for r in rows_meta]
        cols = [torch.as_tensor(np.stack([row[c] for row in rows])) for c in range(len(rows[0]))]
        return replay.append(cols, torch.as_tensor(weights).to(dev))
    col_meta, base, stride = layout
    # one host->device copy of the body; every column is appended from it in place
    src = torch.frombuffer(bytearray(body) if staging is None else staging, dtype=torch.uint8)
    dbody = src.to(dev, non_blocking=False)
    cols, strides = [], []
    for c, e in enumerate(col_meta):
        h = e["header"]
        dt = np.lib.format.descr_to_dtype(h["descr"])
        if h["fortran_order"] and len(h["shape"]) > 1:
            raise ValueError("Fortran-ordered row arrays are not supported by the device ingest")
        tdt = {np.dtype("uint8"): torch.uint8, np.dtype("int32"): torch.int32, np.dtype("int64"): torch.int64,
               np.dtype("float32"): torch.float32, np.dtype("float64"): torch.float64}[dt]
        # a strided view over the body: row i of column c at base + i * stride + offset
        start = base + e["offset"]
        elems = e["length"] // dt.itemsize
        view = dbody[start:start + (n - 1) * stride + e["length"]]
        cols.append(_BodyColumn(view, tdt, elems))
        strides.append(stride)
    w = torch.as_tensor(np.array(weights)).to(dev)  # (a copy: the message buffer is read-only)
    return replay.append_strided(cols, w, strides)


class _BodyColumn:
    """a column living inside a device copy of a message body (rows `stride` bytes apart)"""

    def __init__(self, view, dtype, row_elems):
        self.view, self.dtype, self.row_elems = view, dtype, row_elems
