"""The LZ4 frame codec of compressed wire messages (csrc/lz4frame.cpp).  The reference holds
no LZ4 fixture and python-lz4 is not in the image, so frames are built here byte by byte from
the published format (test-only builder) and the checksum is pinned by the xxhash package's
xxh32.  Covered: stored and compressed blocks, overlapping matches, linked blocks, block /
content checksums, frames without a content size, corruption errors, the encoder's round
trip, and a compressed Client.append message (test/apex-dqn/worker.py:60) through
pack.deserialize.  Parity with python-lz4's own byte stream: unpinned (no fixture)."""
import struct

import numpy as np
import pytest
import xxhash

from reth_amd import _lib, pack

MAGIC = struct.pack("<I", 0x184D2204)


def _xxh(b):
    return xxhash.xxh32(bytes(b), seed=0).intdigest()


def frame(blocks, content=None, block_checksum=False, content_checksum=False, linked=False, bsid=4):
    """blocks: list of (kind, bytes) with kind 'raw' (stored) or 'lz4' (a compressed block)"""
    flg = 0x40 | (0 if linked else 0x20) | (0x10 if block_checksum else 0) | (0x04 if content_checksum else 0)
    desc = bytes([flg | (0x08 if content is not None else 0), bsid << 4])
    if content is not None:
        desc += struct.pack("<Q", len(content))
    out = MAGIC + desc + bytes([(_xxh(desc) >> 8) & 0xff])
    for kind, b in blocks:
        out += struct.pack("<I", len(b) | (0x80000000 if kind == "raw" else 0)) + b
        if block_checksum:
            out += struct.pack("<I", _xxh(b))
    out += struct.pack("<I", 0)
    if content_checksum:
        out += struct.pack("<I", _xxh(content))
    return out


def seq(lit, off=0, mlen=0):
    """one LZ4 sequence: literals, then (unless last) a match of mlen >= 4 at offset off"""
    ll, ml = len(lit), (mlen - 4 if mlen else 0)
    out = bytes([(min(ll, 15) << 4) | (min(ml, 15) if mlen else 0)])
    if ll >= 15:
        x = ll - 15
        out += b"\xff" * (x // 255) + bytes([x % 255])
    out += lit
    if mlen:
        out += struct.pack("<H", off)
        if ml >= 15:
            x = ml - 15
            out += b"\xff" * (x // 255) + bytes([x % 255])
    return out


def test_xxh32_matches_the_xxhash_package():
    rng = np.random.default_rng(0)
    for n in (0, 1, 3, 4, 15, 16, 17, 33, 1000):
        b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        for seed in (0, 7):
            assert _lib.lib().rth_xxh32(b, n, seed) == xxhash.xxh32(b, seed=seed).intdigest()


def test_stored_and_compressed_blocks_with_checksums():
    a = b"hello, ape-x! " * 3
    blk = seq(b"abcd", 4, 20) + seq(b"xyz")  # the match repeats "abcd" (overlapping copy)
    want_blk = b"abcd" * 6 + b"xyz"
    content = a + want_blk
    f = frame([("raw", a), ("lz4", blk)], content=content, block_checksum=True, content_checksum=True)
    assert bytes(pack.lz4_decompress(f)) == content


def test_run_length_offset_one_and_long_lengths():
    lit = bytes(range(40))  # a literal run > 15
    blk = seq(lit, 1, 300) + seq(b"end!!")  # offset 1: repeat the last byte 300 times
    want = lit + bytes([39]) * 300 + b"end!!"
    assert bytes(pack.lz4_decompress(frame([("lz4", blk)]))) == want  # no content size: bound by blocks


def test_linked_blocks_reach_into_the_previous_block():
    b1 = seq(b"0123456789abcdef")
    b2 = seq(b"", 16, 16) + seq(b"!")  # the second block copies the whole first one
    want = b"0123456789abcdef" * 2 + b"!"
    assert bytes(pack.lz4_decompress(frame([("lz4", b1), ("lz4", b2)], content=want, linked=True))) == want


@pytest.mark.parametrize("break_", ["magic", "header", "content", "offset", "block"])
def test_corruption_is_an_error(break_):
    content = b"abcdabcdabcd--"
    blk = seq(b"abcd", 4, 8) + seq(b"--")
    f = bytearray(frame([("lz4", blk)], content=content, content_checksum=True, block_checksum=True))
    if break_ == "magic":
        f[0] ^= 1
    elif break_ == "header":
        f[6] ^= 1  # content size byte: the header checksum no longer matches
    elif break_ == "content":
        f[-1] ^= 1
    elif break_ == "block":
        f[-9 - 4 - 1] ^= 1  # last byte of the block body: its block checksum mismatches
    else:
        bad = seq(b"ab", 9, 4) + seq(b"x")  # offset past the produced output
        f = bytearray(frame([("lz4", bad)]))
    with pytest.raises(_lib.RethHipError):
        pack.lz4_decompress(bytes(f))


@pytest.mark.parametrize("n", [0, 1, 13, 5000, 300_000])
def test_encoder_round_trip(n):
    rng = np.random.default_rng(n)
    # compressible: repeated frames with noise (what the apex rows look like)
    base = rng.integers(0, 256, 97, dtype=np.uint8)
    data = np.resize(base, n)
    data[rng.random(n) < 0.05] = 7
    raw = data.tobytes()
    f = pack.lz4_compress(raw)
    assert bytes(pack.lz4_decompress(f)) == raw
    if n >= 5000:
        assert len(f) < len(raw) // 2
    noise = rng.integers(0, 256, n, dtype=np.uint8).tobytes()  # incompressible: a stored block
    assert bytes(pack.lz4_decompress(pack.lz4_compress(noise))) == noise


def test_compressed_append_message_round_trip():
    """Client.append(buffer.data, loss, compress=True) as worker.py:60 sends it"""
    rng = np.random.default_rng(3)
    n = 16
    s0 = rng.integers(0, 256, (n, 4, 84, 84)).astype(np.float32)
    cols = [s0, rng.integers(0, 6, n).astype(np.int64), rng.random(n).astype(np.float32), s0[::-1].copy(),
            np.zeros(n, np.float32)]
    rows = [pack.serialize([np.asarray(c[i]) for c in cols]) for i in range(n)]
    loss = rng.random(n).astype(np.float32)
    msg = pack.serialize([rows, loss], compress=True)
    plain = pack.serialize([rows, loss])
    assert len(msg) < len(plain)
    header, _ = pack.read_header(msg)
    assert header[pack.KEY_COMPRESS] is True
    got_rows, got_loss = pack.deserialize(msg)
    np.testing.assert_array_equal(got_loss, loss)
    for i, r in enumerate(got_rows):
        for c, x in zip(cols, pack.deserialize(bytes(r))):
            np.testing.assert_array_equal(x, c[i])
