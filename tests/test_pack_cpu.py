"""The reth_buffer wire format (utils/pack.py) against messages the reference itself
produced (tests/golden/pack.npz, time.time() pinned): byte-identical serialize, and
deserialize of the reference's messages."""
import types

import numpy as np
import pytest


@pytest.fixture
def pinned_time(monkeypatch):
    from reth_amd import pack

    monkeypatch.setattr(pack, "time", types.SimpleNamespace(time=lambda: 1234.5))
    return pack


def test_append_message_bytes_and_rows(golden, pinned_time):
    pack = pinned_time
    g = golden("pack.npz")
    msg = g["app_msg"].tobytes()
    cols = [g["app_s0"], g["app_a"], g["app_r"], g["app_s1"], g["app_done"]]
    rows, w = pack.deserialize(msg)
    assert np.array_equal(w, g["app_w"]) and w.dtype == np.float32
    assert len(rows) == len(w)
    for i, row in enumerate(rows):
        vals = pack.deserialize(row)
        for c, v in enumerate(vals):
            assert v.dtype == cols[c].dtype and np.array_equal(v, cols[c][i, ...])
    ours = pack.serialize([[pack.serialize([c[i, ...] for c in cols]) for i in range(len(w))], g["app_w"]])
    assert bytes(ours) == msg


def test_generic_object_roundtrip(golden, pinned_time):
    pack = pinned_time
    g = golden("pack.npz")
    msg = g["obj_msg"].tobytes()
    obj = pack.deserialize(msg)
    assert np.array_equal(obj["x"][0], g["obj_x0"]) and bytes(obj["x"][1]) == b"raw-bytes"
    assert obj["x"][2:] == [3, "s", 2.5] and obj["e"] == [[], {}]
    # the reference writes a Fortran array's elements in C order under a fortran_order=True
    # header, so its own deserialize returns them scrambled; ours returns the same array
    f = g["obj_f"]
    assert np.array_equal(obj["f"], np.ascontiguousarray(f).ravel().reshape(f.shape[::-1]).T)
    assert obj["z"].shape == () and obj["z"] == 7.0
    again = {"x": [g["obj_x0"], b"raw-bytes", 3, "s", 2.5], "f": np.asfortranarray(g["obj_f"]),
             "z": np.array(7.0, "f8"), "e": [[], {}]}
    assert bytes(pack.serialize(again)) == msg


def test_update_message(golden, pinned_time):
    pack = pinned_time
    g = golden("pack.npz")
    idx, w, step = pack.deserialize(g["upd_msg"].tobytes())
    assert np.array_equal(idx, np.arange(5)) and np.array_equal(w, g["app_w"][:5]) and step is True
    header, _ = pack.read_header(g["upd_msg"].tobytes())
    assert header["time"] == 1234.5 and header["body_len"] == idx.nbytes + w.nbytes
    # compress=True: an LZ4-frame body (csrc/lz4frame.cpp; tests/test_lz4_cpu.py), same object back
    idx2, w2, step2 = pack.deserialize(pack.serialize([idx, w, step], compress=True))
    assert np.array_equal(idx2, idx) and np.array_equal(w2, w) and step2 is True
