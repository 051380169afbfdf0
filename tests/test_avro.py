"""Avro codec: round trips (property-based), framing, nullable unions, malformed input."""
import json
import struct

import numpy as np
import pytest
from hypothesis import given, settings, strategies as st

from streamml.data.avro import AvroCodec, compile_schema, frame, unframe
from streamml.data.cardata import FEATURES

KSQL = AvroCodec("cardata-v1")
SRC = AvroCodec("cardata-v1-source")


def _zz(v):
    z = (v << 1) ^ (v >> 63)
    out = b""
    while z >= 0x80:
        out += bytes([(z & 0x7F) | 0x80])
        z >>= 7
    return out + bytes([z])


def test_schemas_compile():
    f = compile_schema("cardata-v1")
    assert len(f) == 19 and all(x.nullable and x.null_branch == 0 for x in f)
    assert [x.kind for x in f][9:13] == ["int"] * 4 and f[-1].kind == "string"
    g = compile_schema("cardata-v1-source")
    assert len(g) == 18 and not any(x.nullable for x in g)
    assert KSQL.numeric_fields[0] == "COOLANT_TEMP" and KSQL.text_fields == ["FAILURE_OCCURRED"]


def test_decode_matches_hand_encoding():
    # one KSQL record: union branch 1 (non-null) for every field
    body = b""
    vals = []
    for i, fs in enumerate(compile_schema("cardata-v1")):
        body += _zz(1)
        if fs.kind == "double":
            v = 1.5 * i
            body += struct.pack("<d", v)
            vals.append(v)
        elif fs.kind == "int":
            v = 20 + i
            body += _zz(v)
            vals.append(v)
        else:
            body += _zz(5) + b"false"
    out = KSQL.decode([frame(body, 42)])
    np.testing.assert_allclose(out["numeric"][0], np.array(vals, dtype=np.float32))
    assert out["schema_id"][0] == 42 and out["ok"][0] == 1
    assert out["text"]["FAILURE_OCCURRED"] == [b"false"]


def test_nulls_and_malformed():
    rows = np.arange(36, dtype=np.float64).reshape(2, 18)
    nm = np.zeros((2, 18), np.uint8)
    nm[1, 3] = 1
    buf, offs = KSQL.encode(rows, {"FAILURE_OCCURRED": ["true", ""]}, null_mask=nm,
                            text_null={"FAILURE_OCCURRED": np.array([0, 1], np.uint8)}, schema_id=7)
    recs = KSQL.split(buf, offs)
    bad = recs[0][:-3]                       # truncated record
    out = KSQL.decode(recs + [bad, b"\x01garbage"])
    assert list(out["ok"]) == [1, 1, 0, 0] and out["n_errors"] == 2
    assert np.isnan(out["numeric"][1, 3]) and out["null"][1, 3] == 1
    assert out["text"]["FAILURE_OCCURRED"][0] == b"true" and out["text_null"]["FAILURE_OCCURRED"][1] == 1
    with pytest.raises(Exception):
        KSQL.decode(recs + [bad], strict=True)


@settings(max_examples=60, deadline=None)
@given(st.lists(st.tuples(st.lists(st.floats(-1e6, 1e6, allow_nan=False, width=32), min_size=18, max_size=18),
                          st.lists(st.booleans(), min_size=18, max_size=18),
                          st.sampled_from(["true", "false", ""])), min_size=1, max_size=20),
       st.integers(0, 2 ** 31 - 1))
def test_roundtrip_property(rows, sid):
    num = np.array([r[0] for r in rows], dtype=np.float64)
    ints = [i for i, f in enumerate(compile_schema("cardata-v1")) if f.kind == "int"]
    num[:, ints] = np.round(num[:, ints])
    nm = np.array([r[1] for r in rows], dtype=np.uint8)
    text = {"FAILURE_OCCURRED": [r[2] for r in rows]}
    buf, offs = KSQL.encode(num, text, null_mask=nm, schema_id=sid)
    out = KSQL.decode((buf, offs))
    assert (out["ok"] == 1).all() and (out["schema_id"] == sid).all()
    exp = np.where(nm == 1, np.nan, num).astype(np.float32)
    np.testing.assert_array_equal(out["null"], nm)
    np.testing.assert_allclose(out["numeric"], exp, rtol=1e-6, equal_nan=True)
    assert [b.decode() for b in out["text"]["FAILURE_OCCURRED"]] == text["FAILURE_OCCURRED"]


def test_source_schema_float_fields_and_no_framing():
    num = np.random.default_rng(0).uniform(0, 100, size=(50, 18))
    ints = [i for i, f in enumerate(compile_schema("cardata-v1-source")) if f.kind == "int"]
    num[:, ints] = np.round(num[:, ints])
    buf, offs = SRC.encode(num, framing=False)
    out = SRC.decode((buf, offs), framing=False, want_f64=True)
    np.testing.assert_allclose(out["numeric"], num.astype(np.float32), rtol=1e-6)
    assert (out["schema_id"] == -1).all()


def test_frame_unframe():
    assert unframe(frame(b"abc", 258)) == (258, b"abc")
    with pytest.raises(ValueError):
        unframe(b"\x01\x00\x00\x00\x01x")
