"""GPU parity of the SDK-side entry points: the whole SendMessages body
(SendMessagesEncoder::encode, send_messages.rs:89-181) with its batch encoded on
the device, PolledMessages::from_bytes (polled_messages.rs:61-90) and the
producer's buffering / flush (producer_sharding.rs:136-247, producer.rs:406-470),
each against the reference's golden vectors and the oracle (oracle/sdk_ref.py +
the C restatement's encoder). Byte work: every check is exact."""
import numpy as np
import pytest

from golden_util import reference_vectors
from iggy_amd import abi
from iggy_amd.codec import Producer, raw_messages
from oracle import oracle as O
from oracle import sdk_ref as S

pytestmark = pytest.mark.gpu

GOLDEN_METADATA = bytes.fromhex("120000000104010000000104020000000100" + "02000000")


@pytest.fixture(scope="module")
def cx():
    from iggy_amd.codec import Codec
    c = Codec(0)
    yield c
    c.close()


def _msgs(n, pl_lo, pl_hi, uh_max=0, seed=0, ts0=1_700_000_000_000_000, ts_jitter=1000):
    rng = np.random.default_rng(seed)
    pls = rng.integers(pl_lo, pl_hi + 1, n).astype(np.uint32)
    uhl = rng.integers(0, uh_max + 1, n).astype(np.uint32) if uh_max else np.zeros(n, np.uint32)
    ids = rng.integers(1, 2**63, 2 * n, dtype=np.uint64)
    ots = (ts0 + rng.integers(0, ts_jitter, n)).astype(np.uint64)
    pay = rng.integers(0, 256, int(pls.sum()), dtype=np.uint8)
    uhs = rng.integers(0, 256, int(uhl.sum()), dtype=np.uint8)
    return dict(ids=ids, ots=ots, pay=pay, pls=pls, uhs=uhs, uhl=uhl)


def _raw(m, with_uh=True):
    return raw_messages(m["ids"], m["ots"], m["pay"], m["pls"], m["uhs"] if with_uh else None,
                        m["uhl"] if with_uh else None)


def _slice(m, a, b):
    po = np.concatenate([[0], np.cumsum(m["pls"], dtype=np.uint64)]).astype(np.int64)
    uo = np.concatenate([[0], np.cumsum(m["uhl"], dtype=np.uint64)]).astype(np.int64)
    return dict(ids=m["ids"][2 * a:2 * b].copy(), ots=m["ots"][a:b].copy(), pay=m["pay"][po[a]:po[b]].copy(),
                pls=m["pls"][a:b].copy(), uhs=m["uhs"][uo[a]:uo[b]].copy(), uhl=m["uhl"][a:b].copy())


def _oracle_body(stream, topic, part, m):
    rc, e, batch = O.encode_batch(_raw(m))
    assert rc == 0, e
    return S.send_messages_body(stream, topic, part, batch, len(m["pls"]))


def _hdr(stream, topic, part):
    h = abi.SendMessagesHeader()
    h.stream_id, h.topic_id, h.partitioning = abi.Identifier.raw(*stream), abi.Identifier.raw(*topic), \
        abi.Partitioning.raw(*part)
    return h


def _send(cx, h, raw, cap=None):
    import ctypes
    need = cx._L.iggy_send_messages_encoded_size(ctypes.byref(h), ctypes.byref(raw)) if raw.count else 1024
    out = np.zeros(cap if cap is not None else need, dtype=np.uint8)
    n = ctypes.c_uint64(0)
    e = abi.WireError()
    rc = cx._L.iggy_codec_send_messages_encode(cx.handle, ctypes.byref(h), ctypes.byref(raw), out.ctypes.data,
                                               out.size, ctypes.byref(n), ctypes.byref(e))
    return rc, e, out[: n.value].tobytes()


NUM1 = (S.ID_NUMERIC, (1).to_bytes(4, "little"))
NUM2 = (S.ID_NUMERIC, (2).to_bytes(4, "little"))
BAL = (S.PART_BALANCED, b"")


def test_golden_send_messages_body(cx):
    """message-batch.test.ts:47-60 + :98-112: metadata prefix and the Rust produce batch."""
    ref = reference_vectors()
    ms = ref["messages"]
    m = dict(ids=np.array([[x["id"], 0] for x in ms], np.uint64).reshape(-1),
             ots=np.array([x["origin_timestamp"] for x in ms], np.uint64),
             pay=np.frombuffer(b"".join(x["payload"].encode() for x in ms), np.uint8).copy(),
             pls=np.array([len(x["payload"]) for x in ms], np.uint32),
             uhs=np.frombuffer(b"".join(x["user_headers"].encode() for x in ms), np.uint8).copy(),
             uhl=np.array([len(x["user_headers"]) for x in ms], np.uint32))
    rc, e, body = _send(cx, _hdr(NUM1, NUM2, BAL), _raw(m))
    assert rc == 0, e
    assert body == GOLDEN_METADATA + bytes.fromhex(ref["produce_batch_hex"])


@pytest.mark.parametrize("shape", [(1, 0, 0, 0), (100, 0, 300, 0), (2000, 64, 4096, 0), (500, 0, 100, 40),
                                   (300_000, 0, 64, 0)])
def test_send_messages_body_matches_oracle(cx, shape):
    n, lo, hi, uh = shape
    m = _msgs(n, lo, hi, uh, seed=n)
    stream, topic = (S.ID_STRING, b"orders"), NUM2
    part = (S.PART_MESSAGES_KEY, b"customer-42")
    rc, e, body = _send(cx, _hdr(stream, topic, part), _raw(m))
    assert rc == 0, e
    assert body == _oracle_body(stream, topic, part, m)
    # the body decodes as the server reads it (send_messages.rs:286-299)
    ml = int.from_bytes(body[:4], "little")
    err, dec, used = S.decode_metadata(body[4:4 + ml])
    assert err is None and used == ml and dec[3] == n
    rc2, e2, h2, frames = O.decode_batch_slice_with(np.frombuffer(body[4 + ml:], np.uint8).copy())
    assert rc2 == 0 and h2.message_count == n


def test_send_messages_errors(cx):
    m = _msgs(3, 1, 5)
    h = _hdr(NUM1, NUM2, BAL)
    empty = abi.RawMessages(0, None, None, None, None, None, None)
    rc, e, _ = _send(cx, h, empty)
    assert (rc, e.kind, e.reason) == (abi.ERR_VALIDATION,) * 2 + (abi.V_EMPTY_BATCH,)
    m["ots"][2] = m["ots"][0] + 2**32 + 5  # delta past u32 (send_messages.rs:132-135)
    m["ots"][1] = m["ots"][0]
    rc, e, _ = _send(cx, h, _raw(m))
    assert rc == abi.ERR_INVALID_TIMESTAMP_DELTA and e.a == 2**32 + 5
    rc, e, _ = _send(cx, h, _raw(_msgs(3, 1, 5)), cap=40)
    assert rc == abi.ERR_CAPACITY


def test_polled_messages_from_bytes_golden(cx):
    """message-batch.test.ts:62-75 / :114-140: prefix 3/101/2, two messages resolved."""
    import ctypes
    ref = reference_vectors()
    body = np.frombuffer(bytes.fromhex(ref["poll_body_hex"]), np.uint8).copy()
    out = (abi.PolledMessage * 8)()
    pf = abi.PolledPrefix()
    n = ctypes.c_uint64(0)
    e = abi.WireError()
    rc = cx._L.iggy_codec_polled_messages_from_bytes(cx.handle, body.ctypes.data, body.size, ctypes.byref(pf),
                                                     out, 8, ctypes.byref(n), ctypes.byref(e))
    assert rc == 0, e
    assert (pf.partition_id, pf.current_offset, pf.count) == (3, 101, 2)
    assert n.value == 2
    raw = body.tobytes()
    for i, x in enumerate(ref["messages"]):
        pm = out[i]
        assert (pm.id_lo, pm.offset, pm.timestamp, pm.origin_timestamp, pm.checksum) == \
            (x["id"], x["offset"], x["timestamp"], x["origin_timestamp"], x["checksum"])
        assert raw[pm.payload_pos:pm.payload_pos + pm.payload_length] == x["payload"].encode()
        assert raw[pm.user_headers_pos:pm.user_headers_pos + pm.user_headers_length] == x["user_headers"].encode()
    # short prefix -> InvalidNumberEncoding; a broken record -> InvalidMessagePayloadLength
    rc = cx._L.iggy_codec_polled_messages_from_bytes(cx.handle, body.ctypes.data, 15, ctypes.byref(pf), out, 8,
                                                     ctypes.byref(n), ctypes.byref(e))
    assert rc == abi.ERR_INVALID_NUMBER_ENCODING
    bad = body.copy()
    bad[16 + 256 + 40] = 1
    rc = cx._L.iggy_codec_polled_messages_from_bytes(cx.handle, bad.ctypes.data, bad.size, ctypes.byref(pf), out, 8,
                                                     ctypes.byref(n), ctypes.byref(e))
    assert rc == abi.ERR_INVALID_MESSAGE_PAYLOAD_LENGTH


def _run_producer(cx, calls, direct, batch_length=0, batch_size=0):
    """calls: [(stream, topic, part, msgs dict)] -> checks flush against the oracle."""
    p = Producer(cx, batch_length=batch_length, batch_size=batch_size, direct=direct)
    dues, nbytes = [], 0
    for k, (st, tp, pt, m) in enumerate(calls):
        due = p.append(abi.Identifier.raw(*st), abi.Identifier.raw(*tp), abi.Partitioning.raw(*pt), _raw(m))
        nbytes += S.shard_message_size(st, tp, m["pls"], m["uhl"])
        dues.append(due)
        assert due == (True if direct else S.flush_due(k + 1, nbytes, batch_length, batch_size))
    ent, b, msgs = p.pending()
    assert (ent, b) == (len(calls), nbytes)
    # oracle: plan over the concatenated message list
    entries, m0 = [], 0
    for st, tp, pt, m in calls:
        entries.append(((st, tp, pt), m0, m0 + len(m["pls"])))
        m0 += len(m["pls"])
    plan = S.plan_requests(entries, direct, batch_length)
    allm = {k: np.concatenate([c[3][k] for c in calls]) for k in calls[0][3]}
    cap = 400 * len(plan) + sum(len(c[3]["pay"]) + len(c[3]["uhs"]) + 48 * len(c[3]["pls"]) for c in calls)
    rc, e, out, reqs = p.flush(cap=cap)
    assert rc == 0, e
    assert len(reqs) == len(plan)
    raw = out.tobytes()
    for rq, (k, a, b2) in zip(reqs, plan):
        st, tp, pt = entries[k][0]
        assert (rq.entry, rq.first_message, rq.messages) == (k, a, b2 - a)
        if not rq.sent:
            continue
        sub = _slice(allm, a, b2)
        exp_rc, exp_e, batch = O.encode_batch(_raw(sub))
        assert rq.error.kind == exp_rc, (rq.error, exp_e)
        if exp_rc == 0:
            assert raw[rq.offset:rq.offset + rq.length] == S.send_messages_body(st, tp, pt, batch, b2 - a)
    assert p.pending()[:2] == (0, 0)
    p.close()
    return reqs


def test_producer_background_merges_same_destination(cx):
    a = ((S.ID_STRING, b"orders"), NUM2, BAL)
    b = ((S.ID_STRING, b"orders"), NUM2, (S.PART_PARTITION_ID, (3).to_bytes(4, "little")))
    calls = [(*a, _msgs(10, 0, 200, seed=1)), (*a, _msgs(1000, 64, 1100, seed=2)), (*b, _msgs(7, 5, 9, 20, seed=3)),
             (*a, _msgs(300, 0, 50, seed=4)), (*a, _msgs(2, 1, 1, seed=5))]
    reqs = _run_producer(cx, calls, direct=False, batch_length=5)
    assert [r.messages for r in reqs] == [1010, 7, 302]


def test_producer_background_size_trigger_and_many_requests(cx):
    # 20 alternating destinations: more requests than the context's 8 asynchronous slots
    dests = [((S.ID_NUMERIC, (s % 2).to_bytes(4, "little")), NUM1, BAL) for s in range(20)]
    calls = [(*d, _msgs(50 + 10 * i, 0, 2000, seed=10 + i)) for i, d in enumerate(dests)]
    _run_producer(cx, calls, direct=False, batch_size=150_000)


def test_producer_direct_chunks_and_failed_tail(cx):
    a = (NUM1, NUM2, (S.PART_MESSAGES_KEY, b"k"))
    good = _msgs(2500, 0, 300, seed=7)
    bad = _msgs(900, 10, 20, seed=8)
    bad["ots"][:] = bad["ots"][0]
    bad["ots"][450] += 2**32  # chunk 1 (of 300) fails: chunks 2.. are not sent (producer.rs:446-452)
    reqs = _run_producer(cx, [(*a, good), (*a, bad), (*a, _msgs(5, 1, 3, seed=9))], direct=True, batch_length=300)
    per = [(r.entry, r.sent, r.error.kind) for r in reqs]
    assert per[:9] == [(0, 1, 0)] * 9
    assert per[9:12] == [(1, 1, 0), (1, 1, abi.ERR_INVALID_TIMESTAMP_DELTA), (1, 0, 0)]
    assert per[12] == (2, 1, 0)
