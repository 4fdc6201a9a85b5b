"""Native control plane: wire format, priority queue, TCP / in-process communicators,
compression.  Mirrors the reference's message model (include/pipeline/message.hpp,
binary_serializer.hpp) — the reference has no tests for it."""
import struct
import time

import numpy as np
import pytest
import torch

from dcnn_amd.ops._ext import native
from dcnn_amd.parallel.pipeline import messages as M

comm = native().comm
C = M.CommandType


def test_command_order_matches_reference():
    names = ["_START", "FORWARD_JOB", "BACKWARD_JOB", "UPDATE_PARAMETERS", "TRAIN_MODE", "EVAL_MODE", "SHUTDOWN",
             "CONFIG_TRANSFER", "CONFIG_RECEIVED", "LOAD_PARAMS", "PARAMS_LOADED", "SEND_PARAMS", "PARAMS_TRANSFER",
             "STATUS_REQUEST", "STATUS_RESPONSE", "PARAMETERS_UPDATED", "HEALTH_CHECK", "ERROR_REPORT",
             "JOB_FAILURE", "BARRIER_SYNC", "CHECKPOINT_REQUEST", "CHECKPOINT_COMPLETE", "UPDATE_LOAD",
             "REPORT_LOAD", "LOAD_REPORT", "PRINT_PROFILING", "PROFILING_PRINTED", "CLEAR_PROFILING",
             "PROFILING_CLEARED"]
    assert [C[n].value for n in names] == list(range(len(names)))


def test_legacy_job_wire_layout():
    """Byte-exact reference framing: u8 ver | u8 endian | u64 len | strings | u16 cmd | u64 type | job."""
    a = np.arange(6, dtype=np.float32).reshape(2, 3)
    m = comm.Message("stage_1", int(C.FORWARD_JOB))
    m.set_tensor(9, a, legacy=True)
    b = comm.serialize(m)
    assert b[0] == 1 and b[1] == 1
    (blen,) = struct.unpack_from("<Q", b, 2)
    assert blen == len(b) - 10
    off = 10
    (n,) = struct.unpack_from("<Q", b, off)
    assert b[off + 8:off + 8 + n] == b"stage_1"
    off += 8 + n
    (n,) = struct.unpack_from("<Q", b, off)
    off += 8 + n
    cmd, ptype, mb, nd = struct.unpack_from("<HQQQ", b, off)
    assert (cmd, ptype, mb, nd) == (int(C.FORWARD_JOB), 1, 9, 2)
    off += 2 + 24
    assert struct.unpack_from("<QQ", b, off) == (2, 3)
    np.testing.assert_array_equal(np.frombuffer(b[off + 16:], dtype=np.float32), a.reshape(-1))
    r = comm.deserialize(b)
    assert r.mb_id == 9 and list(r.shape) == [2, 3]
    np.testing.assert_array_equal(np.frombuffer(r, dtype=np.float32).reshape(2, 3), a)


@pytest.mark.parametrize("kind", ["text", "flag", "load", "none"])
def test_scalar_payload_roundtrip(kind):
    m = comm.Message("coordinator", int(C.STATUS_RESPONSE))
    if kind == "text":
        m.text = b"hello \x00 world"
    elif kind == "flag":
        m.flag = True
    elif kind == "load":
        m.load = (1.5, 2.5, 0.25, 100.0)
    r = comm.deserialize(comm.serialize(m))
    assert r.payload_type == m.payload_type
    if kind == "text":
        assert r.text == b"hello \x00 world"
    if kind == "flag":
        assert r.flag is True
    if kind == "load":
        assert r.load == pytest.approx((1.5, 2.5, 0.25, 100.0))


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("codec", ["none", "zlib", "zstd"])
def test_typed_job_roundtrip(dtype, codec):
    if codec == "zstd" and not comm.zstd_available():
        pytest.skip("libzstd not present")
    t = torch.randn(2, 5, 4, 3).to(dtype).contiguous(memory_format=torch.channels_last)
    m = M.job_message("x", C.FORWARD_JOB, 3, t, codec)
    r = comm.deserialize(comm.serialize(m))
    back = M.message_tensor(r)
    assert back.dtype == dtype and tuple(back.shape) == (2, 5, 4, 3)
    assert back.is_contiguous(memory_format=torch.channels_last)
    assert torch.equal(back, t)


def test_truncated_frame_rejected():
    m = comm.Message("a", int(C.FORWARD_JOB))
    m.set_tensor(0, np.ones(10, np.float32), legacy=True)
    b = comm.serialize(m)
    with pytest.raises(Exception):
        comm.deserialize(b[:-4])


def test_priority_queue_order():
    a = comm.InProcessCommunicator("tq_a")
    b = comm.InProcessCommunicator("tq_b")
    try:
        for c in (C.SHUTDOWN, C.BACKWARD_JOB, C.UPDATE_PARAMETERS, C.FORWARD_JOB, C.BACKWARD_JOB):
            a.send(comm.Message("tq_b", int(c)))
        got = [b.recv(100).command for _ in range(5)]
        assert got == [C.FORWARD_JOB, C.BACKWARD_JOB, C.BACKWARD_JOB, C.UPDATE_PARAMETERS, C.SHUTDOWN]
        assert b.recv(10) is None
        assert b.messages_received == 5
    finally:
        a.close()
        b.close()


def test_inprocess_alias_and_unknown_recipient():
    a = comm.InProcessCommunicator("al_a")
    b = comm.InProcessCommunicator("al_b")
    try:
        a.alias("next_stage", "al_b")
        a.send(comm.Message("next_stage", int(C.TRAIN_MODE)))
        m = b.recv(100)
        assert m.command == C.TRAIN_MODE and m.sender == "al_a"
        with pytest.raises(Exception):
            a.send(comm.Message("nobody", int(C.TRAIN_MODE)))
    finally:
        a.close()
        b.close()


def test_tcp_roundtrip_and_large_payload():
    s = comm.TcpCommunicator("srv", "127.0.0.1", 0)
    c = comm.TcpCommunicator("cli", "127.0.0.1", 0)
    try:
        c.connect("server", "127.0.0.1", s.port, 5000)
        assert s.wait_for_peer("cli", 5000)
        big = torch.randn(64, 128, 8, 8)
        c.send(M.job_message("server", C.FORWARD_JOB, 5, big))
        c.send(M.text_message("server", C.CONFIG_TRANSFER, "{}"))
        m = s.recv(5000)
        assert m.command == C.FORWARD_JOB and m.sender == "cli" and m.mb_id == 5
        assert torch.equal(M.message_tensor(m), big)
        m2 = s.recv(5000)
        assert m2.text == b"{}"
        # reply over the accepted connection
        s.send(M.flag_message("cli", C.HEALTH_CHECK, True))
        r = c.recv(5000)
        assert r.flag and r.sender == "server"
        assert c.bytes_sent > big.numel() * 4
    finally:
        c.close()
        s.close()


def test_compression_roundtrip():
    data = (b"abcd" * 5000) + bytes(range(256))
    for codec in (1, 2):
        if codec == 2 and not comm.zstd_available():
            continue
        z = comm.compress(data, codec, 3)
        assert len(z) < len(data)
        assert comm.decompress(z, codec, len(data)) == data
