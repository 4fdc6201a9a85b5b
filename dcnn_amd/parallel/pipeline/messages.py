"""Python view of the native control-plane message model (``_native.comm``).

``CommandType`` mirrors the reference enum (include/pipeline/command_type.hpp:20-68) — the
numeric order is both the wire value and the dequeue priority (FORWARD_JOB first).  Tensors
travel either *inline* in a message (TCP / in-process transport, reference-compatible
``Job<float>`` or the typed extension carrying bf16 and compressed payloads) or as metadata
only, with the bytes moved GPU-to-GPU by RCCL (see ``transport.py``).
"""
from __future__ import annotations

import enum
from typing import Optional, Sequence, Tuple

import numpy as np
import torch

from ...ops._ext import native


def comm():
    return native().comm


CommandType = enum.IntEnum("CommandType", {k: v for k, v in sorted(native().comm.COMMANDS.items(),
                                                                         key=lambda kv: kv[1])})

# payload types (comm.h)
P_NONE, P_JOB, P_STRING, P_BOOL, P_LOAD, P_TYPED_JOB = range(6)
CODECS = {"none": 0, "zlib": 1, "zstd": 2}

_DT = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2, torch.int64: 3, torch.uint8: 4, torch.float64: 5}
_DT_INV = {v: k for k, v in _DT.items()}
_NP = {0: np.float32, 1: np.uint16, 2: np.float16, 3: np.int64, 4: np.uint8, 5: np.float64}
CL_FLAG = 0x10  # dtype bit: payload is the NHWC physical buffer of a channels_last NCHW tensor


def Message(recipient: str, command: int):
    return comm().Message(recipient, int(command))


def text_message(recipient: str, command: int, text: str):
    m = Message(recipient, command)
    m.text = text.encode()
    return m


def flag_message(recipient: str, command: int, flag: bool):
    m = Message(recipient, command)
    m.flag = bool(flag)
    return m


def _physical(t: torch.Tensor) -> Tuple[torch.Tensor, int]:
    """(contiguous physical buffer, layout flag) without an NHWC->NCHW round trip."""
    if t.dim() == 4 and not t.is_contiguous() and t.is_contiguous(memory_format=torch.channels_last):
        return t.permute(0, 2, 3, 1), CL_FLAG
    return t.contiguous(), 0


def tensor_meta(t: torch.Tensor) -> Tuple[list, int]:
    phys, flag = _physical(t)
    return list(phys.shape), _DT[t.dtype] | flag


def job_message(recipient: str, command: int, mb_id: int, t: Optional[torch.Tensor], codec: str = "none",
                legacy: bool = False):
    """Message carrying tensor ``t`` inline (copied to host)."""
    m = Message(recipient, command)
    if t is None:
        m.set_job_meta(int(mb_id), [], 0)
        return m
    phys, flag = _physical(t.detach())
    host = phys.to("cpu")
    if legacy:  # reference Job<float>: fp32, logical NCHW
        m.set_tensor(int(mb_id), t.detach().to("cpu", torch.float32).contiguous().numpy(), 0, 0, 3, True)
        return m
    arr = host.view(torch.uint16).numpy() if host.dtype == torch.bfloat16 else host.numpy()
    m.set_tensor(int(mb_id), arr, _DT[t.dtype] | flag, CODECS[codec], 3, False)
    return m


def meta_message(recipient: str, command: int, mb_id: int, t: Optional[torch.Tensor]):
    """Message with only shape/dtype of ``t`` (bytes travel on the RCCL data plane)."""
    m = Message(recipient, command)
    if t is None:
        m.set_job_meta(int(mb_id), [], 0)
    else:
        shape, code = tensor_meta(t)
        m.set_job_meta(int(mb_id), shape, code)
    return m


def has_tensor(m) -> bool:
    return m.payload_type in (P_JOB, P_TYPED_JOB) and len(m.shape) > 0


def alloc_for(m, device) -> Tuple[torch.Tensor, torch.Tensor]:
    """(physical receive buffer, logical view) for a metadata-only job message."""
    code = m.dtype
    dt = _DT_INV[code & 0x0F]
    phys = torch.empty(list(m.shape), dtype=dt, device=device)
    return phys, (phys.permute(0, 3, 1, 2) if code & CL_FLAG else phys)


def message_tensor(m, device=None) -> Optional[torch.Tensor]:
    """Decode an inline tensor payload (zero-copy view of the message buffer, then to device)."""
    if not has_tensor(m):
        return None
    if m.codec:
        m.decompress()
    code = m.dtype if m.payload_type == P_TYPED_JOB else 0
    arr = np.frombuffer(m, dtype=_NP[code & 0x0F]).reshape(list(m.shape))
    t = torch.from_numpy(arr)
    if (code & 0x0F) == 1:
        t = t.view(torch.bfloat16)
    if code & CL_FLAG:
        t = t.permute(0, 3, 1, 2)
    if device is not None:
        t = t.to(device)
    else:
        t = t.clone()  # detach from the message buffer
    return t


def command_name(c: int) -> str:
    return comm().command_name(int(c))


def names(cmds: Sequence[int]):
    return [command_name(c) for c in cmds]
