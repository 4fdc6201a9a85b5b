"""Endpoints and per-stage configuration (reference include/pipeline/endpoint.hpp:17-94 and
include/pipeline/stage_config.hpp:8-35), JSON round-trippable."""
from __future__ import annotations

import json
from dataclasses import dataclass, field
from typing import Any, Dict, Optional


@dataclass
class Endpoint:
    communication_type: str = "tcp"          # "tcp" | "in_process"
    parameters: Dict[str, Any] = field(default_factory=dict)

    @staticmethod
    def network(host: str, port: int) -> "Endpoint":
        return Endpoint("tcp", {"host": host, "port": int(port)})

    @staticmethod
    def in_process(comm_id: str) -> "Endpoint":
        return Endpoint("in_process", {"id": comm_id})

    def get(self, key, default=None):
        return self.parameters.get(key, default)

    def to_json(self) -> dict:
        return {"communication_type": self.communication_type, "parameters": dict(self.parameters)}

    @staticmethod
    def from_json(j: Optional[dict]) -> Optional["Endpoint"]:
        if not j:
            return None
        return Endpoint(j.get("communication_type", "tcp"), dict(j.get("parameters", {})))


@dataclass
class StageConfig:
    stage_id: str
    stage_index: int
    num_stages: int
    model_config: dict
    optimizer_config: dict
    next_stage_endpoint: Optional[Endpoint] = None
    prev_stage_endpoint: Optional[Endpoint] = None
    coordinator_endpoint: Optional[Endpoint] = None
    device: str = "CPU"                      # "CPU" | "GPU" | "GPU:i"
    transport: str = "message"               # "message" (inline tensors) | "p2p" (RCCL/gloo send/recv)
    codec: str = "none"                      # inline payload compression
    compute_dtype: str = "auto"              # "auto" (bf16 on GPU) | "float32" | "bfloat16"
    seed: Optional[int] = None
    first_layer_input_grad: bool = False     # stage 0 does not return dL/dinput (reference G9)
    ranks: Optional[Dict[str, int]] = None   # torch.distributed ranks: {"prev": r, "next": r, "coordinator": r}
    profiling: bool = True
    use_graph: bool = False                  # GPU: replay per-micro-batch hipGraphs after the first step
    heartbeat_s: float = 0.0                 # > 0: unsolicited HEALTH_CHECK beats to the coordinator (faults.py)
    fault: Optional[list] = None             # fault-injection specs (faults.FaultSpec.parse), tests / drills

    def to_json(self) -> dict:
        d = dict(self.__dict__)
        for k in ("next_stage_endpoint", "prev_stage_endpoint", "coordinator_endpoint"):
            d[k] = d[k].to_json() if d[k] is not None else None
        return d

    def dumps(self) -> str:
        return json.dumps(self.to_json())

    @staticmethod
    def from_json(j) -> "StageConfig":
        if isinstance(j, (str, bytes)):
            j = json.loads(j)
        j = dict(j)
        for k in ("next_stage_endpoint", "prev_stage_endpoint", "coordinator_endpoint"):
            j[k] = Endpoint.from_json(j.get(k))
        return StageConfig(**j)
