"""Pipeline stage event loop (reference include/pipeline/pipeline_stage.hpp:29-308).

A stage owns one partition of the model, its optimizer and a communicator.  It pops one
message at a time from the native priority queue (FORWARD_JOB before BACKWARD_JOB before
control traffic) and dispatches on the command.  Differences from the reference, on
purpose:

* every command listed in the enum has a handler (SEND/LOAD_PARAMS, STATUS, HEALTH_CHECK,
  BARRIER_SYNC, CHECKPOINT_REQUEST, REPORT_LOAD with a serialised LoadTracker);
* handler failures are reported to the coordinator (ERROR_REPORT / JOB_FAILURE with the
  traceback) instead of killing the stage;
* stage 0 does not ship the unused input gradient back unless asked to;
* activations stay in the stage's compute dtype (bf16 on MI355X) end to end;
* a GPU stage runs on its own HIP stream (stages sharing a GPU overlap instead of serialising
  on the null stream) with its device current on the stage thread, and from its second training
  step on replays per-micro-batch hipGraphs (``graphs.StageGraphs``) instead of launching every
  layer op from Python.
"""
from __future__ import annotations

import json
import os
import threading
import time
import traceback
from typing import Optional

import torch

from ...nn.optimizers import OptimizerFactory
from ...nn.sequential import Sequential, _all_layers
from ...nn.layers import BatchNorm
from . import messages as M
from .config import StageConfig
from .faults import FaultInjector, FaultSpec, Heartbeat, InjectedFault, env_faults
from .graphs import StageGraphs
from .transport import LocalTransport, MessageTransport, P2PTransport

C = M.CommandType


def flat_state(model: Sequential) -> torch.Tensor:
    """Parameters (in ``parameters()`` order) then BN running mean/var, as one fp32 vector."""
    parts = [p.detach().reshape(-1).float().cpu() for p in model.parameters()]
    for l in _all_layers(model.layers):
        if isinstance(l, BatchNorm):
            parts += [l.running_mean.detach().reshape(-1).float().cpu(), l.running_var.detach().reshape(-1).float().cpu()]
    return torch.cat(parts) if parts else torch.zeros(0)


def load_flat_state(model: Sequential, flat: torch.Tensor) -> None:
    flat = flat.reshape(-1).float().cpu()
    off = 0
    with torch.no_grad():
        for p in model.parameters():
            n = p.numel()
            p.copy_(flat[off:off + n].view(p.shape))
            off += n
        for l in _all_layers(model.layers):
            if isinstance(l, BatchNorm):
                n = l.running_mean.numel()
                l.running_mean.copy_(flat[off:off + n])
                l.running_var.copy_(flat[off + n:off + 2 * n])
                off += 2 * n
    if off != flat.numel():
        raise RuntimeError(f"flat state size mismatch: consumed {off} of {flat.numel()}")
    if model.arena is not None:
        model.arena.sync_shadow(force=True)


def flat_optimizer_state(opt) -> torch.Tensor:
    """Optimizer state as one fp64 vector: [learning rate, step counter t, then every state
    tensor of ``state_dict()`` in key order] (Adam: m, v; SGD with momentum: velocity)."""
    d = opt.state_dict() if opt is not None else {}
    parts = [torch.tensor([float(opt.get_learning_rate()) if opt is not None else 0.0, float(d.get("t", 0))],
                          dtype=torch.float64)]
    for k in sorted(d):
        if isinstance(d[k], list):
            parts += [x.detach().reshape(-1).double().cpu() for x in d[k]]
    return torch.cat(parts)


def load_flat_optimizer_state(opt, flat: torch.Tensor) -> None:
    """Inverse of :func:`flat_optimizer_state` (the optimizer must already be attached)."""
    flat = flat.reshape(-1).double().cpu()
    d = opt.state_dict()
    off = 2
    out = {"t": int(flat[1].item())}
    for k in sorted(d):
        if isinstance(d[k], list):
            lst = []
            for x in d[k]:
                n = x.numel()
                lst.append(flat[off:off + n].view(x.shape).to(x.dtype))
                off += n
            out[k] = lst
    if off != flat.numel():
        raise RuntimeError(f"optimizer state size mismatch: consumed {off} of {flat.numel()}")
    opt.load_state_dict(out)
    opt.set_learning_rate(float(flat[0].item()))


# SEND_PARAMS / LOAD_PARAMS with micro-batch id FULL_STATE carry the optimizer state too: the
# parameter vector (fp32, flat_state) is followed by flat_optimizer_state widened into the same
# fp64 message, headed by the parameter count
FULL_STATE = 1


def pack_full_state(model, opt) -> torch.Tensor:
    fp = flat_state(model).double()
    return torch.cat([torch.tensor([float(fp.numel())], dtype=torch.float64), fp, flat_optimizer_state(opt)])


def unpack_full_state(model, opt, flat: torch.Tensor) -> None:
    flat = flat.reshape(-1).double()
    n = int(flat[0].item())
    load_flat_state(model, flat[1:1 + n].float())
    load_flat_optimizer_state(opt, flat[1 + n:])


class PipelineStage:
    def __init__(self, communicator, p2p_groups=None, verbose: bool = False):
        self.comm = communicator
        self.id = communicator.id
        self.groups = p2p_groups
        self.verbose = verbose
        self.cfg: Optional[StageConfig] = None
        self.model: Optional[Sequential] = None
        self.optimizer = None
        self.transport = MessageTransport()
        self.running = False
        self.thread: Optional[threading.Thread] = None
        self.counts = {"forward": 0, "backward": 0, "update": 0}
        self.fwd_ms = []
        self.bwd_ms = []
        self.last_error: Optional[str] = None
        self.stream: Optional[torch.cuda.Stream] = None
        self.graphs: Optional[StageGraphs] = None
        self.steps_done = 0
        self.faults = FaultInjector([])
        self.heartbeat: Optional[Heartbeat] = None
        self.crashed = False

    # ------------------------------------------------------------------ loop
    def run(self, poll_ms: int = 200) -> None:
        self.running = True
        while self.running:
            msg = self.comm.recv(poll_ms)
            if msg is None:
                continue
            self.process_message(msg)

    def start_thread(self) -> threading.Thread:
        self.thread = threading.Thread(target=self.run, name=f"pipeline-{self.id}", daemon=True)
        self.thread.start()
        return self.thread

    def stop(self) -> None:
        self.running = False
        if self.heartbeat is not None:
            self.heartbeat.stop()

    def _crash(self) -> None:
        """Injected crash: the stage goes silent (no reply, no heartbeat, loop exits)."""
        self.crashed = True
        self.stop()

    def _device(self):
        return self.model.device.torch_device

    def _reply(self, command, text: Optional[str] = None, flag: Optional[bool] = None):
        m = M.Message("coordinator", command)
        if text is not None:
            m.text = text.encode()
        elif flag is not None:
            m.flag = flag
        self._send(m)

    def _send(self, m):
        if hasattr(self.comm, "wait_for_peer"):
            self.comm.wait_for_peer(m.recipient, 30000)
        self.comm.send(m)

    def _wait_peer(self, name):
        if hasattr(self.comm, "wait_for_peer") and not self.comm.wait_for_peer(name, 30000):
            raise RuntimeError(f"{self.id}: peer '{name}' never connected")

    # ------------------------------------------------------------------ dispatch
    def process_message(self, msg) -> None:
        if self.stream is not None:
            with torch.cuda.device(self.stream.device), torch.cuda.stream(self.stream):
                self._process(msg)
        else:
            self._process(msg)

    def _process(self, msg) -> None:
        cmd = msg.command
        try:
            if self.faults:
                act = self.faults.check(cmd)
                if act == "drop":
                    return
                if act == "crash":
                    self._crash()
                    return
                if act == "raise":
                    raise InjectedFault(f"{self.id}: injected fault on {M.command_name(cmd)}")
            if cmd == C.FORWARD_JOB:
                self._forward(msg)
            elif cmd == C.BACKWARD_JOB:
                self._backward(msg)
            elif cmd == C.UPDATE_PARAMETERS:
                if msg.payload_type == M.P_STRING:  # hyper-parameter change from the coordinator
                    hp = json.loads(msg.text.decode())
                    if "learning_rate" in hp:
                        self.optimizer.set_learning_rate(hp["learning_rate"])
                self.optimizer.update()
                self.optimizer.clear_gradients()
                self.counts["update"] += 1
                self.steps_done += 1
                self._reply(C.PARAMETERS_UPDATED)
            elif cmd == C.TRAIN_MODE:
                self.model.set_training(True)
            elif cmd == C.EVAL_MODE:
                self.model.set_training(False)
            elif cmd == C.SHUTDOWN:
                self.transport.flush()
                self.stop()
            elif cmd == C.CONFIG_TRANSFER:
                self._configure(msg.text.decode())
            elif cmd == C.SEND_PARAMS:
                self._wait_peer("coordinator")
                if msg.payload_type == M.P_STRING and msg.text.decode() == "full":
                    self.comm.send(M.job_message("coordinator", C.PARAMS_TRANSFER, FULL_STATE,
                                                 pack_full_state(self.model, self.optimizer)))
                else:
                    self.comm.send(M.job_message("coordinator", C.PARAMS_TRANSFER, 0, flat_state(self.model)))
            elif cmd in (C.LOAD_PARAMS, C.PARAMS_TRANSFER):
                if msg.payload_type in (M.P_JOB, M.P_TYPED_JOB) and int(msg.mb_id) == FULL_STATE:
                    unpack_full_state(self.model, self.optimizer, M.message_tensor(msg))
                else:
                    load_flat_state(self.model, M.message_tensor(msg))
                self._reply(C.PARAMS_LOADED)
            elif cmd == C.STATUS_REQUEST:
                self._reply(C.STATUS_RESPONSE, json.dumps(self.status()))
            elif cmd == C.HEALTH_CHECK:
                self._reply(C.HEALTH_CHECK, flag=True)
            elif cmd == C.BARRIER_SYNC:
                if self.model is not None and self.model.device.is_gpu():
                    torch.cuda.synchronize(self._device())
                self.transport.flush()
                self._reply(C.BARRIER_SYNC)
            elif cmd == C.CHECKPOINT_REQUEST:
                path = msg.text.decode()
                self.model.save_to_file(path)
                self._reply(C.CHECKPOINT_COMPLETE, path)
            elif cmd == C.REPORT_LOAD:
                self._report_load()
            elif cmd == C.UPDATE_LOAD:
                self._reply(C.LOAD_REPORT, json.dumps(self.status()))
            elif cmd == C.PRINT_PROFILING:
                txt = self.model.print_profiling_summary() if self.model is not None else ""
                self._reply(C.PROFILING_PRINTED, txt or "")
            elif cmd == C.CLEAR_PROFILING:
                self.model.clear_profiling_data()
                self.fwd_ms.clear()
                self.bwd_ms.clear()
                self._reply(C.PROFILING_CLEARED)
            else:
                raise RuntimeError(f"unhandled command {M.command_name(cmd)}")
        except Exception:
            self.last_error = traceback.format_exc()
            kind = C.JOB_FAILURE if cmd in (C.FORWARD_JOB, C.BACKWARD_JOB) else C.ERROR_REPORT
            try:
                self._reply(kind, f"{self.id}: {M.command_name(cmd)} failed\n{self.last_error}")
            except Exception:
                pass
            if self.verbose:
                print(self.last_error, flush=True)

    # ------------------------------------------------------------------ handlers
    def _configure(self, text: str) -> None:
        cfg = StageConfig.from_json(text)
        self.cfg = cfg
        model = Sequential.load_from_config(cfg.model_config)
        if cfg.seed is not None:
            model.set_seed(int(cfg.seed))
        dev = cfg.device
        if dev.upper().startswith("GPU") and not torch.cuda.is_available():
            raise RuntimeError(f"{self.id}: GPU requested but no GPU is visible")
        self.stream = None
        self.graphs = None
        self.steps_done = 0
        if dev.upper().startswith("GPU"):
            idx = int(dev.split(":")[1]) if ":" in dev else 0
            self.stream = torch.cuda.Stream(device=idx)
            torch.cuda.set_device(idx)
        model.set_device(dev)
        if cfg.compute_dtype not in ("auto", "", None):
            model.set_compute_dtype(getattr(torch, cfg.compute_dtype))
        model.initialize()
        model.set_first_layer_input_grad(cfg.first_layer_input_grad if cfg.stage_index == 0 else True)
        model.enable_profiling(cfg.profiling)
        self.model = model
        self.optimizer = OptimizerFactory.create_from_config(cfg.optimizer_config)
        self.optimizer.attach(model)
        if self.stream is not None:
            # initialisation ran on this thread's default stream; order the stage stream after it
            self.stream.wait_stream(torch.cuda.current_stream(self.stream.device))
            if cfg.use_graph:
                self.graphs = StageGraphs(model, self.stream)
        if hasattr(self.comm, "set_id"):  # network worker: adopt the stage name before dialing peers
            self.comm.set_id(cfg.stage_id)
            self.id = cfg.stage_id
        self._connect_peers(cfg)
        self._make_transport(cfg)
        self.faults = FaultInjector([FaultSpec.parse(f) for f in (cfg.fault or [])] + env_faults(cfg.stage_id))
        if self.heartbeat is not None:
            self.heartbeat.stop()
            self.heartbeat = None
        if cfg.heartbeat_s and cfg.heartbeat_s > 0:
            self.heartbeat = Heartbeat(self._send, cfg.heartbeat_s).start()
        self._reply(C.CONFIG_RECEIVED, self.id)

    def _connect_peers(self, cfg: StageConfig) -> None:
        comm = self.comm
        is_tcp = hasattr(comm, "connect")
        for name, ep in (("next_stage", cfg.next_stage_endpoint), ("prev_stage", cfg.prev_stage_endpoint),
                         ("coordinator", cfg.coordinator_endpoint)):
            if ep is None:
                continue
            if ep.communication_type == "in_process":
                if ep.get("id") != name:
                    comm.alias(name, ep.get("id"))
            elif is_tcp:
                peer_id = ep.get("id")
                if name == "next_stage":
                    comm.connect(name, ep.get("host"), int(ep.get("port")), 60000)
                    if peer_id:
                        comm.alias(peer_id, name)
                elif peer_id:
                    # prev stage / coordinator connect to us; route the logical name to their id
                    comm.alias(name, peer_id)
            else:
                raise RuntimeError(f"endpoint type {ep.communication_type} needs a TCP communicator")

    def _resolve(self, name: str) -> str:
        c = self.cfg
        table = {"next_stage": c.next_stage_endpoint, "prev_stage": c.prev_stage_endpoint,
                 "coordinator": c.coordinator_endpoint}
        ep = table.get(name)
        return ep.get("id", name) if ep is not None else name

    def _make_transport(self, cfg: StageConfig) -> None:
        if cfg.transport == "p2p":
            ranks = {}
            for k, v in (cfg.ranks or {}).items():
                ranks[k] = int(v)
                ranks[self._resolve(k)] = int(v)
            self.transport = P2PTransport(self.id, ranks, self.groups, self._resolve)
        elif cfg.transport == "local":
            self.transport = LocalTransport(self.id, self._resolve)
        else:
            self.transport = MessageTransport(cfg.codec)

    def _forward(self, msg) -> None:
        mb = int(msg.mb_id)
        t0 = time.perf_counter()
        x = self.transport.recv(msg, self._device())
        if self._graph_ok():
            out = self.graphs.forward(x, mb)
        else:
            if self.graphs is not None:
                self.graphs.forget_forward(mb)
            out = self.model.forward(x, mb, return_on_input_device=False)
        last = self.cfg.stage_index == self.cfg.num_stages - 1
        self.transport.send(self.comm, "coordinator" if last else "next_stage", C.FORWARD_JOB, mb, out)
        self.counts["forward"] += 1
        self.fwd_ms.append((time.perf_counter() - t0) * 1e3)

    def _backward(self, msg) -> None:
        mb = int(msg.mb_id)
        t0 = time.perf_counter()
        g = self.transport.recv(msg, self._device())
        if self.graphs is not None and self.graphs.can_backward(mb):
            gin = self.graphs.backward(g, mb)
        else:
            gin = self.model.backward(g, mb, return_on_input_device=False)
        first = self.cfg.stage_index == 0
        if first and not self.cfg.first_layer_input_grad:
            gin = None
        self.transport.send(self.comm, "coordinator" if first else "prev_stage", C.BACKWARD_JOB, mb, gin)
        self.counts["backward"] += 1
        self.bwd_ms.append((time.perf_counter() - t0) * 1e3)

    def _graph_ok(self) -> bool:
        """Replay graphs once one eager training step has run (allocations settled, per-layer
        profile recorded) and only for training forwards."""
        return self.graphs is not None and self.steps_done >= 1 and self.model.training

    def status(self) -> dict:
        m = self.model
        d = {"id": self.id, "counts": dict(self.counts), "pid": os.getpid()}
        if self.graphs is not None:
            d["graphs"] = {"captures": self.graphs.captures, "replays": self.graphs.replays}
        if m is not None:
            d.update(device=str(m.device.torch_device), layers=[l.name for l in m.layers],
                     num_parameters=m.num_parameters(),
                     forward_times_us=dict(m.forward_times_us), backward_times_us=dict(m.backward_times_us))
        return d

    def _report_load(self) -> None:
        from ...utils.hardware import process_rss_kb
        from ...ops._ext import native
        f = sum(self.fwd_ms) / len(self.fwd_ms) if self.fwd_ms else 0.0
        b = sum(self.bwd_ms) / len(self.bwd_ms) if self.bwd_ms else 0.0
        try:
            cpu = float(native().cpu_utilization_total(20)) / 100.0
        except Exception:
            cpu = -1.0
        m = M.Message("coordinator", C.LOAD_REPORT)
        m.load = (f, b, cpu, process_rss_kb() / 1024.0)
        self._send(m)
