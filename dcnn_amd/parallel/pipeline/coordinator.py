"""Pipeline coordinator (reference include/pipeline/coordinator.hpp:30-599,
distributed_coordinator.hpp, in_process_coordinator.hpp).

The coordinator owns the full model description, the optimizer config, the loss and the
partitioner.  ``initialize()`` partitions the model and builds one ``StageConfig`` per stage;
``deploy_stages()`` ships them (CONFIG_TRANSFER) and waits for CONFIG_RECEIVED.  Training
steps then exchange micro-batches with the first / last stage:

* ``sync_process_batch`` — GPipe: all forwards, all losses, all backwards.
* ``async_process_batch`` — the reference's semi-async schedule (coordinator.hpp:273-326):
  every forward is issued at once, and each output's loss + backward is launched the moment
  it arrives while stages keep prioritising forwards.
* ``one_f_one_b_process_batch`` — 1F1B (PipeDream-flush): at most ``max_in_flight`` micro-batches
  (default: the number of stages) are between their forward and the end of their backward; a new
  forward is injected each time a backward completes. Every stage then holds the activations of
  at most that many micro-batches (GPipe / semi-async hold all of them) while the steady state
  alternates one forward with one backward per stage.
* ``update_parameters()`` — UPDATE_PARAMETERS broadcast + join PARAMETERS_UPDATED.

Gradient semantics: each micro-batch's loss gradient is the micro-batch mean; by default it
is scaled by 1/num_microbatches so the accumulated gradient equals the full-batch mean
(``grad_scale="mean"``, what the reference's own microbatching_test intended).
``grad_scale="sum"`` reproduces the reference's summed behaviour.

Fixed reference defects: stage names are not duplicated (G1), the topology is always
initialised before deployment (G2), in-process delivery cannot deadlock (G3).
"""
from __future__ import annotations

import json
import threading
import time
from typing import Dict, List, Optional, Sequence

import torch

from ...nn.loss import Loss, LossFactory
from ...nn.sequential import Partition, Sequential
from . import messages as M
from .config import Endpoint, StageConfig
from .faults import HEARTBEAT_TEXT
from .partitioner import CostPartitioner, NaivePartitioner, Partitioner
from .stage import FULL_STATE, PipelineStage, flat_state, load_flat_state
from .transport import MAILBOX, LocalTransport, MessageTransport, P2PTransport

C = M.CommandType


class PipelineError(RuntimeError):
    pass


class StageFailure(PipelineError):
    """A stage stopped responding: missed heartbeats or a lost control-plane connection."""

    def __init__(self, stage: str, why: str):
        super().__init__(f"{stage}: {why}")
        self.stage = stage


class Coordinator:
    def __init__(self, model: Sequential, optimizer, loss, num_stages: int, num_microbatches: int = 1,
                 partitioner: Optional[Partitioner] = None, input_shape: Optional[Sequence[int]] = None,
                 device: str = "CPU", stage_devices: Optional[Sequence[str]] = None, transport: str = "message",
                 codec: str = "none", grad_scale: str = "mean", seed: Optional[int] = None,
                 timeout_s: float = 120.0, use_graph: Optional[bool] = None, profiling: bool = True,
                 heartbeat_s: float = 0.0, heartbeat_misses: int = 3):
        self.model = model
        self.optimizer_config = optimizer.get_config() if hasattr(optimizer, "get_config") else dict(optimizer)
        self.loss: Loss = LossFactory.create(loss) if isinstance(loss, str) else loss
        self.num_stages = int(num_stages)
        self.num_microbatches = int(num_microbatches)
        self.partitioner = partitioner or NaivePartitioner()
        self.input_shape = list(input_shape) if input_shape else None
        self.device = torch.device("cuda", _gpu_index(device)) if device.upper().startswith("GPU") else torch.device("cpu")
        self.stage_devices = list(stage_devices) if stage_devices else ["CPU"] * self.num_stages
        self.transport_kind = transport
        self.codec = codec
        self.grad_scale = grad_scale
        self.seed = seed
        self.timeout_s = timeout_s
        self.use_graph = use_graph        # None: hipGraph replay on every GPU stage
        self.profiling = bool(profiling)  # per-layer timings (eager steps) for balance_load
        self.stage_names = [f"stage_{i}" for i in range(self.num_stages)]
        self.partitions: List[Partition] = []
        self.stage_configs: List[StageConfig] = []
        self.comm = None
        self.transport = None
        self.deployed = False
        self.last_correct = 0
        # failure detection (faults.py): stage heartbeats every heartbeat_s; a stage silent for
        # heartbeat_s * heartbeat_misses is declared failed
        self.heartbeat_s = float(heartbeat_s)
        self.heartbeat_misses = int(heartbeat_misses)
        self._last_beat: Dict[str, float] = {}
        self._stash: Dict[int, list] = {}
        # recovery: parameter snapshots every snapshot_every steps, re-deploy + reload on failure
        self.snapshot_every = 0
        self._replay_log, self._replay_pending = [], False
        self.max_recoveries = 0
        self.recoveries = 0
        self.steps = 0
        self._snapshot: Optional[List[torch.Tensor]] = None
        self._snapshot_step = -1

    # ------------------------------------------------------------------ topology
    def set_partitioner(self, p: Partitioner) -> None:
        self.partitioner = p

    def set_loss_function(self, loss) -> None:
        self.loss = LossFactory.create(loss) if isinstance(loss, str) else loss

    def set_num_microbatches(self, n: int) -> bool:
        if n <= 0:
            return False
        self.num_microbatches = int(n)
        return True

    def initialize(self) -> None:
        self.partitions = self.partitioner.get_partitions(self.model, self.num_stages, self.input_shape)
        self.stage_configs = []
        for i, part in enumerate(self.partitions):
            self.stage_configs.append(StageConfig(
                stage_id=self.stage_names[i], stage_index=i, num_stages=self.num_stages,
                model_config=self.model.get_config(part), optimizer_config=dict(self.optimizer_config),
                device=self.stage_devices[i], transport=self.transport_kind, codec=self.codec,
                seed=None if self.seed is None else self.seed + i, profiling=self.profiling,
                use_graph=(self.stage_devices[i].upper().startswith("GPU") if self.use_graph is None
                           else bool(self.use_graph)),
                heartbeat_s=self.heartbeat_s))
        self._init_topology()

    def _init_topology(self) -> None:
        raise NotImplementedError

    def _endpoint(self, i: int) -> Endpoint:
        raise NotImplementedError

    def _coordinator_endpoint(self) -> Endpoint:
        raise NotImplementedError

    def _wire_configs(self) -> None:
        for i, c in enumerate(self.stage_configs):
            c.coordinator_endpoint = self._coordinator_endpoint()
            c.next_stage_endpoint = self._endpoint(i + 1) if i + 1 < self.num_stages else None
            c.prev_stage_endpoint = self._endpoint(i - 1) if i > 0 else None

    def deploy_stages(self) -> None:
        if not self.stage_configs:
            self.initialize()
        # deploy back to front so each stage's "next_stage" listener is configured first
        for i in range(self.num_stages - 1, -1, -1):
            self.comm.send(M.text_message(self.stage_names[i], C.CONFIG_TRANSFER, self.stage_configs[i].dumps()))
            self.join(C.CONFIG_RECEIVED, 1, self.timeout_s)
        self.deployed = True
        now = time.time()
        self._last_beat = {s: now for s in self.stage_names}

    def start(self) -> None:
        self.broadcast(C.TRAIN_MODE)

    def stop(self) -> None:
        if self.comm is None:
            return
        try:
            self.broadcast(C.SHUTDOWN)
        except Exception:
            pass

    def broadcast(self, command, text: Optional[str] = None) -> None:
        for s in self.stage_names:
            m = M.Message(s, command)
            if text is not None:
                m.text = text.encode()
            self.comm.send(m)

    # ------------------------------------------------------------------ messaging
    def _check_errors(self) -> None:
        """Raise on a stage's ERROR_REPORT / JOB_FAILURE, on missed heartbeats and on a lost
        control-plane connection (called by every waiting loop)."""
        for kind in (C.ERROR_REPORT, C.JOB_FAILURE):
            if self.comm.count(kind):
                m = self.comm.recv_command(kind, 0)
                raise PipelineError(m.text.decode() if m is not None else "stage error")
        if not self.deployed:
            return
        if self.heartbeat_s > 0:
            while self.comm.count(int(C.HEALTH_CHECK)):
                m = self.comm.recv_command(int(C.HEALTH_CHECK), 0)
                if m is None:
                    break
                if not self._take_beat(m):
                    self._stash.setdefault(int(C.HEALTH_CHECK), []).append(m)
            now = time.time()
            limit = self.heartbeat_s * self.heartbeat_misses
            for s in self.stage_names:
                last = self._last_beat.get(s, now)
                if now - last > limit:
                    raise StageFailure(s, f"no heartbeat for {now - last:.1f} s (interval {self.heartbeat_s} s)")
        self._check_links()

    def _check_links(self) -> None:
        """Transport-level liveness (network coordinators: a dropped TCP connection)."""

    def _take_beat(self, m) -> bool:
        if m.command == C.HEALTH_CHECK and bytes(m.text) == HEARTBEAT_TEXT:
            self._last_beat[m.sender.split("/", 1)[-1]] = time.time()
            return True
        return False

    def join(self, command, n: int, timeout_s: Optional[float] = None) -> List:
        """Collect ``n`` messages of ``command`` (raises on stage errors / failures / timeout)."""
        deadline = time.time() + (timeout_s or self.timeout_s)
        out = []
        stash = self._stash.get(int(command))
        while stash and len(out) < n:
            out.append(stash.pop(0))
        while len(out) < n:
            self._check_errors()
            m = self.comm.recv_command(int(command), 50)
            if m is not None:
                if not self._take_beat(m):
                    out.append(m)
            elif time.time() > deadline:
                raise PipelineError(f"timeout waiting for {n} x {M.command_name(command)} (got {len(out)})")
        return out

    def forward(self, x: torch.Tensor, mb_id: int) -> None:
        self.transport.send(self.comm, self.stage_names[0], C.FORWARD_JOB, mb_id, x)

    def backward(self, grad: torch.Tensor, mb_id: int) -> None:
        self.transport.send(self.comm, self.stage_names[-1], C.BACKWARD_JOB, mb_id, grad)

    def _output(self, msg) -> torch.Tensor:
        return self.transport.recv(msg, self.device)

    def _loss_grad(self, out, y, mb):
        # the micro-batch mean (1 / num_microbatches) is applied inside the fused loss kernel
        scale = 1.0 / self.num_microbatches if self.grad_scale == "mean" and self.num_microbatches > 1 else 1.0
        loss, grad, correct = self.loss.loss_and_grad(out, y.to(out.device, non_blocking=True), grad_scale=scale)
        return loss, (grad if grad.dtype == out.dtype else grad.to(out.dtype)), correct

    def _finish(self, losses, corrects) -> float:
        """ONE host sync per step: the micro-batch losses / correct counts stay on the device
        until every backward has been issued."""
        m = max(len(losses), 1)
        if not losses:
            self.last_correct = 0
            return 0.0
        tot = torch.stack([l.reshape(()).float() for l in losses]).sum()
        cor = torch.stack([c.reshape(()).to(torch.int64) for c in corrects]).sum()
        both = torch.stack([tot.double(), cor.double()]).cpu()
        self.last_correct = int(both[1])
        return float(both[0]) / m

    # ------------------------------------------------------------------ schedules
    def split(self, x: torch.Tensor, y: torch.Tensor):
        """Split along the batch; the last micro-batch takes the remainder (reference split)."""
        m = self.num_microbatches
        n = x.shape[0]
        base = n // m
        xs, ys, s = [], [], 0
        for i in range(m):
            e = n if i == m - 1 else s + base
            xs.append(x[s:e])
            ys.append(y[s:e])
            s = e
        return xs, ys

    def sync_process_batch(self, xs: Sequence[torch.Tensor], ys: Sequence[torch.Tensor]) -> float:
        m = len(xs)
        for i in range(m):
            self.forward(xs[i], i)
        outs = {}
        for msg in self.join(C.FORWARD_JOB, m):
            outs[int(msg.mb_id)] = self._output(msg)
        losses, corrects = [], []
        for i in range(m):
            loss, grad, c = self._loss_grad(outs[i], ys[i], i)
            losses.append(loss)
            corrects.append(c)
            self.backward(grad, i)
        self.join(C.BACKWARD_JOB, m)
        return self._finish(losses, corrects)

    def async_process_batch(self, xs: Sequence[torch.Tensor], ys: Sequence[torch.Tensor]) -> float:
        m = len(xs)
        for i in range(m):
            self.forward(xs[i], i)
        losses, corrects, done = [], [], 0
        deadline = time.time() + self.timeout_s
        while done < m:
            self._check_errors()
            msg = self.comm.recv_command(int(C.FORWARD_JOB), 50)
            if msg is None:
                if time.time() > deadline:
                    raise PipelineError("timeout waiting for pipeline outputs")
                continue
            mb = int(msg.mb_id)
            out = self._output(msg)
            loss, grad, c = self._loss_grad(out, ys[mb], mb)
            self.backward(grad, mb)
            losses.append(loss)
            corrects.append(c)
            done += 1
        self.join(C.BACKWARD_JOB, m)
        return self._finish(losses, corrects)

    def one_f_one_b_process_batch(self, xs: Sequence[torch.Tensor], ys: Sequence[torch.Tensor],
                                  max_in_flight: Optional[int] = None) -> float:
        m = len(xs)
        cap = max(1, int(max_in_flight or self.num_stages))
        losses, corrects = [], []
        sent = done = 0
        while sent < min(m, cap):
            self.forward(xs[sent], sent)
            sent += 1
        self.max_in_flight_seen = sent
        deadline = time.time() + self.timeout_s
        kinds = [int(C.FORWARD_JOB), int(C.BACKWARD_JOB)]
        while done < m:
            self._check_errors()
            # wait for EITHER completion: polling one queue with a timeout while the other kind
            # arrives left the GPU idle for the rest of the timeout (profiles/pipeline_1f1b_r3.md)
            msg = self.comm.recv_any(kinds, 20)
            if msg is None:
                if time.time() > deadline:
                    raise PipelineError(f"1F1B: timeout ({done}/{m} backwards done)")
                continue
            if int(msg.command) == int(C.FORWARD_JOB):  # an output: loss, then its backward
                mb = int(msg.mb_id)
                loss, grad, c = self._loss_grad(self._output(msg), ys[mb], mb)
                self.backward(grad, mb)
                losses.append(loss)
                corrects.append(c)
            else:  # a backward finished: admit the next forward
                done += 1
                if sent < m:
                    self.forward(xs[sent], sent)
                    sent += 1
                    self.max_in_flight_seen = max(self.max_in_flight_seen, sent - done)
        return self._finish(losses, corrects)

    SCHEDULES = ("sync", "gpipe", "semi_async", "1f1b")

    def train_step(self, x: torch.Tensor, y: torch.Tensor, schedule: str = "semi_async") -> float:
        xs, ys = self.split(x, y)
        if schedule in ("sync", "gpipe"):
            fn = self.sync_process_batch
        elif schedule in ("semi_async", "async"):
            fn = self.async_process_batch
        elif schedule in ("1f1b", "one_f_one_b"):
            fn = self.one_f_one_b_process_batch
        else:
            raise ValueError(f"unknown pipeline schedule '{schedule}' (one of {self.SCHEDULES})")
        if self.max_recoveries <= 0:
            loss = fn(xs, ys)
            self.update_parameters()
            self.steps += 1
            return loss
        while True:
            try:
                if self._snapshot is None:
                    self.snapshot()
                if self._replay_pending:
                    # a recovery rolled the stages (parameters, BN statistics and optimizer state)
                    # back to the last snapshot: re-train the batches stepped since then (same
                    # order, same schedule, same learning rate) before this one
                    cur_lr = self.get_learning_rate()
                    for rfn, rxs, rys, rlr in self._replay_log:
                        if rlr != self.get_learning_rate():
                            self.set_learning_rate(rlr)
                        rfn(rxs, rys)
                        self.update_parameters()
                        self.steps += 1
                    if cur_lr != self.get_learning_rate():
                        self.set_learning_rate(cur_lr)
                    self._replay_pending = False
                lr = self.get_learning_rate()
                loss = fn(xs, ys)
                self.update_parameters()
                self.steps += 1
                if self.steps % self.snapshot_every == 0:
                    self.snapshot()
                else:
                    # clones: a loader that refills its batch buffers in place must not change
                    # what a replay trains on
                    self._replay_log.append((fn, [x.clone() for x in xs], [y.clone() for y in ys], lr))
                return loss
            except PipelineError:
                if self.recoveries >= self.max_recoveries:
                    raise
                self.recover()  # then replay the batches since the snapshot and retry this one

    # ------------------------------------------------------------------ recovery
    def enable_recovery(self, snapshot_every: int = 1, max_recoveries: int = 3) -> None:
        """Survive stage failures: snapshot every stage's parameters + BN statistics every
        ``snapshot_every`` steps; on a failed step (stage error, missed heartbeats, lost
        connection, timeout) re-deploy every stage, reload the last snapshot and retry the batch,
        at most ``max_recoveries`` times. The snapshot holds each stage's optimizer state too
        (Adam moments and step counter, SGD momentum, the learning rate in effect), so a replay
        neither double-counts nor drops an update."""
        self.snapshot_every = max(1, int(snapshot_every))
        self.max_recoveries = int(max_recoveries)

    def snapshot(self) -> None:
        self._snapshot = self.collect_parameters(full=True)
        self._snapshot_step = self.steps
        self._replay_log = []  # (schedule fn, micro-batches x, y) of every step after the snapshot
        self._replay_pending = False

    def recover(self) -> None:
        """Restart failed stages, re-deploy the topology and reload the last snapshot."""
        self.recoveries += 1
        self.deployed = False
        for c in self.stage_configs:  # a drill's injected faults fire once (DCNN_FAULT re-arms per deployment)
            c.fault = None
        self._restart_stages()
        self._drain()
        self.deploy_stages()
        if self._snapshot is not None:
            for i, flat in enumerate(self._snapshot):
                self.comm.send(M.job_message(self.stage_names[i], C.LOAD_PARAMS, FULL_STATE, flat))
            self.join(C.PARAMS_LOADED, self.num_stages)
            self.steps = self._snapshot_step
            self._lr_dirty = True  # the next update re-broadcasts the coordinator's learning rate
            self._replay_pending = bool(self._replay_log)
        self.start()

    def _restart_stages(self) -> None:
        """Bring every stage back to an accepting state (subclasses: re-create / re-dial)."""

    def _drain(self) -> None:
        """Drop every message left over from the failed attempt."""
        self._stash.clear()
        while self.comm.recv(0) is not None:
            pass

    def evaluate_batch(self, x: torch.Tensor, y: torch.Tensor):
        """Forward-only pass in eval mode: (mean loss, correct)."""
        xs, ys = self.split(x, y)
        for i, xi in enumerate(xs):
            self.forward(xi, i)
        losses, corrects = [], []
        for msg in self.join(C.FORWARD_JOB, len(xs)):
            out = self._output(msg)
            loss, _, c = self.loss.loss_and_grad(out, ys[int(msg.mb_id)].to(out.device), want_grad=False)
            losses.append(loss)
            corrects.append(c)
        mean = self._finish(losses, corrects)
        return mean, self.last_correct

    def update_parameters(self) -> None:
        """UPDATE_PARAMETERS broadcast; a pending learning-rate change rides along as JSON."""
        text = None
        if self._lr_dirty:
            text = json.dumps({"learning_rate": self.get_learning_rate()})
            self._lr_dirty = False
        self.broadcast(C.UPDATE_PARAMETERS, text)
        self.join(C.PARAMETERS_UPDATED, self.num_stages)

    # optimizer-like surface so LR schedulers can drive every stage through the coordinator
    _lr_dirty = False

    def get_learning_rate(self) -> float:
        return float(self.optimizer_config["parameters"].get("learning_rate", 0.0))

    def set_learning_rate(self, lr: float) -> None:
        self.optimizer_config["parameters"]["learning_rate"] = float(lr)
        self._lr_dirty = True

    # ------------------------------------------------------------------ parameters / checkpoints
    def collect_parameters(self, full: bool = False) -> List[torch.Tensor]:
        """SEND_PARAMS -> PARAMS_TRANSFER: flat fp32 state per stage (params + BN stats); with
        ``full`` the fp64 parameter + optimizer state (stage.pack_full_state)."""
        for s in self.stage_names:
            self.comm.send(M.text_message(s, C.SEND_PARAMS, "full") if full else M.Message(s, C.SEND_PARAMS))
        got = {m.sender: M.message_tensor(m) for m in self.join(C.PARAMS_TRANSFER, self.num_stages)}
        return [got[self._sender_key(i)] for i in range(self.num_stages)]

    def _sender_key(self, i: int) -> str:
        return self.stage_names[i]

    def send_parameters(self, model: Optional[Sequential] = None) -> None:
        """LOAD_PARAMS: push ``model``'s (default: the coordinator's) weights to every stage."""
        model = model or self.model
        if not model.initialized:
            model.initialize()
        for i, part in enumerate(self.partitions):
            sub = Sequential("tmp")
            sub.layers = model.layers[part.start_layer:part.end_layer]
            sub.arena = None
            flat = flat_state(sub)
            self.comm.send(M.job_message(self.stage_names[i], C.LOAD_PARAMS, 0, flat))
        self.join(C.PARAMS_LOADED, self.num_stages)

    def gather_model(self) -> Sequential:
        """Coordinator-side copy of the full trained model (for checkpoints / evaluation)."""
        flats = self.collect_parameters()
        if not self.model.initialized:
            self.model.initialize()
        for part, flat in zip(self.partitions, flats):
            sub = Sequential("tmp")
            sub.layers = self.model.layers[part.start_layer:part.end_layer]
            sub.arena = None
            load_flat_state(sub, flat)
        if self.model.arena is not None:
            self.model.arena.sync_shadow(force=True)
        return self.model

    def save_checkpoint(self, path: str) -> None:
        self.gather_model().save_to_file(path)

    # ------------------------------------------------------------------ monitoring
    def print_profiling_on_all_stages(self) -> List[str]:
        self.broadcast(C.PRINT_PROFILING)
        return [m.text.decode() for m in self.join(C.PROFILING_PRINTED, self.num_stages)]

    def clear_profiling_data(self) -> None:
        self.broadcast(C.CLEAR_PROFILING)
        self.join(C.PROFILING_CLEARED, self.num_stages)

    def status(self) -> List[dict]:
        self.broadcast(C.STATUS_REQUEST)
        return sorted((json.loads(m.text.decode()) for m in self.join(C.STATUS_RESPONSE, self.num_stages)),
                      key=lambda d: d["id"])

    def health_check(self, timeout_s: float = 10.0) -> Dict[str, bool]:
        self.broadcast(C.HEALTH_CHECK)
        alive = {s: False for s in self.stage_names}
        try:
            for m in self.join(C.HEALTH_CHECK, self.num_stages, timeout_s):
                alive[m.sender] = bool(m.flag)
        except PipelineError:
            pass
        return alive

    def barrier(self) -> None:
        self.broadcast(C.BARRIER_SYNC)
        self.join(C.BARRIER_SYNC, self.num_stages)

    def load_reports(self) -> Dict[str, tuple]:
        self.broadcast(C.REPORT_LOAD)
        return {m.sender: m.load for m in self.join(C.LOAD_REPORT, self.num_stages)}

    def balance_load(self) -> List[Partition]:
        """Re-partition from measured per-layer device times (STATUS_RESPONSE) and redeploy,
        carrying the trained weights over (the reference stubs this, coordinator.hpp:331)."""
        stats = self.status()
        costs = []
        for st, part in zip(stats, self.partitions):
            f, b = st.get("forward_times_us", {}), st.get("backward_times_us", {})
            for l in self.model.layers[part.start_layer:part.end_layer]:
                key = l.name or l.type()
                costs.append(f.get(key, 0.0) + b.get(key, 0.0))
        if not any(costs):
            return self.partitions
        new = CostPartitioner(costs).get_partitions(self.model, self.num_stages)
        if new == self.partitions:
            return new
        trained = self.gather_model()
        self.partitions = new
        for i, part in enumerate(new):
            self.stage_configs[i].model_config = self.model.get_config(part)
        self.deploy_stages()
        self.send_parameters(trained)
        return new


def _gpu_index(dev: str) -> int:
    parts = dev.split(":")
    return int(parts[1]) if len(parts) > 1 else 0


class InProcessCoordinator(Coordinator):
    """All stages in this process, each on its own thread and device (reference
    include/pipeline/in_process_coordinator.hpp).  Tensors are handed over by reference
    (``transport="local"``) — across GPUs that is a single xGMI peer copy."""

    _instances = 0

    def __init__(self, *a, **kw):
        kw.setdefault("transport", "local")
        super().__init__(*a, **kw)
        InProcessCoordinator._instances += 1
        self._tag = f"ip{InProcessCoordinator._instances}"
        self.stages: List[PipelineStage] = []

    def _cid(self, name):
        return f"{self._tag}/{name}"

    def _restart_stages(self) -> None:
        """Every stage gets a fresh thread and communicator (a crashed or hung stage's thread is
        abandoned: its communicator is closed, so it can no longer send)."""
        comm_mod = M.comm()
        new = []
        for s, st in zip(self.stage_names, self.stages):
            st.stop()
            st.comm.close()
            c = comm_mod.InProcessCommunicator(self._cid(s))
            ns = PipelineStage(c)
            ns.start_thread()
            new.append(ns)
        old, self.stages = self.stages, new
        for st in old:
            if st.thread is not None:
                st.thread.join(timeout=1.0)
        MAILBOX.purge(self._tag + "/")

    def _init_topology(self) -> None:
        comm_mod = M.comm()
        self.comm = comm_mod.InProcessCommunicator(self._cid("coordinator"))
        for s in self.stage_names:
            self.comm.alias(s, self._cid(s))
        self.stages = []
        for s in self.stage_names:
            c = comm_mod.InProcessCommunicator(self._cid(s))
            st = PipelineStage(c)
            st.start_thread()
            self.stages.append(st)
        self._wire_configs()
        if self.transport_kind == "local":
            self.transport = LocalTransport(self._cid("coordinator"), self._cid)
        else:
            self.transport = MessageTransport(self.codec)

    def _endpoint(self, i):
        return Endpoint.in_process(self._cid(self.stage_names[i]))

    def _coordinator_endpoint(self):
        return Endpoint.in_process(self._cid("coordinator"))

    def join(self, command, n, timeout_s=None):
        out = super().join(command, n, timeout_s)
        for m in out:  # report stage names without the instance tag
            m.sender = m.sender.split("/", 1)[-1]
        return out

    def stop(self) -> None:
        super().stop()
        for st in self.stages:
            if st.thread is not None:
                st.thread.join(timeout=30)
        for st in self.stages:
            st.comm.close()
        if self.comm is not None:
            self.comm.close()
            self.comm = None


class DistributedCoordinator(Coordinator):
    """Stages are separate processes (``NetworkStageWorker``) reached over the native TCP
    control plane (reference distributed_coordinator.hpp).  With ``transport="p2p"`` the
    coordinator and stages must share a ``torch.distributed`` world: tensors then move
    rank-to-rank with RCCL (gloo on CPU) and only metadata crosses TCP."""

    def __init__(self, model, optimizer, loss, stage_endpoints: Sequence[Endpoint], num_microbatches: int = 1,
                 host: str = "127.0.0.1", port: int = 0, stage_ranks: Optional[Sequence[int]] = None,
                 coordinator_rank: int = 0, p2p_groups=None, **kw):
        super().__init__(model, optimizer, loss, len(stage_endpoints), num_microbatches, **kw)
        self.stage_endpoints = list(stage_endpoints)
        self.host, self.port = host, port
        self.stage_ranks = list(stage_ranks) if stage_ranks is not None else None
        self.coordinator_rank = coordinator_rank
        self.p2p_groups = p2p_groups

    def _init_topology(self) -> None:
        comm_mod = M.comm()
        self.comm = comm_mod.TcpCommunicator("coordinator", "0.0.0.0", int(self.port))
        self.port = self.comm.port
        for i, ep in enumerate(self.stage_endpoints):
            self.comm.connect(self.stage_names[i], ep.get("host"), int(ep.get("port")), 60000)
        self._wire_configs()
        if self.transport_kind == "p2p":
            if self.stage_ranks is None:
                raise ValueError("transport='p2p' needs stage_ranks")
            for i, c in enumerate(self.stage_configs):
                r = {"coordinator": self.coordinator_rank}
                if i > 0:
                    r["prev_stage"] = self.stage_ranks[i - 1]
                if i + 1 < self.num_stages:
                    r["next_stage"] = self.stage_ranks[i + 1]
                c.ranks = r
            ranks = {s: r for s, r in zip(self.stage_names, self.stage_ranks)}
            ranks["coordinator"] = self.coordinator_rank
            self.transport = P2PTransport("coordinator", ranks, self.p2p_groups)
        else:
            self.transport = MessageTransport(self.codec)

    def _check_links(self) -> None:
        alive = set(self.comm.peers())
        for s in self.stage_names:
            if s not in alive:
                raise StageFailure(s, "control-plane connection lost")

    def _restart_stages(self) -> None:
        """Re-dial every stage endpoint (the connect loop retries until the worker, restarted by
        its supervisor, listens again) and send it a fresh configuration."""
        for i, ep in enumerate(self.stage_endpoints):
            self.comm.connect(self.stage_names[i], ep.get("host"), int(ep.get("port")), int(self.timeout_s * 1000))

    def _endpoint(self, i):
        ep = self.stage_endpoints[i]
        return Endpoint("tcp", {"host": ep.get("host"), "port": int(ep.get("port")), "id": self.stage_names[i]})

    def _coordinator_endpoint(self):
        return Endpoint("tcp", {"host": self.host, "port": self.port, "id": "coordinator"})

    def stop(self) -> None:
        super().stop()
        if self.transport is not None:
            self.transport.flush()
        time.sleep(0.05)
        if self.comm is not None:
            self.comm.close()
            self.comm = None
