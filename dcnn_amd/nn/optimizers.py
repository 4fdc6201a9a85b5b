"""Optimizers (reference `include/nn/optimizers.hpp:25-306`): SGD(+momentum), Adam, AdamW.

``attach(params, grads)`` as in the reference. When the attached tensors are exactly the views
of one :class:`ParamArena` (the normal case: a Sequential or a pipeline stage), the update is
ONE fused kernel over the flat buffer which also refreshes the bf16 shadow weights. The step
scalars live in a tiny device tensor ``{lr, bc1, bc2, t}``: Adam's step counter and bias
corrections advance ON THE DEVICE (``adam_scalars``, captured in the step graph ahead of the
update), and the learning rate is uploaded only when it changes — a replayed training step needs
no host-to-device transfer besides its input batch. A CPU arena is updated by the native
backend's flat-buffer loops (``ops/cpu.py``), in the arena's dtype (float32 or float64).
"""
from __future__ import annotations

import math
from typing import List, Optional

import torch


class OptimizerConfig(dict):
    def __init__(self, type: str, name: str = "", parameters: Optional[dict] = None):
        super().__init__(type=type, name=name, parameters=dict(parameters or {}))

    @property
    def type(self):
        return self["type"]

    def to_json(self):
        return dict(self)

    @staticmethod
    def from_json(j):
        return OptimizerConfig(j.get("type", ""), j.get("name", ""), j.get("parameters", {}))


def _arena_of(params: List[torch.Tensor]):
    """Return the ParamArena if params are exactly its views in order (fused flat path)."""
    if not params:
        return None
    base = params[0]._base if params[0]._base is not None else None
    if base is None:
        return None
    for p in params:
        if p._base is None or p._base.data_ptr() != base.data_ptr():
            return None
    return base


class Optimizer:
    def __init__(self, learning_rate: float):
        self.learning_rate = float(learning_rate)
        self.params: List[torch.Tensor] = []
        self.grads: List[torch.Tensor] = []
        self.arena = None
        self._flat_p = self._flat_g = None
        self._hyper = None
        self._hyper_dirty = True  # device scalars must be (re)uploaded before the next step

    def attach(self, params, grads=None, arena=None) -> None:
        if grads is None and hasattr(params, "parameters"):
            model = params
            params, grads = model.parameters(), model.gradients()
            arena = getattr(model, "arena", None)
        self.params, self.grads = list(params), list(grads)
        if len(self.params) != len(self.grads):
            raise ValueError("params/grads length mismatch")
        self.arena = arena
        if self.arena is not None:
            ptrs = [p.data_ptr() for p in self.params]
            own = [self.arena.param(i).data_ptr() for i in range(len(self.arena.specs))]
            if ptrs != own:
                self.arena = None
        if self.arena is not None:
            self._flat_p, self._flat_g = self.arena.data, self.arena.grad
        # re-attaching resets the step state (Adam t, m, v): the device scalars (step counter,
        # learning rate) must be re-uploaded too, or the device keeps counting from the old t
        self._hyper_dirty = True
        self._on_attach()

    def _on_attach(self):
        pass

    def update(self) -> None:
        raise NotImplementedError

    step = property(lambda self: self.update)

    def clear_gradients(self) -> None:
        if self.arena is not None:
            self.arena.zero_grad()
        else:
            for g in self.grads:
                g.zero_()

    zero_grad = clear_gradients

    def set_learning_rate(self, lr: float) -> None:
        if float(lr) != self.learning_rate:
            self._hyper_dirty = True
        self.learning_rate = float(lr)

    def get_learning_rate(self) -> float:
        return self.learning_rate

    _HYPER_SLOTS = 8

    def _device_hyper(self, vals):
        """Device copy of step scalars (read by the kernel; graph-replay safe).

        Uploaded from a ring of pinned host slots with an asynchronous copy: a pageable copy
        would be staged synchronously and stall the host until the stream drains, so the next
        step's graph launches could not run ahead of the GPU. A slot is rewritten only after the
        event of its previous copy has completed (eight steps earlier, in practice never waits).
        """
        dev = self._flat_p.device
        if self._hyper is None:
            self._hyper = torch.zeros(4, dtype=torch.float32, device=dev)
            self._hyper_host = torch.zeros(self._HYPER_SLOTS, 4, dtype=torch.float32).pin_memory()
            self._hyper_ev = [None] * self._HYPER_SLOTS
            self._hyper_i = 0
        k = self._hyper_i
        self._hyper_i = (k + 1) % self._HYPER_SLOTS
        if self._hyper_ev[k] is not None:
            self._hyper_ev[k].synchronize()
        slot = self._hyper_host[k]
        slot.copy_(torch.tensor(list(vals) + [0.0] * (4 - len(vals)), dtype=torch.float32))
        # the copy and the event that guards the pinned slot go on the SAME stream: the current
        # stream of the arena's device (a pipeline stage thread may have another device current)
        s = torch.cuda.current_stream(dev)
        with torch.cuda.stream(s):
            self._hyper.copy_(slot, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(s)
        self._hyper_ev[k] = ev
        return self._hyper

    def state_dict(self) -> dict:
        return {}

    def load_state_dict(self, d: dict) -> None:
        pass


class SGD(Optimizer):
    def __init__(self, learning_rate: float = 0.01, momentum: float = 0.0):
        super().__init__(learning_rate)
        self.momentum = float(momentum)
        self.velocity = None

    def _on_attach(self):
        if self.momentum > 0:
            if self.arena is not None:
                self.velocity = [self.arena.new_zeros()]
            else:
                self.velocity = [torch.zeros_like(p) for p in self.params]

    def prepare_step(self):
        if self.arena is not None and self._flat_p.is_cuda and (self._hyper_dirty or self._hyper is None):
            self._device_hyper([self.learning_rate])
            self._hyper_dirty = False

    def launch_step(self):
        from ..ops import hip
        hip.sgd_step(self._flat_p, self._flat_g, self.velocity[0] if self.momentum > 0 else None, self.arena.shadow,
                     self.learning_rate, self.momentum, self._hyper)
        self.arena.mark_synced()

    def fused(self) -> bool:
        return self.arena is not None and self._flat_p.is_cuda

    def update(self):
        if self.arena is not None:
            p, g = self._flat_p, self._flat_g
            if p.is_cuda:
                self.prepare_step()
                self.launch_step()
                return
            from ..ops import cpu
            cpu.sgd_step(p, g, self.velocity[0] if self.momentum > 0 else None, self.learning_rate, self.momentum)
            self.arena.sync_shadow()
            return
        for i, (p, g) in enumerate(zip(self.params, self.grads)):
            self._sgd_torch(p, g, self.velocity[i] if self.momentum > 0 else None)

    def _sgd_torch(self, p, g, v):
        with torch.no_grad():
            if v is not None:
                v.mul_(self.momentum).sub_(self.learning_rate * g)
                p.add_(v)
            else:
                p.sub_(self.learning_rate * g)

    def name(self):
        return "SGD"

    def get_config(self):
        return OptimizerConfig("sgd", "SGD", {"learning_rate": self.learning_rate, "momentum": self.momentum})

    def clone(self):
        return SGD(self.learning_rate, self.momentum)

    def state_dict(self):
        return {"velocity": [v.detach().cpu() for v in self.velocity] if self.velocity else []}

    def load_state_dict(self, d):
        if d.get("velocity") and self.velocity:
            for v, s in zip(self.velocity, d["velocity"]):
                v.copy_(s)


class Adam(Optimizer):
    def __init__(self, learning_rate: float = 0.001, beta1: float = 0.9, beta2: float = 0.999,
                 epsilon: float = 1e-8, weight_decay: float = 0.0, decouple_weight_decay: bool = False):
        super().__init__(learning_rate)
        self.beta1, self.beta2, self.epsilon = float(beta1), float(beta2), float(epsilon)
        self.weight_decay = float(weight_decay)
        self.decouple_weight_decay = bool(decouple_weight_decay)
        self.t = 0
        self.m = self.v = None

    def _on_attach(self):
        if self.arena is not None:
            self.m = [self.arena.new_zeros()]
            self.v = [self.arena.new_zeros()]
        else:
            self.m = [torch.zeros_like(p) for p in self.params]
            self.v = [torch.zeros_like(p) for p in self.params]
        self.t = 0

    def fused(self) -> bool:
        return self.arena is not None and self._flat_p.is_cuda

    def prepare_step(self):
        """Host side of a step (graph-replay safe): advance the host step counter; upload the
        device scalars only when stale (first step, learning-rate change, loaded state) — the
        device counter then equals t - 1 and ``launch_step`` advances it on the device."""
        self.t += 1
        self._bc = (1.0 - self.beta1 ** self.t, 1.0 - self.beta2 ** self.t)
        if self.fused() and (self._hyper_dirty or self._hyper is None):
            self._device_hyper([self.learning_rate, 0.0, 0.0, float(self.t - 1)])
            self._hyper_dirty = False

    def launch_step(self):
        """Device side: the scalar update (t, bias corrections) and ONE kernel over the flat
        buffer, both reading their scalars from device memory."""
        from ..ops import hip
        from ..ops._ext import kernels, stream_ptr
        kernels().adam_scalars(self._hyper.data_ptr(), float(self.beta1), float(self.beta2),
                               stream_ptr(self._flat_p.device))
        bc1, bc2 = self._bc
        hip.adam_step(self._flat_p, self._flat_g, self.m[0], self.v[0], self.arena.shadow, self.learning_rate,
                      self.beta1, self.beta2, self.epsilon, bc1, bc2, self.weight_decay,
                      self.decouple_weight_decay, self._hyper)
        self.arena.mark_synced()

    def update(self):
        if self.fused():
            self.prepare_step()
            self.launch_step()
            return
        self.t += 1
        bc1 = 1.0 - self.beta1 ** self.t
        bc2 = 1.0 - self.beta2 ** self.t
        if self.arena is not None and not self._flat_p.is_cuda:
            from ..ops import cpu   # native flat-buffer step (CPU arena, float32 or float64)
            cpu.adam_step(self._flat_p, self._flat_g, self.m[0], self.v[0], self.learning_rate, self.beta1,
                          self.beta2, self.epsilon, bc1, bc2, self.weight_decay, self.decouple_weight_decay)
            self.arena.sync_shadow()
            return
        pairs = [(self._flat_p, self._flat_g)] if self.arena is not None else list(zip(self.params, self.grads))
        with torch.no_grad():
            for i, (p, g) in enumerate(pairs):
                m, v = self.m[i], self.v[i]
                m.mul_(self.beta1).add_((1 - self.beta1) * g)
                v.mul_(self.beta2).add_((1 - self.beta2) * g * g)
                upd = self.learning_rate * (m / bc1) / (torch.sqrt(v / bc2) + self.epsilon)
                if self.weight_decay > 0:
                    if self.decouple_weight_decay:
                        p.sub_(self.weight_decay * self.learning_rate * p)
                    else:
                        upd = upd + self.weight_decay * self.learning_rate * p
                p.sub_(upd)
        if self.arena is not None:
            self.arena.sync_shadow()

    def name(self):
        return "AdamW" if self.decouple_weight_decay else "Adam"

    def get_config(self):
        t = "adamw" if self.decouple_weight_decay else "adam"
        return OptimizerConfig(t, self.name(), dict(learning_rate=self.learning_rate, beta1=self.beta1,
                                                    beta2=self.beta2, epsilon=self.epsilon,
                                                    weight_decay=self.weight_decay,
                                                    decouple_weight_decay=self.decouple_weight_decay))

    def clone(self):
        return Adam(self.learning_rate, self.beta1, self.beta2, self.epsilon, self.weight_decay,
                    self.decouple_weight_decay)

    def state_dict(self):
        return {"t": self.t, "m": [x.detach().cpu() for x in self.m or []], "v": [x.detach().cpu() for x in self.v or []]}

    def load_state_dict(self, d):
        self.t = int(d.get("t", 0))
        self._hyper_dirty = True
        for dst, src in zip(self.m or [], d.get("m", [])):
            dst.copy_(src)
        for dst, src in zip(self.v or [], d.get("v", [])):
            dst.copy_(src)


class AdamW(Adam):
    def __init__(self, learning_rate=0.001, beta1=0.9, beta2=0.999, epsilon=1e-8, weight_decay=0.01):
        super().__init__(learning_rate, beta1, beta2, epsilon, weight_decay, True)


class OptimizerFactory:
    @staticmethod
    def create_from_config(config) -> Optimizer:
        if isinstance(config, dict) and not isinstance(config, OptimizerConfig):
            config = OptimizerConfig.from_json(config)
        t = config["type"]
        p = config["parameters"]
        if t == "sgd":
            return SGD(p.get("learning_rate", 0.01), p.get("momentum", 0.0))
        if t in ("adam", "adamw"):
            return Adam(p.get("learning_rate", 0.001), p.get("beta1", 0.9), p.get("beta2", 0.999),
                        p.get("epsilon", 1e-8), p.get("weight_decay", 0.0),
                        p.get("decouple_weight_decay", t == "adamw"))
        raise ValueError(f"Unknown optimizer type: {t}")
