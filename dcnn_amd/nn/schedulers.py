"""Learning-rate schedulers (reference `include/nn/schedulers.hpp:42-698`, same step semantics).

Unlike the reference (G14: schedulers never used by a driver) the trainers here accept a
scheduler and step it per optimizer step or per epoch.
"""
from __future__ import annotations

import math
from typing import List, Optional


class SchedulerConfig(dict):
    def __init__(self, type: str, name: str = "", parameters: Optional[dict] = None):
        super().__init__(type=type, name=name or type, parameters=dict(parameters or {}))

    @property
    def type(self):
        return self["type"]

    def get(self, k, d=None):  # type: ignore[override]
        if k in ("type", "name", "parameters"):
            return super().get(k, d)
        return self["parameters"].get(k, d)


class Scheduler:
    type_name = "scheduler"

    def __init__(self, optimizer):
        self.optimizer = optimizer
        self.base_lr = optimizer.get_learning_rate() if optimizer is not None else 0.0
        self.current_step = 0

    def step(self, *a):
        raise NotImplementedError

    def get_lr(self) -> float:
        return self.optimizer.get_learning_rate() if self.optimizer is not None else self.base_lr

    def set_lr(self, lr: float) -> None:
        if self.optimizer is not None:
            self.optimizer.set_learning_rate(lr)

    def get_base_lr(self) -> float:
        return self.base_lr

    def get_current_step(self) -> int:
        return self.current_step

    def reset(self) -> None:
        self.current_step = 0
        self.set_lr(self.base_lr)

    def name(self) -> str:
        return type(self).__name__

    def _params(self) -> dict:
        return {}

    def get_config(self) -> SchedulerConfig:
        return SchedulerConfig(self.type_name, self.name(), self._params())


class StepLR(Scheduler):
    type_name = "step_lr"

    def __init__(self, optimizer, step_size: int, gamma: float = 0.1):
        super().__init__(optimizer)
        self.step_size, self.gamma = int(step_size), float(gamma)

    def step(self):
        self.current_step += 1
        if self.current_step % self.step_size == 0:
            self.set_lr(self.get_lr() * self.gamma)

    def _params(self):
        return {"step_size": self.step_size, "gamma": self.gamma}


class MultiStepLR(Scheduler):
    type_name = "multi_step_lr"

    def __init__(self, optimizer, milestones: List[int], gamma: float = 0.1):
        super().__init__(optimizer)
        self.milestones = sorted(int(m) for m in milestones)
        self.gamma = float(gamma)
        self.idx = 0

    def step(self):
        self.current_step += 1
        if self.idx < len(self.milestones) and self.current_step >= self.milestones[self.idx]:
            self.set_lr(self.get_lr() * self.gamma)
            self.idx += 1

    def reset(self):
        super().reset()
        self.idx = 0

    def _params(self):
        return {"milestones": self.milestones, "gamma": self.gamma}


class ExponentialLR(Scheduler):
    type_name = "exponential_lr"

    def __init__(self, optimizer, gamma: float = 0.95):
        super().__init__(optimizer)
        self.gamma = float(gamma)

    def step(self):
        self.current_step += 1
        self.set_lr(self.get_lr() * self.gamma)

    def _params(self):
        return {"gamma": self.gamma}


class CosineAnnealingLR(Scheduler):
    type_name = "cosine_annealing_lr"

    def __init__(self, optimizer, T_max: int, eta_min: float = 0.0):
        super().__init__(optimizer)
        self.T_max, self.eta_min = int(T_max), float(eta_min)

    def step(self):
        self.current_step += 1
        s = self.current_step % self.T_max
        self.set_lr(self.eta_min + (self.base_lr - self.eta_min) * (1 + math.cos(math.pi * s / self.T_max)) / 2)

    def _params(self):
        return {"T_max": self.T_max, "eta_min": self.eta_min}


class CosineAnnealingWarmRestarts(Scheduler):
    type_name = "cosine_annealing_warm_restarts"

    def __init__(self, optimizer, T_0: int, T_mult: int = 1, eta_min: float = 0.0):
        super().__init__(optimizer)
        self.T_0, self.T_mult, self.eta_min = int(T_0), int(T_mult), float(eta_min)
        self.T_cur, self.T_i = 0, self.T_0

    def step(self):
        self.current_step += 1
        self.T_cur += 1
        if self.T_cur >= self.T_i:
            self.T_cur = 0
            self.T_i *= self.T_mult
        self.set_lr(self.eta_min + (self.base_lr - self.eta_min) * (1 + math.cos(math.pi * self.T_cur / self.T_i)) / 2)

    def reset(self):
        super().reset()
        self.T_cur, self.T_i = 0, self.T_0

    def _params(self):
        return {"T_0": self.T_0, "T_mult": self.T_mult, "eta_min": self.eta_min}


class LinearWarmup(Scheduler):
    type_name = "linear_warmup"

    def __init__(self, optimizer, warmup_steps: int, start_lr: float = 0.0):
        super().__init__(optimizer)
        self.warmup_steps, self.start_lr = int(warmup_steps), float(start_lr)
        self.set_lr(self.start_lr)

    def step(self):
        self.current_step += 1
        if self.current_step <= self.warmup_steps:
            p = self.current_step / self.warmup_steps
            self.set_lr(self.start_lr + p * (self.base_lr - self.start_lr))

    def is_warmup_complete(self):
        return self.current_step >= self.warmup_steps

    def _params(self):
        return {"warmup_steps": self.warmup_steps, "start_lr": self.start_lr}


class WarmupCosineAnnealing(Scheduler):
    type_name = "warmup_cosine_annealing"

    def __init__(self, optimizer, warmup_steps: int, total_steps: int, start_lr: float = 0.0, eta_min: float = 0.0):
        super().__init__(optimizer)
        self.warmup_steps, self.total_steps = int(warmup_steps), int(total_steps)
        self.start_lr, self.eta_min = float(start_lr), float(eta_min)
        self.set_lr(self.start_lr)

    def step(self):
        self.current_step += 1
        if self.current_step <= self.warmup_steps:
            p = self.current_step / self.warmup_steps
            self.set_lr(self.start_lr + p * (self.base_lr - self.start_lr))
        else:
            p = min((self.current_step - self.warmup_steps) / (self.total_steps - self.warmup_steps), 1.0)
            self.set_lr(self.eta_min + (self.base_lr - self.eta_min) * (1 + math.cos(math.pi * p)) / 2)

    def _params(self):
        return {"warmup_steps": self.warmup_steps, "total_steps": self.total_steps, "start_lr": self.start_lr,
                "eta_min": self.eta_min}


class ReduceLROnPlateau(Scheduler):
    type_name = "reduce_lr_on_plateau"

    def __init__(self, optimizer, mode: str = "min", factor: float = 0.1, patience: int = 10,
                 threshold: float = 1e-4, min_lr: float = 0.0):
        super().__init__(optimizer)
        self.mode, self.factor, self.patience = mode, float(factor), int(patience)
        self.threshold, self.min_lr = float(threshold), float(min_lr)
        self.best = 1e10 if mode == "min" else -1e10
        self.bad = 0

    def step(self, metric: Optional[float] = None):
        self.current_step += 1
        if metric is None:
            return
        better = metric < self.best - self.threshold if self.mode == "min" else metric > self.best + self.threshold
        if better:
            self.best, self.bad = metric, 0
        else:
            self.bad += 1
            if self.bad >= self.patience:
                self.set_lr(max(self.get_lr() * self.factor, self.min_lr))
                self.bad = 0

    def reset(self):
        super().reset()
        self.best = 1e10 if self.mode == "min" else -1e10
        self.bad = 0

    def _params(self):
        return {"mode": self.mode, "factor": self.factor, "patience": self.patience, "threshold": self.threshold,
                "min_lr": self.min_lr}


class PolynomialLR(Scheduler):
    type_name = "polynomial_lr"

    def __init__(self, optimizer, total_steps: int, power: float = 1.0, end_lr: float = 0.0):
        super().__init__(optimizer)
        self.total_steps, self.power, self.end_lr = int(total_steps), float(power), float(end_lr)

    def step(self):
        self.current_step += 1
        p = min(self.current_step / self.total_steps, 1.0)
        self.set_lr((self.base_lr - self.end_lr) * (1 - p) ** self.power + self.end_lr)

    def _params(self):
        return {"total_steps": self.total_steps, "power": self.power, "end_lr": self.end_lr}


class OneCycleLR(Scheduler):
    type_name = "one_cycle_lr"

    def __init__(self, optimizer, max_lr: float, total_steps: int, pct_start: float = 0.3, div_factor: float = 25.0,
                 final_div_factor: float = 1e4):
        super().__init__(optimizer)
        self.max_lr, self.total_steps = float(max_lr), int(total_steps)
        self.pct_start, self.div_factor, self.final_div_factor = float(pct_start), float(div_factor), float(final_div_factor)
        self.initial_lr = self.max_lr / self.div_factor
        self.min_lr = self.initial_lr / self.final_div_factor
        self.step_up = int(self.total_steps * self.pct_start)
        self.step_down = self.total_steps - self.step_up
        self.set_lr(self.initial_lr)

    def step(self):
        self.current_step += 1
        if self.current_step <= self.step_up:
            p = self.current_step / self.step_up
            lr = self.initial_lr + p * (self.max_lr - self.initial_lr)
        else:
            p = (self.current_step - self.step_up) / self.step_down
            lr = self.min_lr + (self.max_lr - self.min_lr) * (1 + math.cos(math.pi * p)) / 2
        self.set_lr(lr)

    def _params(self):
        return {"max_lr": self.max_lr, "total_steps": self.total_steps, "pct_start": self.pct_start,
                "div_factor": self.div_factor, "final_div_factor": self.final_div_factor}


class SchedulerFactory:
    @staticmethod
    def create(name: str, optimizer, params: Optional[dict] = None) -> Scheduler:
        return SchedulerFactory.create_from_config(SchedulerConfig(name, name, params or {}), optimizer)

    @staticmethod
    def create_from_config(cfg, optimizer) -> Scheduler:
        if not isinstance(cfg, SchedulerConfig):
            cfg = SchedulerConfig(cfg["type"], cfg.get("name", ""), cfg.get("parameters", {}))
        t, g = cfg.type, cfg.get
        if t == "step_lr":
            return StepLR(optimizer, g("step_size", 10), g("gamma", 0.1))
        if t == "multi_step_lr":
            return MultiStepLR(optimizer, g("milestones", []), g("gamma", 0.1))
        if t == "exponential_lr":
            return ExponentialLR(optimizer, g("gamma", 0.95))
        if t == "cosine_annealing_lr":
            return CosineAnnealingLR(optimizer, g("T_max", 100), g("eta_min", 0.0))
        if t == "cosine_annealing_warm_restarts":
            return CosineAnnealingWarmRestarts(optimizer, g("T_0", 10), g("T_mult", 1), g("eta_min", 0.0))
        if t == "linear_warmup":
            return LinearWarmup(optimizer, g("warmup_steps", 100), g("start_lr", 0.0))
        if t == "warmup_cosine_annealing":
            return WarmupCosineAnnealing(optimizer, g("warmup_steps", 100), g("total_steps", 1000), g("start_lr", 0.0),
                                         g("eta_min", 0.0))
        if t == "reduce_lr_on_plateau":
            return ReduceLROnPlateau(optimizer, g("mode", "min"), g("factor", 0.1), g("patience", 10),
                                     g("threshold", 1e-4), g("min_lr", 0.0))
        if t == "polynomial_lr":
            return PolynomialLR(optimizer, g("total_steps", 100), g("power", 1.0), g("end_lr", 0.0))
        if t == "one_cycle_lr":
            return OneCycleLR(optimizer, g("max_lr", 0.1), g("total_steps", 100), g("pct_start", 0.3),
                              g("div_factor", 25.0), g("final_div_factor", 1e4))
        raise ValueError(f"Unknown scheduler type: {t}")
