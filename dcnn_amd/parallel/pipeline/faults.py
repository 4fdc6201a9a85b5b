"""Failure detection and fault injection for the pipeline runtime.

The reference pipeline only has join timeouts (``Coordinator::join`` with 60 s /
30 s defaults, no retry, reconnect, heartbeat or fault injection). Here:

* :class:`Heartbeat` — a stage-side thread that sends an unsolicited ``HEALTH_CHECK`` message
  with the text ``"heartbeat"`` to the coordinator every ``interval_s``. It runs beside the
  stage's event loop, so a stage busy with a long job still beats; a stage whose process or
  thread died stops beating. The coordinator (``Coordinator._check_errors``) raises
  ``coordinator.StageFailure`` naming the stage once ``misses`` intervals pass without a beat —
  seconds instead of the job timeout.
* :class:`FaultInjector` — deterministic fault injection for tests and drills: after the
  ``after``-th message of a command the stage ``raise``s (reported as JOB_FAILURE /
  ERROR_REPORT), ``drop``s the message, ``hang``s for ``seconds`` (a stall: heartbeats keep
  coming, the job timeout fires) or ``crash``es (event loop and heartbeat stop, no reply: what
  a killed worker looks like). Configured per stage through ``StageConfig.fault`` or the
  ``DCNN_FAULT`` environment variable (``"stage_1:FORWARD_JOB:3:crash"``, several specs
  separated by ``;``).

Recovery (``Coordinator.enable_recovery`` / ``recover``) lives in coordinator.py: parameter
snapshots every N steps, re-deployment of every stage (in-process stages are re-created, network
stages are re-dialled with the TCP connect retry loop) and a reload of the last snapshot.
"""
from __future__ import annotations

import os
import threading
import time
from dataclasses import dataclass
from typing import Callable, List, Optional

from . import messages as M

C = M.CommandType

HEARTBEAT_TEXT = b"heartbeat"
ACTIONS = ("raise", "drop", "hang", "crash")


class InjectedFault(RuntimeError):
    pass


@dataclass
class FaultSpec:
    command: int          # CommandType value the fault counts
    after: int            # fires on the after-th message of that command (1-based)
    action: str           # raise | drop | hang | crash
    seconds: float = 0.0  # hang duration

    @staticmethod
    def parse(spec) -> "FaultSpec":
        if isinstance(spec, dict):
            cmd = spec["command"]
            after, action, seconds = spec.get("after", 1), spec.get("action", "raise"), spec.get("seconds", 0.0)
        else:
            parts = str(spec).split(":")
            if len(parts) < 3:
                raise ValueError(f"fault spec '{spec}': expected COMMAND:AFTER:ACTION[:SECONDS]")
            cmd, after, action = parts[0], parts[1], parts[2]
            seconds = float(parts[3]) if len(parts) > 3 else 0.0
        if isinstance(cmd, str):
            cmd = int(getattr(C, cmd))
        if action not in ACTIONS:
            raise ValueError(f"fault action '{action}' not one of {ACTIONS}")
        return FaultSpec(int(cmd), int(after), action, float(seconds))

    def to_json(self) -> dict:
        return {"command": M.command_name(self.command), "after": self.after, "action": self.action,
                "seconds": self.seconds}


def env_faults(stage_id: str) -> List[FaultSpec]:
    """Specs of ``DCNN_FAULT`` ("STAGE:COMMAND:AFTER:ACTION[:SECONDS]; ...") for ``stage_id``."""
    out = []
    for item in os.environ.get("DCNN_FAULT", "").split(";"):
        item = item.strip()
        if not item:
            continue
        stage, rest = item.split(":", 1)
        if stage == stage_id:
            out.append(FaultSpec.parse(rest))
    return out


class FaultInjector:
    def __init__(self, specs: List[FaultSpec]):
        self.specs = list(specs)
        self.seen = {}
        self.fired: List[FaultSpec] = []

    def __bool__(self):
        return bool(self.specs)

    def check(self, command: int) -> Optional[str]:
        """Count one message of ``command``; the action to take now (or None)."""
        command = int(command)
        self.seen[command] = self.seen.get(command, 0) + 1
        for s in self.specs:
            if s.command == command and self.seen[command] == s.after and s not in self.fired:
                self.fired.append(s)
                if s.action == "hang":
                    time.sleep(s.seconds)
                    return None
                return s.action
        return None


class Heartbeat:
    """Sends ``HEALTH_CHECK("heartbeat")`` to the coordinator every ``interval_s`` until stopped."""

    def __init__(self, send: Callable[[object], None], interval_s: float):
        self.send = send
        self.interval_s = float(interval_s)
        self._stop = threading.Event()
        self.thread = threading.Thread(target=self._run, name="pipeline-heartbeat", daemon=True)
        self.beats = 0

    def start(self) -> "Heartbeat":
        self.thread.start()
        return self

    def stop(self) -> None:
        self._stop.set()

    def _run(self) -> None:
        while not self._stop.is_set():
            m = M.Message("coordinator", C.HEALTH_CHECK)
            m.text = HEARTBEAT_TEXT
            try:
                self.send(m)
                self.beats += 1
            except Exception:
                pass  # coordinator gone / connection down: keep trying until stopped
            self._stop.wait(self.interval_s)
