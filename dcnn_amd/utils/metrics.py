"""Structured metrics sink and per-process CPU-usage logger.

The reference reports progress with prints (``include/nn/train.hpp:130-268``) and measures its
distributed runs from outside: a logger samples each container's CPU utilisation into
``<tag>_*.csv`` files (``t_sec, cpu_percent, tag``) that ``src/plot_cpu_range.py:1-118`` plots.
Here both are library pieces:

* :class:`MetricsSink` — append-only JSON-lines records (``{"t": ..., "event": ..., **fields}``)
  the trainers (``nn/train.py``, ``parallel/pipeline/train.py``) emit per batch-log interval and
  per epoch (images/s, loss, accuracy, learning rate, memory), to a file named by ``METRICS_FILE``
  or passed in. Optionally mirrored to Prometheus gauges (``prometheus_client``, when importable
  and ``METRICS_PROMETHEUS_PORT`` is set) for live scraping.
* :class:`CpuUsageLogger` — a background thread sampling a process's CPU time from
  ``/proc/<pid>/stat`` (or the whole machine from ``/proc/stat``) into the reference's CSV format,
  so ``tools/plot_cpu_range.py`` plots coordinator/worker CPU use the same way. Pipeline workers
  start one when ``CPU_LOG_DIR`` is set.
"""
from __future__ import annotations

import csv
import json
import os
import threading
import time
from typing import Optional


class MetricsSink:
    """JSON-lines metrics records; a no-op when constructed with no path and no env."""

    def __init__(self, path: Optional[str] = None, tag: str = "", prometheus_port: Optional[int] = None):
        self.path = path if path is not None else os.environ.get("METRICS_FILE", "")
        self.tag = tag
        self._lock = threading.Lock()
        self._f = None
        self._t0 = time.time()
        if self.path:
            os.makedirs(os.path.dirname(os.path.abspath(self.path)), exist_ok=True)
            self._f = open(self.path, "a", buffering=1)
        self._gauges = {}
        self._prom = None
        port = prometheus_port if prometheus_port is not None else int(os.environ.get("METRICS_PROMETHEUS_PORT", "0"))
        if port:
            try:
                import prometheus_client as pc
                pc.start_http_server(port, addr="127.0.0.1")
                self._prom = pc
            except Exception:  # optional: a sink without the mirror still works
                self._prom = None

    @property
    def enabled(self) -> bool:
        return self._f is not None or self._prom is not None

    def log(self, event: str, **fields) -> None:
        if not self.enabled:
            return
        rec = {"t": round(time.time() - self._t0, 6), "event": event}
        if self.tag:
            rec["tag"] = self.tag
        rec.update({k: (float(v) if hasattr(v, "item") else v) for k, v in fields.items()})
        with self._lock:
            if self._f is not None:
                self._f.write(json.dumps(rec) + "\n")
            if self._prom is not None:
                for k, v in rec.items():
                    if isinstance(v, (int, float)) and k != "t":
                        name = f"dcnn_{event}_{k}".replace("-", "_").replace(".", "_")
                        g = self._gauges.get(name)
                        if g is None:
                            g = self._gauges[name] = self._prom.Gauge(name, f"{event} {k}")
                        g.set(v)

    def close(self) -> None:
        with self._lock:
            if self._f is not None:
                self._f.close()
                self._f = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def read_metrics(path: str):
    """All records of a JSON-lines metrics file."""
    with open(path) as f:
        return [json.loads(line) for line in f if line.strip()]


_CLK = os.sysconf("SC_CLK_TCK") if hasattr(os, "sysconf") else 100


def _proc_cpu_seconds(pid: int) -> float:
    with open(f"/proc/{pid}/stat") as f:
        parts = f.read().rsplit(")", 1)[1].split()
    # fields after the comm: state(0) ... utime(11) stime(12) cutime(13) cstime(14)
    return (int(parts[11]) + int(parts[12]) + int(parts[13]) + int(parts[14])) / _CLK


def _machine_busy_total():
    with open("/proc/stat") as f:
        v = [int(x) for x in f.readline().split()[1:]]
    idle = v[3] + (v[4] if len(v) > 4 else 0)
    return sum(v) - idle, sum(v)


class CpuUsageLogger:
    """Samples CPU utilisation every ``interval`` seconds into ``<log_dir>/<tag>_<stamp>.csv``.

    ``pid``: a process (default: this one; its children's reaped time included), in percent of
    one core like ``top`` / ``docker stats``; ``pid=0``: the whole machine in percent of all cores.
    """

    def __init__(self, log_dir: str, tag: str, interval: float = 0.5, pid: Optional[int] = None):
        self.tag, self.interval = tag, interval
        self.pid = os.getpid() if pid is None else pid
        os.makedirs(log_dir, exist_ok=True)
        self.path = os.path.join(log_dir, f"{tag}_{time.strftime('%Y%m%d_%H%M%S')}_{os.getpid()}.csv")
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self.samples = 0

    def _sample(self):
        if self.pid:
            return _proc_cpu_seconds(self.pid), time.monotonic()
        busy, total = _machine_busy_total()
        return busy, total

    def _run(self):
        with open(self.path, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["t_sec", "cpu_percent", "tag"])
            t0 = time.monotonic()
            prev = self._sample()
            while not self._stop.wait(self.interval):
                try:
                    cur = self._sample()
                except OSError:  # the process is gone
                    break
                d0, d1 = cur[0] - prev[0], cur[1] - prev[1]
                pct = 100.0 * d0 / d1 if d1 > 0 else 0.0
                prev = cur
                w.writerow([f"{time.monotonic() - t0:.3f}", f"{pct:.2f}", self.tag])
                f.flush()
                self.samples += 1

    def start(self) -> "CpuUsageLogger":
        self._thread = threading.Thread(target=self._run, name=f"cpu-log-{self.tag}", daemon=True)
        self._thread.start()
        return self

    def stop(self) -> str:
        self._stop.set()
        if self._thread is not None:
            self._thread.join()
        return self.path

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()


def maybe_start_cpu_logger(tag: str) -> Optional[CpuUsageLogger]:
    """A running :class:`CpuUsageLogger` for this process when ``CPU_LOG_DIR`` is set."""
    d = os.environ.get("CPU_LOG_DIR", "")
    if not d:
        return None
    return CpuUsageLogger(d, tag, float(os.environ.get("CPU_LOG_INTERVAL", "0.5"))).start()
