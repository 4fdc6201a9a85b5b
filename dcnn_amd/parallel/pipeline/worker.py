"""Network stage worker (reference examples/network_worker.cpp:14-194 and
include/pipeline/network_stage_worker.hpp:25-114).

    python -m dcnn_amd.parallel.pipeline.worker <port> [--gpu] [--device GPU:1]
                                                     [--num-threads N] [--ecore] [--show-cores]

Listens on ``port`` with the native TCP communicator, waits for CONFIG_TRANSFER from the
coordinator and runs the stage event loop until SHUTDOWN.  ``--ecore`` pins the process to
the efficiency cores reported by the native hardware probe (no-op on hosts without a P/E
split).  Under ``torch.distributed`` (``launch.py``) the worker also joins the P2P groups so
activations can move over RCCL.
"""
from __future__ import annotations

import argparse
import os
import sys

import torch


class NetworkStageWorker:
    def __init__(self, port: int, use_gpu: bool = False, device: str = "", host: str = "0.0.0.0",
                 p2p_groups=None, verbose: bool = True):
        from . import messages as M
        from .stage import PipelineStage
        self.comm = M.comm().TcpCommunicator(f"worker@{port}", host, int(port))
        self.port = self.comm.port
        self.stage = PipelineStage(self.comm, p2p_groups=p2p_groups, verbose=verbose)
        self.default_device = device or ("GPU" if use_gpu else "CPU")

    def run(self) -> None:
        from ...utils.metrics import maybe_start_cpu_logger
        cpu_log = maybe_start_cpu_logger(f"worker-{self.port}")  # CPU_LOG_DIR: tools/plot_cpu_range.py input
        try:
            self.stage.run()
        finally:
            self.stage.transport.flush()
            self.comm.close()
            if cpu_log is not None:
                cpu_log.stop()

    def start_thread(self):
        return self.stage.start_thread()


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="dcnn_amd pipeline stage worker")
    ap.add_argument("port", type=int)
    ap.add_argument("--gpu", action="store_true")
    ap.add_argument("--device", default="")
    ap.add_argument("--num-threads", type=int, default=0)
    ap.add_argument("--ecore", action="store_true")
    ap.add_argument("--max-ecores", type=int, default=0)
    ap.add_argument("--show-cores", action="store_true")
    a = ap.parse_args(argv)
    from ...ops._ext import native
    n = native()
    if a.show_cores:
        info = n.read_cpu_info()
        print(f"P-cores: {info['pcores']}\nE-cores: {info['ecores']}", flush=True)
    if a.ecore:
        ecores = list(n.read_cpu_info()["ecores"])
        if a.max_ecores:
            ecores = ecores[:a.max_ecores]
        if ecores:
            n.set_thread_affinity(ecores)
    if a.num_threads:
        torch.set_num_threads(a.num_threads)
    if a.gpu and not torch.cuda.is_available():
        print("--gpu requested but no GPU visible", file=sys.stderr)
        return 2
    w = NetworkStageWorker(a.port, a.gpu, a.device)
    print(f"stage worker listening on port {w.port} (pid {os.getpid()})", flush=True)
    w.run()
    return 0


if __name__ == "__main__":
    sys.exit(main())
