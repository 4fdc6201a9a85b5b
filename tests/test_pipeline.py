"""Pipeline parallelism: partitioners, in-process coordinator parity with single-process
micro-batched training, control commands, and the multi-process TCP + gloo-P2P path."""
import json
import os
import subprocess
import sys

import pytest
import torch

from dcnn_amd.models import zoo
from dcnn_amd.nn.loss import LossFactory
from dcnn_amd.nn.optimizers import SGD, Adam
from dcnn_amd.nn.sequential import Partition
from dcnn_amd.parallel.pipeline import (FlopPartitioner, InProcessCoordinator, NaivePartitioner, StageConfig,
                                        Endpoint, balanced_split)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_naive_partitioner_matches_reference_rule():
    m = zoo.create_model("resnet18_tiny_imagenet")
    L = len(m.layers)
    parts = NaivePartitioner().get_partitions(m, 3)
    base, rem = divmod(L, 3)
    sizes = [p.end_layer - p.start_layer for p in parts]
    assert sizes == [base + (1 if i < rem else 0) for i in range(3)]
    assert parts[0].start_layer == 0 and parts[-1].end_layer == L


def test_balanced_split_is_optimal():
    costs = [5, 1, 1, 1, 8, 2, 2]
    parts = balanced_split(costs, 3)
    sums = [sum(costs[p.start_layer:p.end_layer]) for p in parts]
    assert max(sums) == 8
    assert [(p.start_layer, p.end_layer) for p in parts][-1][1] == len(costs)


def test_flop_partitioner_balances_better_than_naive():
    m = zoo.create_model("resnet50_tiny_imagenet")
    shape = [32, 3, 64, 64]
    f = [a + b for a, b in zip(m.forward_complexity(shape), m.backward_complexity(shape))]

    def worst(parts):
        return max(sum(f[p.start_layer:p.end_layer]) for p in parts)

    flop = FlopPartitioner(shape).get_partitions(m, 4)
    naive = NaivePartitioner().get_partitions(m, 4)
    assert worst(flop) <= worst(naive)


def test_stage_config_json_roundtrip():
    c = StageConfig("stage_1", 1, 2, {"name": "m", "layers": []}, {"type": "adam", "parameters": {}},
                    next_stage_endpoint=Endpoint.network("127.0.0.1", 9000),
                    coordinator_endpoint=Endpoint.in_process("coord"), ranks={"coordinator": 0})
    d = StageConfig.from_json(c.dumps())
    assert d.next_stage_endpoint.get("port") == 9000
    assert d.coordinator_endpoint.communication_type == "in_process"
    assert d.prev_stage_endpoint is None and d.ranks == {"coordinator": 0}


def _reference_microbatched(model, x, y, m, opt, lossname="softmax_crossentropy", scale=True):
    lf = LossFactory.create(lossname)
    if not opt.params:
        opt.attach(model)
    n = x.shape[0] // m
    tot = 0.0
    for i in range(m):
        out = model.forward(x[i * n:(i + 1) * n], i)
        l, g, _ = lf.loss_and_grad(out, y[i * n:(i + 1) * n])
        tot += float(l)
        model.backward(g / m if scale else g, i)
    opt.update()
    opt.clear_gradients()
    return tot / m


@pytest.mark.parametrize("schedule", ["sync", "semi_async"])
@pytest.mark.parametrize("transport", ["local", "message"])
def test_inprocess_pipeline_matches_single_process(schedule, transport):
    torch.manual_seed(0)
    model = zoo.create_model("resnet9_cifar10")
    model.set_seed(3)
    model.initialize()
    ref = model.clone()
    ref.initialize()
    ref.load_parameters([p.clone() for p in model.parameters()])
    x = torch.randn(8, 3, 32, 32)
    y = torch.randint(0, 10, (8,))
    coord = InProcessCoordinator(model, Adam(1e-3), "softmax_crossentropy", num_stages=3, num_microbatches=4,
                                 transport=transport)
    try:
        coord.initialize()
        coord.deploy_stages()
        coord.send_parameters(model)
        coord.start()
        losses = [coord.train_step(x, y, schedule) for _ in range(2)]
        ref_opt = Adam(1e-3)
        ref_losses = [_reference_microbatched(ref, x, y, 4, ref_opt) for _ in range(2)]
        assert losses == pytest.approx(ref_losses, rel=1e-5)
        got = coord.gather_model()
        for a, b in zip(got.parameters(), ref.parameters()):
            torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)
    finally:
        coord.stop()


def test_inprocess_control_commands(tmp_path):
    model = zoo.create_model("mnist_cnn")
    coord = InProcessCoordinator(model, SGD(0.05), "softmax_crossentropy", num_stages=2, num_microbatches=2,
                                 partitioner=FlopPartitioner([2, 1, 28, 28]))
    try:
        coord.initialize()
        coord.deploy_stages()
        coord.start()
        x, y = torch.randn(4, 1, 28, 28), torch.randint(0, 10, (4,))
        coord.train_step(x, y)
        assert coord.health_check() == {"stage_0": True, "stage_1": True}
        st = coord.status()
        assert [s["counts"]["forward"] for s in st] == [2, 2]
        assert [s["counts"]["update"] for s in st] == [1, 1]
        loads = coord.load_reports()
        assert set(loads) == {"stage_0", "stage_1"} and all(v[0] > 0 for v in loads.values())
        coord.barrier()
        loss, correct = coord.evaluate_batch(x, y)
        assert loss > 0 and 0 <= correct <= 4
        # learning-rate change reaches every stage
        coord.set_learning_rate(0.01)
        coord.train_step(x, y)
        assert all(s.optimizer.get_learning_rate() == pytest.approx(0.01) for s in coord.stages)
        # checkpoint gathered at the coordinator round-trips through the reference format
        path = str(tmp_path / "pipe_ckpt")
        coord.save_checkpoint(path)
        from dcnn_amd.nn.sequential import Sequential
        re = Sequential.from_file(path)
        for a, b in zip(re.parameters(), coord.model.parameters()):
            torch.testing.assert_close(a, b)
        coord.clear_profiling_data()
    finally:
        coord.stop()


def test_stage_error_is_reported():
    from dcnn_amd.parallel.pipeline import PipelineError
    model = zoo.create_model("mnist_cnn")
    coord = InProcessCoordinator(model, SGD(0.05), "softmax_crossentropy", num_stages=2, num_microbatches=1)
    try:
        coord.initialize()
        coord.deploy_stages()
        with pytest.raises(PipelineError):
            coord.train_step(torch.randn(2, 3, 5, 5), torch.randint(0, 10, (2,)))  # wrong input shape
    finally:
        coord.stop()


@pytest.mark.parametrize("transport,schedule", [("p2p", "semi_async"), ("p2p", "1f1b"), ("message", "sync")])
def test_multiprocess_pipeline_gloo(transport, schedule):
    """3 processes (coordinator co-located with stage 0) over TCP control + gloo P2P data; the
    separate forward / backward groups carry 1F1B's interleaved traffic without blocking."""
    port = 29800 + {"semi_async": 0, "1f1b": 20, "sync": 40}[schedule]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "3",
           "--master-addr", "127.0.0.1", "--master-port", str(port - 100),
           "-m", "dcnn_amd.parallel.pipeline.launch", "--model", "mnist_cnn", "--batch", "8",
           "--microbatches", "4", "--steps", "2", "--warmup", "1", "--cpu", "--base-port", str(port),
           "--transport", transport, "--schedule", schedule]
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{") and "pipeline" in l][-1]
    d = json.loads(line)
    assert d["stages"] == 3 and d["value"] > 0 and d["loss"] == d["loss"]
    # persistent receive slots: every rank allocates at most one buffer per (peer, command,
    # micro-batch) — 4 micro-batches x (activation in, gradient in) — over all 3 steps
    allocs = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{") and "slot_allocs" in l]
    assert len(allocs) == 3
    for a in allocs:
        assert a["steps"] == 3 and a["slot_allocs"] <= (8 if transport == "p2p" else 0), allocs


def _run_schedule(schedule, steps=2, stages=3, mbs=6):
    model = zoo.create_model("mnist_cnn")
    coord = InProcessCoordinator(model, SGD(0.05, 0.9), "softmax_crossentropy", num_stages=stages,
                                 num_microbatches=mbs, partitioner=NaivePartitioner(), seed=5)
    try:
        coord.initialize()
        coord.deploy_stages()
        coord.start()
        g = torch.Generator().manual_seed(2)
        x = torch.randn(12, 1, 28, 28, generator=g)
        y = torch.randint(0, 10, (12,), generator=g)
        losses = [coord.train_step(x, y, schedule) for _ in range(steps)]
        return losses, coord.collect_parameters(), getattr(coord, "max_in_flight_seen", None)
    finally:
        coord.stop()


def test_one_f_one_b_matches_sync_and_bounds_in_flight():
    """1F1B (at most num_stages micro-batches between forward and backward completion) trains
    exactly like GPipe: per stage the backwards arrive in micro-batch order in both schedules and
    the native CPU kernels are deterministic, so losses and parameters are bit-identical."""
    ls, ps, _ = _run_schedule("sync")
    lf, pf, inflight = _run_schedule("1f1b")
    assert inflight is not None and inflight <= 3
    assert ls == lf
    for a, b in zip(ps, pf):
        assert torch.equal(a, b)


def test_unknown_schedule_rejected():
    model = zoo.create_model("mnist_cnn")
    coord = InProcessCoordinator(model, SGD(0.05), "softmax_crossentropy", num_stages=1, num_microbatches=1)
    try:
        coord.initialize()
        coord.deploy_stages()
        with pytest.raises(ValueError):
            coord.train_step(torch.randn(2, 1, 28, 28), torch.randint(0, 10, (2,)), "zigzag")
    finally:
        coord.stop()


class _FakeRcclPlane:
    """Stands in for parallel.rccl.RcclP2P: per-(direction key, src, dst) FIFO queues shared by
    the ranks of one test, recording every call (what P2PTransport's routing chose)."""

    def __init__(self, rank, queues, log):
        self.rank, self.q, self.log = rank, queues, log

    def send(self, key, t, peer):
        self.log.append(("send", key, self.rank, peer, tuple(t.shape), bool(t.is_contiguous())))
        self.q.setdefault((key, self.rank, peer), []).append(t.clone())

    def recv(self, key, t, src):
        self.log.append(("recv", key, src, self.rank, tuple(t.shape)))
        t.copy_(self.q[(key, src, self.rank)].pop(0))
        return t


class _Outbox:
    def __init__(self, sender):
        self.sender, self.sent = sender, []

    def send(self, m):
        m.sender = self.sender
        self.sent.append(m)


def test_p2p_transport_routes_through_rccl_plane():
    """P2PTransport with the in-tree plane (rccl=...): forward jobs between stages ride the "fwd"
    communicator, backward jobs "bwd", traffic to / from the coordinator the "cfwd" / "cbwd" ones;
    channels-last activations travel as their physical NHWC buffer and come back as the same
    logical NCHW tensor; receive slots are reused across steps; rank-local peers bypass RCCL."""
    from dcnn_amd.parallel.pipeline import messages as M
    from dcnn_amd.parallel.pipeline.transport import P2PTransport
    C = M.CommandType
    ranks = {"coordinator": 0, "stage_0": 0, "stage_1": 1}
    q, log = {}, []
    t0 = P2PTransport("stage_0", ranks, None, rccl=_FakeRcclPlane(0, q, log))
    t1 = P2PTransport("stage_1", ranks, None, rccl=_FakeRcclPlane(1, q, log))
    tc = P2PTransport("coordinator", ranks, None, rccl=_FakeRcclPlane(0, q, log))
    g = torch.Generator().manual_seed(0)
    for step in range(2):
        act = torch.randn(4, 8, 5, 6, generator=g).to(memory_format=torch.channels_last)
        o0 = _Outbox("stage_0")
        t0.send(o0, "stage_1", C.FORWARD_JOB, 3, act)
        got = t1.recv(o0.sent[-1], "cpu")
        assert torch.equal(got, act) and got.shape == act.shape
        grad = torch.randn(4, 8, 5, 6, generator=g)
        o1 = _Outbox("stage_1")
        t1.send(o1, "stage_0", C.BACKWARD_JOB, 3, grad)
        assert torch.equal(t0.recv(o1.sent[-1], "cpu"), grad)
        logits = torch.randn(4, 10, 1, 1, generator=g)
        t1.send(o1, "coordinator", C.FORWARD_JOB, 3, logits)
        assert torch.equal(tc.recv(o1.sent[-1], "cpu"), logits)
        dlog = torch.randn(4, 10, 1, 1, generator=g)
        oc = _Outbox("coordinator")
        tc.send(oc, "stage_1", C.BACKWARD_JOB, 3, dlog)
        assert torch.equal(t1.recv(oc.sent[-1], "cpu"), dlog)
    keys = [(e[0], e[1]) for e in log]
    assert keys[:8] == [("send", "fwd"), ("recv", "fwd"), ("send", "bwd"), ("recv", "bwd"),
                        ("send", "cfwd"), ("recv", "cfwd"), ("send", "cbwd"), ("recv", "cbwd")]
    assert log[0][4] == (4, 5, 6, 8) and log[0][5]  # NHWC physical buffer, contiguous
    assert t1.slot_allocs == 2 and t0.slot_allocs == 1 and tc.slot_allocs == 1  # step 2 reused the slots
    # rank-local peer (coordinator and stage_0 share rank 0): no RCCL call
    n = len(log)
    oc = _Outbox("coordinator")
    tc.send(oc, "stage_0", C.FORWARD_JOB, 4, torch.ones(2, 3, 1, 1))
    assert len(log) == n
