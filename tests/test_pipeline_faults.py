"""Pipeline failure detection, fault injection and recovery (parallel/pipeline/faults.py,
Coordinator.enable_recovery). The reference has join timeouts only."""
import time

import pytest
import torch

from dcnn_amd.models import zoo
from dcnn_amd.nn.optimizers import SGD, Adam
from dcnn_amd.parallel.pipeline import FlopPartitioner, InProcessCoordinator
from dcnn_amd.parallel.pipeline.coordinator import PipelineError, StageFailure
from dcnn_amd.parallel.pipeline.faults import FaultInjector, FaultSpec, env_faults
from dcnn_amd.parallel.pipeline import messages as M

C = M.CommandType


def _coord(faults=None, opt=None, **kw):
    model = zoo.create_model("mnist_cnn")
    model.set_seed(5)
    model.initialize()
    coord = InProcessCoordinator(model, opt if opt is not None else SGD(0.05), "softmax_crossentropy", num_stages=2, num_microbatches=2,
                                 partitioner=FlopPartitioner([2, 1, 28, 28]), **kw)
    coord.initialize()
    for i, f in (faults or {}).items():
        coord.stage_configs[i].fault = f
    coord.deploy_stages()
    coord.send_parameters(model)
    coord.start()
    return coord


def _batches(n):
    g = torch.Generator().manual_seed(11)
    return [(torch.randn(4, 1, 28, 28, generator=g), torch.randint(0, 10, (4,), generator=g)) for _ in range(n)]


def test_fault_spec_parsing(monkeypatch):
    s = FaultSpec.parse("FORWARD_JOB:3:crash")
    assert (s.command, s.after, s.action) == (int(C.FORWARD_JOB), 3, "crash")
    assert FaultSpec.parse({"command": "BACKWARD_JOB", "after": 2, "action": "hang", "seconds": 0.5}).seconds == 0.5
    with pytest.raises(ValueError):
        FaultSpec.parse("FORWARD_JOB:1:explode")
    monkeypatch.setenv("DCNN_FAULT", "stage_1:FORWARD_JOB:2:raise; stage_0:BACKWARD_JOB:1:drop")
    assert [f.action for f in env_faults("stage_1")] == ["raise"]
    assert [f.command for f in env_faults("stage_0")] == [int(C.BACKWARD_JOB)]
    inj = FaultInjector([FaultSpec.parse("FORWARD_JOB:2:drop")])
    assert [inj.check(C.FORWARD_JOB) for _ in range(3)] == [None, "drop", None]


def test_heartbeat_detects_crashed_stage_fast():
    """A crashed stage (no reply, no beats) is named within a few heartbeat intervals instead of
    after the 60 s job timeout."""
    coord = _coord({1: ["FORWARD_JOB:3:crash"]}, heartbeat_s=0.2, heartbeat_misses=3, timeout_s=60.0)
    try:
        (x, y), = _batches(1)
        coord.train_step(x, y, "sync")  # forwards 1, 2 on stage_1
        t0 = time.time()
        with pytest.raises(StageFailure) as e:
            coord.train_step(x, y, "sync")  # forward 3: stage_1 dies
        assert e.value.stage == "stage_1"
        assert time.time() - t0 < 10.0
        assert coord.stages[1].crashed and coord.stages[0].heartbeat.beats > 0
    finally:
        coord.stop()


def test_injected_raise_is_reported_as_job_failure():
    coord = _coord({0: ["BACKWARD_JOB:1:raise"]}, timeout_s=30.0)
    try:
        (x, y), = _batches(1)
        with pytest.raises(PipelineError, match="injected fault"):
            coord.train_step(x, y, "sync")
    finally:
        coord.stop()


def test_stall_is_caught_by_the_job_timeout_not_the_heartbeat():
    """A hung stage keeps beating (its heartbeat thread is alive): the job timeout fires."""
    coord = _coord({1: ["FORWARD_JOB:1:hang:2.5"]}, heartbeat_s=0.2, heartbeat_misses=3, timeout_s=1.0)
    try:
        (x, y), = _batches(1)
        with pytest.raises(PipelineError) as e:
            coord.train_step(x, y, "sync")
        assert not isinstance(e.value, StageFailure) and "timeout" in str(e.value)
    finally:
        coord.stop()


def test_recovery_retries_the_failed_step_from_the_snapshot():
    """Crash mid-step, recover (fresh stages + last snapshot), retry: the trajectory equals an
    uninterrupted run (plain SGD: no optimizer state is lost)."""
    data = _batches(3)
    ref = _coord()
    try:
        ref_losses = [ref.train_step(x, y, "sync") for x, y in data]
        ref_params = [p.clone() for p in ref.gather_model().parameters()]
    finally:
        ref.stop()
    coord = _coord({1: ["FORWARD_JOB:3:crash"]}, heartbeat_s=0.2, heartbeat_misses=3, timeout_s=60.0)
    coord.enable_recovery(snapshot_every=1, max_recoveries=2)
    try:
        losses = [coord.train_step(x, y, "sync") for x, y in data]
        assert coord.recoveries == 1
        assert losses == pytest.approx(ref_losses, rel=1e-6)
        for a, b in zip(coord.gather_model().parameters(), ref_params):
            torch.testing.assert_close(a, b, rtol=1e-6, atol=1e-7)
    finally:
        coord.stop()


def test_recovery_gives_up_after_max_recoveries():
    coord = _coord({0: ["FORWARD_JOB:1:raise"]}, timeout_s=30.0)
    coord.enable_recovery(snapshot_every=1, max_recoveries=0)
    try:
        (x, y), = _batches(1)
        with pytest.raises(PipelineError):
            coord.train_step(x, y, "sync")
        assert coord.recoveries == 0
    finally:
        coord.stop()


def test_recovery_replays_steps_since_an_older_snapshot():
    """snapshot_every=2 and a crash in step 4: the stages roll back to the step-2 snapshot, the
    coordinator re-trains step 3 from its logged micro-batches, then retries step 4 — the final
    parameters equal an uninterrupted run (no step silently lost)."""
    data = _batches(4)
    ref = _coord()
    try:
        ref_losses = [ref.train_step(x, y, "sync") for x, y in data]
        ref_params = [p.clone() for p in ref.gather_model().parameters()]
    finally:
        ref.stop()
    # 2 micro-batches per step: stage_1's 7th forward is the first micro-batch of step 4
    coord = _coord({1: ["FORWARD_JOB:7:crash"]}, heartbeat_s=0.2, heartbeat_misses=3, timeout_s=60.0)
    coord.enable_recovery(snapshot_every=2, max_recoveries=2)
    try:
        losses = [coord.train_step(x, y, "sync") for x, y in data]
        assert coord.recoveries == 1 and coord.steps == 4
        assert losses == pytest.approx(ref_losses, rel=1e-6)
        for a, b in zip(coord.gather_model().parameters(), ref_params):
            torch.testing.assert_close(a, b, rtol=1e-6, atol=1e-7)
    finally:
        coord.stop()


@pytest.mark.parametrize("make_opt", [lambda: Adam(1e-3), lambda: SGD(0.05, momentum=0.9)], ids=["adam", "sgd_momentum"])
def test_recovery_replay_restores_optimizer_state(make_opt):
    """Stateful optimizers: the snapshot carries Adam's moments + step counter (SGD's velocity),
    so replaying step 3 after a crash in step 4 neither double-counts an update on the surviving
    stage nor restarts the restarted stage's moments; a learning-rate change between logged steps
    is replayed too. Final parameters equal an uninterrupted run."""
    data = _batches(4)
    lrs = [None, None, 0.5, None]  # scale the LR before step 3 (a scheduler would)

    def run(coord):
        out = []
        for (x, y), f in zip(data, lrs):
            if f is not None:
                coord.set_learning_rate(coord.get_learning_rate() * f)
            out.append(coord.train_step(x, y, "sync"))
        return out

    ref = _coord(opt=make_opt())
    try:
        ref_losses = run(ref)
        ref_params = [p.clone() for p in ref.gather_model().parameters()]
    finally:
        ref.stop()
    xs_seen = []
    coord = _coord({1: ["FORWARD_JOB:7:crash"]}, opt=make_opt(), heartbeat_s=0.2, heartbeat_misses=3, timeout_s=60.0)
    coord.enable_recovery(snapshot_every=2, max_recoveries=2)
    try:
        losses = run(coord)
        assert coord.recoveries == 1 and coord.steps == 4
        assert losses == pytest.approx(ref_losses, rel=1e-5)
        for a, b in zip(coord.gather_model().parameters(), ref_params):
            torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)
    finally:
        coord.stop()


def test_replay_log_clones_micro_batches():
    coord = _coord()
    coord.enable_recovery(snapshot_every=3, max_recoveries=1)
    try:
        (x, y), = _batches(1)
        coord.train_step(x, y, "sync")
        logged = coord._replay_log[-1][1][0].clone()
        x.fill_(7.0)  # a loader refilling its buffer in place
        torch.testing.assert_close(coord._replay_log[-1][1][0], logged)
    finally:
        coord.stop()
