"""The communicator watchdog's deadline logic (parallel/comm.py CommWatchdog) with injected
events: a collective whose event never completes must end in a RuntimeError on the training
thread within the deadline, after ``on_timeout`` (ncclCommAbort for RcclComm) ran once."""
import time

import pytest

from distributed_training_amd.parallel.comm import CommWatchdog


class _Ev:
    def __init__(self, done=False):
        self.done = done

    def query(self):
        return self.done


def test_completed_collectives_never_fire():
    aborts = []
    wd = CommWatchdog("test", 0.2, lambda: aborts.append(1), poll_s=0.02)
    evs = [_Ev(True) for _ in range(50)]
    for i, e in enumerate(evs):
        wd.track(e, f"all_reduce #{i}")
    time.sleep(0.4)
    assert not aborts and wd.error is None and wd.pending() == 0
    wd.raise_if_error()
    wd.stop()


def test_stalled_collective_aborts_and_raises_within_deadline():
    aborts = []
    wd = CommWatchdog("test", 0.3, lambda: aborts.append(time.monotonic()), poll_s=0.02, exit_grace_s=30)
    t0 = time.monotonic()
    wd.track(_Ev(True), "done one")
    wd.track(_Ev(False), "bucket 3 all_reduce")  # a peer that never joins
    deadline = t0 + 5.0
    while not aborts and time.monotonic() < deadline:
        time.sleep(0.01)
    assert len(aborts) == 1, "watchdog did not abort"
    assert 0.3 <= aborts[0] - t0 < 2.0
    with pytest.raises(RuntimeError, match="bucket 3 all_reduce"):
        wd.raise_if_error()
    wd.stop()


def test_late_completion_within_deadline_is_fine():
    aborts = []
    wd = CommWatchdog("test", 0.5, lambda: aborts.append(1), poll_s=0.02)
    ev = _Ev(False)
    wd.track(ev, "slow but alive")
    time.sleep(0.2)
    ev.done = True
    time.sleep(0.6)
    assert not aborts and wd.error is None
    wd.stop()


def test_disabled_with_nonpositive_timeout():
    wd = CommWatchdog("test", 0.0, lambda: None)
    wd.track(_Ev(False), "x")
    assert wd.pending() == 0 and wd._thread is None
