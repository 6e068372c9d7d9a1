"""bench.py's steps in flight (--in-flight): run_steps hands step i to lane i mod L, from one
host thread per lane or in order from the caller's thread, and re-raises a lane's error."""
import threading

import pytest

import bench


class FakeLane:
    def __init__(self, j, log, fail_at=None):
        self.j, self.log, self.fail_at, self.k = j, log, fail_at, 0

    def step(self):
        if self.fail_at is not None and self.k == self.fail_at:
            raise RuntimeError(f"lane {self.j} failed")
        self.log.append((self.j, threading.get_ident()))
        self.k += 1


@pytest.mark.parametrize("nl,k,threaded", [(1, 7, True), (2, 9, True), (3, 10, True), (2, 9, False), (3, 2, True)])
def test_run_steps_counts(nl, k, threaded):
    log = []
    lanes = [FakeLane(j, log) for j in range(nl)]
    bench.run_steps(lanes, k, threaded)
    per = [sum(1 for j, _ in log if j == q) for q in range(nl)]
    assert per == [len(range(q, k, nl)) for q in range(nl)]
    if not threaded or nl == 1:   # in order, on the caller's thread
        assert [j for j, _ in log] == [i % nl for i in range(k)]
        assert {t for _, t in log} == {threading.get_ident()}
    else:   # lane 0 on the caller's thread, every other lane on one thread of its own
        main = threading.get_ident()
        for q in range(nl):
            ts = {t for j, t in log if j == q}
            if ts:
                assert len(ts) == 1 and (main in ts) == (q == 0), (q, ts)


def test_run_steps_reraises():
    log = []
    lanes = [FakeLane(0, log), FakeLane(1, log, fail_at=2)]
    with pytest.raises(RuntimeError, match="lane 1 failed"):
        bench.run_steps(lanes, 10, True)
