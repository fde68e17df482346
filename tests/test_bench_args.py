"""CPU: bench.py's argument checks: the compact rollout records rebuild flat / rsl history rows only,
so --rollout on is rejected for the other tasks and 'auto' leaves them off at N > 1; --dump-rollout only for windows
that hold one rollout's data."""
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402


def parse(monkeypatch, *argv):
    monkeypatch.setattr(sys, "argv", ["bench.py", *argv])
    return bench.parse()


@pytest.mark.parametrize("task", ["rough", "c5", "cat"])
def test_rollout_on_rejected_for_tasks_without_history_records(monkeypatch, task):
    with pytest.raises(SystemExit):
        parse(monkeypatch, "--task", task, "--rollout", "on")
    a = parse(monkeypatch, "--task", task)  # auto stays accepted (and off for this task at any N)
    assert a.rollout == "auto" and task not in bench.ROLLOUT_TASKS


@pytest.mark.parametrize("task", ["flat", "rsl"])
def test_rollout_on_accepted_for_flat_and_rsl(monkeypatch, task):
    assert parse(monkeypatch, "--task", task, "--rollout", "on").rollout == "on"


def test_dump_rollout_window_bound(monkeypatch):
    parse(monkeypatch, "--rollout", "on", "--steps", "48", "--dump-rollout", "x.npz")
    with pytest.raises(SystemExit):
        parse(monkeypatch, "--rollout", "on", "--steps", "49", "--dump-rollout", "x.npz")
    parse(monkeypatch, "--rollout", "on", "--steps", "24", "--rollout-decode", "--dump-rollout", "x.npz")
    with pytest.raises(SystemExit):
        parse(monkeypatch, "--rollout", "on", "--steps", "25", "--rollout-decode", "--dump-rollout", "x.npz")
