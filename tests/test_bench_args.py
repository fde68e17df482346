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


def test_pmc_summary_matched_by_source_or_device_isa(monkeypatch, tmp_path):
    """bench.load_pmc uses a PMC summary only for the current kernel: the same source hash, or the same device ISA
    hash as profiles/latest_isa.json (which must itself be made from the current source)."""
    import json

    src = bench.kernel_source_sha256()
    p = tmp_path / "pmc.json"
    p.write_text(json.dumps({"source_sha256": src, "kernels": {"step_kernel": {"x": 1}}}))
    assert bench.load_pmc(p)[0] == {"step_kernel": {"x": 1}}
    monkeypatch.setattr(bench, "load_isa", lambda: ({"isa_sha256": "aa"}, "isa"))
    p.write_text(json.dumps({"source_sha256": "old", "isa_sha256": "aa", "kernels": {"step_kernel": {}}}))
    assert bench.load_pmc(p)[0] == {"step_kernel": {}}
    for isa in ("bb", None):
        p.write_text(json.dumps({"source_sha256": "old", "isa_sha256": isa, "kernels": {"step_kernel": {}}}))
        k, why = bench.load_pmc(p)
        assert k == {} and "stale" in why
    monkeypatch.setattr(bench, "load_isa", lambda: ({}, "latest_isa.json: stale (kernel source changed)"))
    p.write_text(json.dumps({"source_sha256": "old", "isa_sha256": "aa", "kernels": {"step_kernel": {}}}))
    assert bench.load_pmc(p)[0] == {}


def test_kernel_source_hash_covers_the_headers(monkeypatch, tmp_path):
    """The summaries' key changes with a header-only edit (csrc/*.h, include/*.h), not only with csrc/h12env.hip."""
    import shutil

    from h12env import build as B

    base = bench.kernel_source_sha256()
    shutil.copytree(ROOT / "h1v2-isaac_amd" / "csrc", tmp_path / "h1v2-isaac_amd" / "csrc")
    shutil.copytree(ROOT / "include", tmp_path / "include")
    monkeypatch.setattr(B, "CSRC", tmp_path / "h1v2-isaac_amd" / "csrc")
    monkeypatch.setattr(B, "REPO", tmp_path)
    assert B.source_sha256() == base
    for f in (tmp_path / "h1v2-isaac_amd" / "csrc" / "h12_math.h", tmp_path / "include" / "h12env.h"):
        old = f.read_bytes()
        f.write_bytes(old + b"\n// edit\n")
        assert B.source_sha256() != base, f.name
        f.write_bytes(old)
