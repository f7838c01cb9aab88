"""bench.py's launch contract (no GPU needed): ``--gpus N`` without WORLD_SIZE starts N ranks through
torch.distributed.run before anything touches the GPU; under torchrun WORLD_SIZE must equal --gpus."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_launcher_cmd_is_the_drivers_torchrun_form():
    cmd = bench.launcher_cmd(["--gpus", "8", "--steps", "5"], 8, 29511)
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd and "--master-port=29511" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == [os.path.join(ROOT, "bench.py"), "--gpus", "8", "--steps", "5"][-4:]


def test_gpus_n_spawns_n_ranks(monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    seen = {}

    def fake_call(cmd, env=None):
        seen["cmd"], seen["env"] = cmd, env
        return 0

    monkeypatch.setattr(bench.subprocess, "call", fake_call)
    argv = ["--gpus", "4", "--steps", "3"]
    assert bench.maybe_launch(bench.parse(argv), argv) == 0
    assert "--nproc-per-node=4" in seen["cmd"] and seen["env"]["MASTER_ADDR"] == "127.0.0.1"


def test_single_gpu_runs_in_process(monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    assert bench.maybe_launch(bench.parse([]), []) is None


@pytest.mark.parametrize("world,gpus,expect", [("4", 4, None), ("2", 4, 2), ("8", 1, 2)])
def test_world_size_must_match_gpus(monkeypatch, world, gpus, expect):
    monkeypatch.setenv("WORLD_SIZE", world)
    argv = ["--gpus", str(gpus)]
    assert bench.maybe_launch(bench.parse(argv), argv) == expect


def test_workloads_parse():
    assert bench.parse([]).workload == "c2"
    a = bench.parse(["--workload", "c3", "--c3-steps", "4"])
    assert a.workload == "c3" and a.c3_steps == 4


def test_traffic_files_are_matched_by_workload(tmp_path, monkeypatch):
    """bench.load_traffic takes the newest committed PMC traffic file whose workload key matches (bf16 and the
    use_fp8 leg have their own keys), and returns None when no pass covers the workload."""
    import json
    import bench
    a, b = tmp_path / "new.json", tmp_path / "old.json"
    a.write_text(json.dumps({"workload": "C2 1024 (use_fp8, e4m3 MFMA Linears)", "hbm_bytes_per_forward": 2.0}))
    b.write_text(json.dumps({"workload": "C2 1024", "hbm_bytes_per_forward": 1.0}))
    monkeypatch.setattr(bench, "TRAFFIC_FILES", [str(tmp_path / "missing.json"), str(a), str(b)])
    assert bench.load_traffic("C2 1024")["hbm_bytes_per_forward"] == 1.0
    assert bench.load_traffic("C2 1024 (use_fp8, e4m3 MFMA Linears)")["file"] == "new.json"
    assert bench.load_traffic("C2 512") is None
