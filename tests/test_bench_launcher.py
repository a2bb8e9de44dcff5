"""bench.py --gpus N starts N rank processes itself when no launcher set WORLD_SIZE (the
driver's scaling runs), refuses a world that disagrees with --gpus, and a launched run reports
n_gpus from the process group.  CPU only: the rank processes join a gloo group."""
import json
import os
import subprocess
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_launch_plan_two_ranks():
    env = {"PATH": "/usr/bin", "HSA_ENABLE_IPC_MODE_LEGACY": "0"}
    plan = bench.launch_plan(["--gpus", "2", "--steps", "3"], env, 29511)
    assert len(plan) == 2
    for r, (cmd, e) in enumerate(plan):
        assert cmd[0] == sys.executable and cmd[-4:] == ["--gpus", "2", "--steps", "3"]
        assert cmd[-5].endswith("bench.py")
        assert (e["WORLD_SIZE"], e["RANK"], e["LOCAL_RANK"]) == ("2", str(r), str(r))
        assert (e["MASTER_ADDR"], e["MASTER_PORT"]) == ("127.0.0.1", "29511")
        assert e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0" and e["PATH"] == "/usr/bin"


def test_no_plan_under_a_launcher_or_for_one_gpu():
    assert bench.launch_plan(["--gpus", "8"], {"WORLD_SIZE": "8"}, 1) == []
    assert bench.launch_plan(["--gpus", "1"], {}, 1) == []
    assert bench.launch_plan([], {}, 1) == []


def test_world_must_match_gpus():
    assert bench.world_of(2, {"WORLD_SIZE": "2", "RANK": "1", "LOCAL_RANK": "1"}) == (2, 1, 1)
    assert bench.world_of(1, {}) == (1, 0, 0)
    with pytest.raises(SystemExit):
        bench.world_of(2, {"WORLD_SIZE": "3", "RANK": "0"})
    with pytest.raises(SystemExit):
        bench.world_of(4, {})  # a rank without a launcher's world cannot claim 4 GPUs


@pytest.mark.parametrize("n", [2, 3])
def test_launched_run_reports_the_world(n):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", str(n), "--workload",
                        "launchcheck"], env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1  # rank 0 only
    assert lines[0]["n_gpus"] == n and lines[0]["rank_sum"] == n * (n - 1) // 2
    assert lines[0]["parallelism"] == f"beta-column shards x{n}"


def test_mismatched_world_is_refused():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--workload",
                        "launchcheck"], env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode != 0 and "mismatched world" in p.stderr
