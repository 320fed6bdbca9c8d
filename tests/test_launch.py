"""scripts/launch.py: command construction and an end-to-end CPU (gloo) job with a log file
that scripts/parse_logs.py can consume."""
import os
import subprocess
import sys

from .test_ps_cpu import ROOT, TINY

sys.path.insert(0, os.path.join(ROOT, "scripts"))
import launch  # noqa: E402


def test_build_command():
    c1 = launch.build_command(1, ["--mode", "sync"])
    assert c1[1].endswith("psx_train.py") and "torch.distributed.run" not in c1
    c8 = launch.build_command(8, ["--mode", "async"], port=12345)
    assert "--nproc-per-node=8" in c8 and "127.0.0.1" in c8 and c8[-2:] == ["--mode", "async"]
    cb = launch.build_command(2, ["--gpus", "2"], bench=True, port=1)
    assert cb[cb.index("--master-port") + 2].endswith("bench.py")


def test_launch_cpu_job_and_parse(tmp_path):
    log = tmp_path / "job.log"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "launch.py"), "--nproc", "2", "--cpu",
                        "--log", str(log), "--", "--mode", "sync"] + TINY, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    from psx.utils.results import parse_experiment

    res = parse_experiment([log], "sync_2workers", verbose=False)
    assert res["server_metrics"]["total_workers"] == 2
    assert res["worker_metrics_aggregated"]["num_workers"] == 2
