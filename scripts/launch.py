#!/usr/bin/env python3
"""Single-node job launcher: one process per MI355X, rank 0 = parameter server.

Replaces the reference's deployment layer (terraform/main.tf: 1 server + N worker ECS tasks
behind an NLB, env SERVER_MODE / TOTAL_WORKERS_EXPECTED / PARAMETER_SERVER_ADDRESS) with a
local rendezvous: it starts `torch.distributed.run` on 127.0.0.1 with one rank per GPU (RCCL
over xGMI), keeps HSA_ENABLE_IPC_MODE_LEGACY=0 for dmabuf IPC, and tees the job's output to
a log file that scripts/parse_logs.py turns into an experiment-result JSON.

  python scripts/launch.py --nproc 8 --log runs/sync_8.log -- --mode sync --epochs 3
  python scripts/launch.py --nproc 1 -- --mode async --workers 4     # loopback, 4 simulated workers
  python scripts/launch.py --nproc 4 --cpu -- --model resnet_tiny    # gloo rehearsal on CPU
  python scripts/launch.py --nproc 8 --max-restarts 2 -- --ckpt-every 100 --resume latest  # fault tolerant

The launcher itself never touches the GPU; the job runs as a child process and its exit code
is returned.
"""
import argparse
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def build_command(nproc: int, train_args, cpu=False, port=None, bench=False, max_restarts=0):
    script = os.path.join(ROOT, "bench.py" if bench else os.path.join("scripts", "psx_train.py"))
    extra = (["--cpu"] if cpu and not bench else []) + list(train_args)
    if nproc <= 1 and not bench:
        return [sys.executable, script] + extra
    port = port or free_port()
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
            f"--max-restarts={max_restarts}", "--master-addr", "127.0.0.1", "--master-port", str(port),
            script] + extra


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    rest = []
    if "--" in argv:
        i = argv.index("--")
        argv, rest = argv[:i], argv[i + 1:]
    ap = argparse.ArgumentParser(description="psx single-node launcher")
    ap.add_argument("--nproc", "--gpus", dest="nproc", type=int, default=1)
    ap.add_argument("--log", default="", help="tee the job output to this file")
    ap.add_argument("--cpu", action="store_true", help="gloo + CPU compute (rehearsal)")
    ap.add_argument("--bench", action="store_true", help="launch bench.py instead of the trainer")
    ap.add_argument("--max-restarts", type=int, default=0,
                    help="restart the whole job this many times after a rank fails; combine with trainer flags "
                         "--ckpt-every N --resume latest to continue from the last server checkpoint")
    ap.add_argument("--dry-run", action="store_true")
    a = ap.parse_args(argv)
    if a.bench:
        rest = ["--gpus", str(a.nproc)] + rest
    cmd = build_command(a.nproc, rest, cpu=a.cpu, bench=a.bench, max_restarts=a.max_restarts)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    env["PYTHONPATH"] = ROOT + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
    print("[launch]", " ".join(cmd), flush=True)
    if a.dry_run:
        return 0
    if not a.log:
        return subprocess.call(cmd, env=env)
    os.makedirs(os.path.dirname(os.path.abspath(a.log)), exist_ok=True)
    with open(a.log, "w") as f:
        p = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, bufsize=1)
        for line in p.stdout:
            sys.stdout.write(line)
            f.write(line)
        return p.wait()


if __name__ == "__main__":
    raise SystemExit(main())
