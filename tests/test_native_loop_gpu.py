"""Native async server event loop (csrc/server/event_loop.cpp, parallel/native_loop.py) on one
MI355X, world size 1 in a subprocess: the co-located worker's path through a whole async run
(loop start, registration, staleness decisions, fused apply + bf16 image, fetch copies in stream
order, JobFinished, loop end), against the Python server loop.

Not covered on a one-GPU box: the remote-worker path (mailbox PUSH/FETCH + ncclRecv/ncclSend to a
peer rank). RCCL refuses two ranks on one device, and rank 0 cannot be its own peer either —
self send/recv from two threads fails with "invalid usage" (RCCL wants both in one group call) —
so that path stays opt-in (PSX_NATIVE_LOOP=1) until a multi-GPU run has exercised it.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(code, port, extra_env=None, timeout=240):
    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    env.update(extra_env or {})
    r = subprocess.run([sys.executable, "-c", code], env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                       timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT ")][-1]
    return json.loads(line[7:])


_ASYNC = r"""
import json, sys
sys.path.insert(0, {root!r})
import psx
from psx.parallel.runner import run_distributed
from psx.utils.config import PSConfig
cfg = PSConfig(model="resnet18", batch_size=64, epochs=1, train_samples=2048, eval_every=0, verbose=0, lr=0.1,
               max_steps=8, mode="async", dtype="bf16").validate()
res = run_distributed(cfg, log=lambda *a, **k: None)
s = res["server"]
print("RESULT " + json.dumps([s["final_param_checksum"], s["global_steps_completed"], s["async_updates"],
                             s["max_staleness_observed"]]))
"""


def test_native_loop_colocated_run_matches_python_loop():
    out = {}
    for flag, port in (("1", 29661), ("0", 29662)):
        out[flag] = _run(_ASYNC.format(root=ROOT), port, {"PSX_NATIVE_LOOP": flag})
    (a, ga, ua, sa), (b, gb, ub, sb) = out["1"], out["0"]
    assert ga == gb == 8 and ua == ub == 8 and sa == sb == 0, out
    assert abs(a - b) <= 2e-4 * max(abs(a), abs(b)), out
