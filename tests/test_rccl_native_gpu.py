"""Native RCCL transport (csrc/comm/rccl_comm.cpp + parallel/rccl.py) on one MI355X.

A one-GPU box can host a single RCCL rank (RCCL refuses two ranks on one device), so these run
world size 1 in a subprocess: communicator bootstrap through the gloo control group, the sync
collectives in stream order, the non-blocking overlap collectives, the gather path, and a whole
sync PS run over the native transport against the torch.distributed one. Multi-rank semantics
are the same channel code as the gloo CPU tests (tests/test_ps_cpu.py).
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_OPS = r"""
import json, sys
sys.path.insert(0, {root!r})
import torch
import psx
from psx.parallel.rccl import RcclTransport
t = RcclTransport(device=torch.device("cuda", 0))
res = {{}}
g = torch.randn(1 << 20, device="cuda").half()
ref = g.clone()
t.reduce_sum_to_server(g)
res["reduce_identity"] = bool(torch.equal(g, ref))
w = torch.randint(0, 255, (3 << 20,), dtype=torch.uint8, device="cuda")
wref = w.clone()
t.broadcast_from_server(w)
res["bcast_identity"] = bool(torch.equal(w, wref))
p = torch.arange(1000, dtype=torch.int32, device="cuda")
out = t.gather_to_server(p)
res["gather"] = len(out) == 1 and bool(torch.equal(out[0], p))
x = torch.randn(4096, device="cuda")
xr = x.clone()
wk = t.reduce_async(x)
wk.wait()
wb = t.broadcast_async(x)
ok = t.completed(wb) or (wb.wait() is True)
torch.cuda.synchronize()
res["async_ops"] = bool(torch.equal(x, xr))
res["async_error"] = t.comm.async_error()
t.close()
print("RESULT " + json.dumps(res))
"""


def _run(code, port, extra_env=None, timeout=240):
    # PSX_COMM_SELF=1: issue the one-rank collectives through RCCL (they are skipped as identities
    # otherwise), so this file exercises the RCCL call path
    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
               PSX_COMM_SELF="1")
    env.update(extra_env or {})
    r = subprocess.run([sys.executable, "-c", code], env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                       timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT ")][-1]
    return json.loads(line[7:])


def test_native_collectives_world1():
    res = _run(_OPS.format(root=ROOT), 29651)
    assert res == {"reduce_identity": True, "bcast_identity": True, "gather": True, "async_ops": True,
                   "async_error": 0}, res


_RUN = r"""
import json, sys
sys.path.insert(0, {root!r})
import psx
from psx.parallel.runner import run_distributed
from psx.utils.config import PSConfig
cfg = PSConfig(model="resnet18", batch_size=64, epochs=1, train_samples=2048, eval_every=0, verbose=0, lr=0.1,
               max_steps=6, mode="sync", codec={codec!r}).validate()
res = run_distributed(cfg, log=lambda *a, **k: None)
print("RESULT " + json.dumps([res["server"]["final_param_checksum"], res["server"]["global_steps_completed"]]))
"""


@pytest.mark.parametrize("codec", ["fp16", "topk"])
def test_sync_run_native_matches_torch_transport(codec):
    out = {}
    for kind, port in (("native", 29652), ("torch", 29653)):
        out[kind] = _run(_RUN.format(root=ROOT, codec=codec), port, {"PSX_TRANSPORT": kind})
    (a, sa), (b, sb) = out["native"], out["torch"]
    assert sa == sb == 6
    assert abs(a - b) <= 2e-4 * max(abs(a), abs(b)), out


def test_unloadable_rccl_falls_back_to_torch_transport():
    """Every rank agrees on the native communicator before ncclCommInitRank; when the library
    cannot be bound the job runs on torch.distributed instead of failing or hanging."""
    res = _run(_RUN.format(root=ROOT, codec="fp16"), 29654, {"PSX_RCCL_LIB": "/nonexistent/librccl.so"})
    assert res[1] == 6


_ROUND = r"""
import json, sys
sys.path.insert(0, {root!r})
import psx
from psx.parallel.runner import run_distributed
from psx.utils.config import PSConfig
cfg = PSConfig(model="resnet18", batch_size=64, epochs=1, train_samples=2048, eval_every=1, test_samples=256,
               verbose=0, lr=0.1, max_steps=6, mode="sync", use_graph={graph!r}, dtype="bf16").validate()
import psx.parallel.runner as R
made = []
_mk = R.make_sync_channel
def spy(*a, **k):
    c = _mk(*a, **k)
    made.append(type(c).__name__)
    return c
R.make_sync_channel = spy
res = run_distributed(cfg, log=lambda *a, **k: None)
w = res["worker"]
print("RESULT " + json.dumps([res["server"]["final_param_checksum"], res["server"]["global_steps_completed"],
                             w["final_test_accuracy_percent"], ",".join(made)]))
"""


@pytest.mark.parametrize("graph", [True, False])
def test_graph_round_matches_serial_round(graph):
    """The round captured in the step graph (parallel/graph_round.py; eager hooks when graphs
    are off) against the serial round (PSX_GRAPH_ROUND=0): same master state, and the worker's
    evaluation after training runs on the broadcast state."""
    out = {}
    for flag, port in (("1", 29654), ("0", 29655)):
        out[flag] = _run(_ROUND.format(root=ROOT, graph=graph), port, {"PSX_GRAPH_ROUND": flag})
    assert "GraphRoundChannel" in out["1"][3] and "GraphRoundChannel" not in out["0"][3]
    (a, sa, acc_a, _), (b, sb, acc_b, _) = out["1"], out["0"]
    assert sa == sb == 6
    assert abs(a - b) <= 2e-4 * max(abs(a), abs(b)), out
    assert acc_a >= 0.0 and acc_b >= 0.0


_SHARD = r"""
import json, sys
sys.path.insert(0, {root!r})
import psx
from psx.parallel.runner import run_distributed
from psx.utils.config import PSConfig
cfg = PSConfig(model="resnet18", batch_size=64, epochs=1, train_samples=2048, eval_every=0, verbose=0, lr=0.1,
               max_steps=6, mode="sync", topology={topo!r}).validate()
res = run_distributed(cfg, log=lambda *a, **k: None)
print("RESULT " + json.dumps([res["server"]["final_param_checksum"], res["server"]["global_steps_completed"]]))
"""


def test_sharded_server_world1_matches_rank0_server():
    """--topology sharded on the native communicator (reduce-scatter / all-gather, range apply
    writing the bf16 image, the HIP engine reading the sharded wire in place with the source-
    indexed fp32 scatter) against the default rank-0 PS; world size 1."""
    out = {}
    for topo, port in (("sharded", 29655), ("colocated", 29656)):
        out[topo] = _run(_SHARD.format(root=ROOT, topo=topo), port)
    (a, sa), (b, sb) = out["sharded"], out["colocated"]
    assert sa == sb == 6
    assert abs(a - b) <= 2e-4 * max(abs(a), abs(b)), out


_P2P = r"""
import json, sys, threading, time
sys.path.insert(0, {root!r})
import torch
import psx
from psx.ops._lib import comm as lib
from psx.parallel.rccl import NativeComm, RcclError, RcclTransport, _check
t = RcclTransport(device=torch.device("cuda", 0))
res = {{}}
c = t.comm
# 1. grouped self ncclSend + ncclRecv (the gather's grouped receive pattern, one peer = self)
src = torch.randn(1 << 18, device="cuda")
dst = torch.zeros_like(src)
_check(lib().psx_comm_group_start(), "ncclGroupStart")
c.send(src, 0)
c.recv(dst, 0)
_check(lib().psx_comm_group_end(), "ncclGroupEnd")
torch.cuda.synchronize()
res["self_sendrecv"] = bool(torch.equal(src, dst))
# 2. a self-receive with no matching send, then ncclCommAbort from a watchdog thread while the
# group may still be pending (RCCL either rejects the unmatched group at ncclGroupEnd or leaves a
# receive spinning; the abort must unblock it either way, within the budget)
lone = torch.zeros(4096, device="cuda")
old_h = c.h.value
err = None
aborted = threading.Event()
def watchdog():
    time.sleep(5.0)
    aborted.set()
    c.destroy(abort=True)
th = threading.Thread(target=watchdog, daemon=True)
th.start()
t0 = time.monotonic()
try:
    _check(lib().psx_comm_group_start(), "ncclGroupStart")
    try:
        c.recv(lone, 0)
    finally:
        _check(lib().psx_comm_group_end(), "ncclGroupEnd")
except RcclError as e:
    err = str(e)[:120]
if not aborted.is_set():  # rejected at enqueue (the ADVICE r4 #2 path): abort it ourselves
    c.destroy(abort=True)
torch.cuda.synchronize()
th.join(timeout=10)
res["unmatched_recv_returned_s"] = round(time.monotonic() - t0, 2)
res["unmatched_recv_error"] = err is not None
# 3. every later call on the aborted handle is refused (never a use of freed memory)
import ctypes
rc = lib().psx_comm_broadcast(ctypes.c_void_p(old_h), src.data_ptr(), 4, 2, 0, None)
res["dead_handle_refused"] = rc == -1002
# 4. the elastic path's re-initialisation: a fresh id, ncclCommInitRank, a working broadcast and a
# working grouped send/recv on the new communicator, process still healthy
uid = NativeComm.new_id()
c2 = NativeComm.from_id(uid, 1, 0, torch.device("cuda", 0))
b = torch.arange(1 << 16, dtype=torch.float32, device="cuda")
bref = b.clone()
c2.broadcast(b, 0)
d2 = torch.zeros_like(b)
_check(lib().psx_comm_group_start(), "ncclGroupStart")
c2.send(b, 0)
c2.recv(d2, 0)
_check(lib().psx_comm_group_end(), "ncclGroupEnd")
torch.cuda.synchronize()
res["reinit_broadcast"] = bool(torch.equal(b, bref))
res["reinit_sendrecv"] = bool(torch.equal(d2, bref))
res["reinit_async_error"] = c2.async_error()
res["new_handle_differs"] = c2.h.value != old_h
c2.destroy()
t.comm = c2  # already destroyed: close() must not touch the aborted first handle
t.close()
print("RESULT " + json.dumps(res))
"""


def test_native_p2p_abort_reinit_world1():
    """The RCCL entry points the 8-GPU run and the elastic recovery use, on real librccl at world
    1: grouped self ncclSend/ncclRecv, ncclCommAbort of a communicator with an unmatched receive
    (from a watchdog thread), refusal of calls on a dead handle, and NativeComm.from_id
    re-initialisation from a fresh id followed by a broadcast and a send/recv pair. (Pair
    communicators, open_pairs, need two ranks: covered by the fakecomm world-3 tests.)"""
    res = _run(_P2P.format(root=ROOT), 29657, timeout=120)
    assert res["self_sendrecv"], res
    assert res["unmatched_recv_returned_s"] < 30.0, res
    assert res["dead_handle_refused"] and res["new_handle_differs"], res
    assert res["reinit_broadcast"] and res["reinit_sendrecv"] and res["reinit_async_error"] == 0, res
