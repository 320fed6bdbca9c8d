"""Control-plane object codec (parallel/objwire.py): tagged JSON, never pickle — round trips of the
values the transports exchange, refusal of anything else, and the gloo all_gather / broadcast over
two processes."""
import os
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from psx.parallel import objwire


@pytest.mark.parametrize("obj", [None, 3, -2.5, "w-r1", True, b"\x00\xffuid" * 16, {0: b"a", 3: b"b"},
                                 {"members": [0, 2, 3], "epoch": 4, "tag": "abc"}, (1, "x", None), [1.0, [2, (3,)]],
                                 {"__b": 1, "k": 2}])
def test_roundtrip(obj):
    assert objwire.loads(objwire.dumps(obj)) == obj


def test_refuses_objects():
    class Evil:
        def __reduce__(self):  # what a pickle payload would run
            return (os.system, ("true",))

    for bad in (Evil(), {1, 2}, object()):
        with pytest.raises(TypeError):
            objwire.dumps(bad)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        g = objwire.all_gather({rank: b"id%d" % rank, "n": "x" * (rank * 50)}, dist.group.WORLD, world)
        b = objwire.broadcast({0: b"uid", 1: b"uid1"} if rank == 0 else None, dist.group.WORLD, 0, rank)
        q.put((rank, g, b))
    finally:
        dist.destroy_process_group()


def test_gloo_all_gather_broadcast():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = dict((r, (g, b)) for r, g, b in (q.get(timeout=60) for _ in range(world)))
    for p in ps:
        p.join(30)
        assert p.exitcode == 0
    for r in range(world):
        g, b = out[r]
        assert g == [{0: b"id0", "n": ""}, {1: b"id1", "n": "x" * 50}]
        assert b == {0: b"uid", 1: b"uid1"}
