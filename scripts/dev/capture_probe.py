"""What another host thread's synchronous HIP calls do while this thread captures a HIP graph
(the async co-located server rank: the worker thread captures its step graphs while the server's
comm thread runs point-to-point). Per capture mode (torch.cuda.graph capture_error_mode) and per
call, one JSON line: the call's return code, how long it blocked, and whether the capture and a
replay still succeeded.

  python scripts/dev/capture_probe.py
"""
import ctypes
import json
import threading
import time

import torch

hip = ctypes.CDLL("libamdhip64.so")
HOLD = 2.0  # seconds the capture stays open


def probe(mode: str, call: str):
    dev = torch.device("cuda")
    x = torch.zeros(1 << 20, device=dev)
    a = torch.ones(1 << 20, device=dev)
    b = torch.empty(1 << 20, device=dev)
    side = torch.cuda.Stream()
    ev = torch.cuda.Event()
    torch.cuda.synchronize()
    res = {}
    started = threading.Event()

    def other():
        started.wait()
        time.sleep(0.3)  # inside the capture window
        t0 = time.perf_counter()
        if call == "hipMemcpy_d2d":
            rc = hip.hipMemcpy(ctypes.c_void_p(b.data_ptr()), ctypes.c_void_p(a.data_ptr()), ctypes.c_size_t(4 << 20), 3)
        elif call == "hipDeviceSynchronize":
            rc = hip.hipDeviceSynchronize()
        elif call == "side_stream_kernel+sync":
            with torch.cuda.stream(side):
                b.copy_(a)
            rc = hip.hipStreamSynchronize(ctypes.c_void_p(side.cuda_stream))
        elif call == "hipEventQuery":
            rc = hip.hipEventQuery(ctypes.c_void_p(ev.cuda_event)) if ev.cuda_event else -1
        elif call == "hipMemcpyAsync_nonblocking+sync":
            st = ctypes.c_void_p()
            hip.hipStreamCreateWithFlags(ctypes.byref(st), 1)  # hipStreamNonBlocking
            rc = hip.hipMemcpyAsync(ctypes.c_void_p(b.data_ptr()), ctypes.c_void_p(a.data_ptr()),
                                    ctypes.c_size_t(4 << 20), 3, st)
            rc = rc or hip.hipStreamSynchronize(st)
            hip.hipStreamDestroy(st)
        elif call in ("hipMalloc+hipFree", "relaxed:hipMalloc+hipFree", "relaxed:hipMemcpy_d2d"):
            if call.startswith("relaxed:"):
                m = ctypes.c_int(2)  # hipStreamCaptureModeRelaxed
                hip.hipThreadExchangeStreamCaptureMode(ctypes.byref(m))
            if call.endswith("hipMemcpy_d2d"):
                rc = hip.hipMemcpy(ctypes.c_void_p(b.data_ptr()), ctypes.c_void_p(a.data_ptr()),
                                   ctypes.c_size_t(4 << 20), 3)
            else:
                p = ctypes.c_void_p()
                rc = hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(1 << 20))
                rc = rc or hip.hipFree(p)
        res["rc"] = int(rc)
        res["blocked_s"] = round(time.perf_counter() - t0, 3)

    th = threading.Thread(target=other)
    th.start()
    ev.record()
    g = torch.cuda.CUDAGraph()
    ok = True
    err = ""
    try:
        with torch.cuda.graph(g, capture_error_mode=mode):
            x.add_(1.0)
            started.set()
            time.sleep(HOLD)
            x.add_(1.0)
    except Exception as e:  # noqa: BLE001
        ok, err = False, f"{type(e).__name__}: {e}"[:200]
    th.join()
    replay = None
    if ok:
        try:
            g.replay()
            torch.cuda.synchronize()
            replay = float(x[0].item())
        except Exception as e:  # noqa: BLE001
            replay = f"{type(e).__name__}: {e}"[:200]
    try:
        torch.cuda.synchronize()
        hip.hipGetLastError()
    except Exception:  # noqa: BLE001
        pass
    print(json.dumps({"mode": mode, "other_thread_call": call, **res, "capture_ok": ok, "capture_error": err,
                      "replay_x": replay}), flush=True)


CALLS = ("side_stream_kernel+sync", "hipEventQuery", "hipMemcpyAsync_nonblocking+sync", "hipMalloc+hipFree",
         "relaxed:hipMalloc+hipFree", "hipMemcpy_d2d", "relaxed:hipMemcpy_d2d", "hipDeviceSynchronize")

if __name__ == "__main__":
    import sys

    # one (mode, call) per process: an invalidated capture leaves a sticky error behind
    probe(sys.argv[1], CALLS[int(sys.argv[2])])
