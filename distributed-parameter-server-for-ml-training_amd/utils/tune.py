"""Developer overrides in ONE environment variable, ``PSX_TUNE="key=value[,key=value...]"`` (a
bare key means "1"), read by this module and by the native planners (csrc/kernels/common.hpp
``tune``). Production runs set nothing; every default is the measured-best path. Round 6 cut the
set from ~50 keys to the 12 below, each exercised by a test (the A/B switches whose other side
was measured slower, and the tile-sweep overrides of the retired sweep scripts, are gone):

  engine (models/engine.py):
    wino=0            direct kernels instead of Winograd (tests/test_wino_gpu.py, test_fp32_gpu.py)
    wino_bnfold=0     BN + ReLU not folded into the next Winograd conv (tests/test_wino_gpu.py)
    wino_bwdfold=0    BN-backward applies not folded (tests/test_wino_fused_gpu.py)
    wgrad_stream=0|1  weight gradients on / off the side stream (default auto;
                      tests/test_deterministic_gpu.py)
    wgrad_rbatch=0    per-layer weight-gradient reductions (tests/test_wgrad_batch_gpu.py)
  conv tile plan (csrc/kernels/conv_v2.hip; tests/test_conv_v2_gpu.py, tests/test_fp32_gpu.py run
  every tile instantiation through them):
    cv_bm, cv_bn, cv_wgm, cv_splits, cv_tapr=0, cv_tapr_bn, cv_tapr_halo=1
"""
from __future__ import annotations

import os


def tune(key: str, default: str | None = None) -> str | None:
    """The value of ``key`` in PSX_TUNE (read now, so a test can change it in-process)."""
    for item in os.environ.get("PSX_TUNE", "").split(","):
        k, sep, v = item.strip().partition("=")
        if k == key:
            return v if sep else "1"
    return default


def tune_flag(key: str, default: bool) -> bool:
    v = tune(key)
    return default if v is None else v not in ("0", "", "false", "off")


def tune_int(key: str, default: int) -> int:
    v = tune(key)
    return default if v is None else int(v)


def with_tune(**kv) -> str:
    """PSX_TUNE string with ``kv`` merged over the current one (for tests / A-B scripts)."""
    cur = {}
    for item in os.environ.get("PSX_TUNE", "").split(","):
        k, sep, v = item.strip().partition("=")
        if k:
            cur[k] = v if sep else "1"
    cur.update({k: str(v) for k, v in kv.items()})
    return ",".join(f"{k}={v}" for k, v in cur.items())


def set_tune(**kv):
    """Set PSX_TUNE to exactly ``kv`` (None values dropped; no keys: unset) — sweeps and A/Bs."""
    items = [f"{k}={v}" for k, v in kv.items() if v is not None]
    if items:
        os.environ["PSX_TUNE"] = ",".join(items)
    else:
        os.environ.pop("PSX_TUNE", None)
