"""Developer tuning overrides: the engine's A/B switches and the kernel planners' tile sweeps in
ONE environment variable, ``PSX_TUNE="key=value[,key=value...]"`` (a bare key means "1"), read
by this module and by the native planners (csrc/kernels/common.hpp ``tune``). Production runs
set nothing; every default is the measured-best path. Keys (lower case):

  engine (models/engine.py): wino (0: direct kernels), wino_fuse, wino_wgf, wino_wgf_minhw,
    wino_maxhw, wino_wgrad, wino_wgrad_maxhw, wino_bnfold, wino_bwdfold, wino_wsplit,
    wgrad_stream (0/1/auto), wgrad_rbatch, tail_split, dgrad_fold_sc, stem_direct (0/1/auto),
    fuse_bnfin, bnfin_apply, fuse_bnbwd, mask_store, unpack_impl (tiles/tap), wino_cfg
  native planners: cv_bm, cv_bn, cv_wgm, cv_splits, cv_f32_128, cv_tapr, cv_tapr_halo,
    cv_tapr_bn, dgrad_s2_bm, dgrad_s2_bn, dgrad_s2_wgm, dgrad_s2_gather, wg_br, wg_bc, wg_ns,
    wg_splits, wg3, wg_share, wgf_br, wgf_bc, wgf_splits, wino_wbr, wino_wq, wino_wq_max,
    wino_wgf_q, wgrad_reduce_v1, wgrad_no_presum, fin_grid
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
