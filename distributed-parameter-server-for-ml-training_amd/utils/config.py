"""Configuration: CLI flags + environment defaults + optional JSON file.

Keeps every flag and environment variable of the reference with the same defaults
(reference: src/parameter_server/server.py:405-433 and src/workers/worker.py:455-482):

  server  --mode {sync,async}  env SERVER_MODE             default sync
          --workers N (1..32)  env TOTAL_WORKERS_EXPECTED  default 4
          --lr 0.1, --port (env SERVER_PORT, 8000), --staleness-bound 5 (now actually wired)
  worker  --server (env PARAMETER_SERVER_ADDRESS, localhost:8000), --worker-name,
          --epochs 3, --batch-size 128, --lr 0.1, --sync-steps 1

and adds the MI355X-native knobs: --gpus/--nproc, --codec, --topk-ratio,
--dtype, --momentum/--weight-decay (server optimizer, default 0 = reference parity), --model,
--synthetic, --ckpt-every/--resume, --sync-semantics {barrier,reference}, --topology.
Precedence: explicit CLI flag > JSON config file (--config) > environment > default.
"""
from __future__ import annotations

import argparse
import dataclasses
import json
import os
from dataclasses import dataclass, field


def _env(name, default, cast=str):
    v = os.environ.get(name)
    return cast(v) if v not in (None, "") else default


@dataclass
class PSConfig:
    # --- reference server flags
    mode: str = "sync"
    workers: int = 4
    lr: float = 0.1
    port: int = 8000
    staleness_bound: int = 5
    # --- reference worker flags
    server: str = "localhost:8000"
    worker_name: str = "worker-node"
    epochs: int = 3
    batch_size: int = 128
    sync_steps: int = 1
    # --- MI355X-native extensions
    accumulate: bool = False       # --sync-steps K: push the mean gradient of the K batches of a window
    #                                instead of the reference's first batch only (K-1 discarded)
    model: str = "resnet18"
    num_classes: int | None = None
    gpus: int = 1                  # processes / GPUs on this node (1 = server+worker co-located)
    topology: str = "colocated"    # colocated: rank 0 = PS + worker 0; dedicated: rank 0 = PS only;
    #                                sharded: every rank = worker + 1/world of the PS (parallel/sharded.py)
    codec: str = "fp16"            # none (fp32 wire) | fp16 (reference) | topk
    topk_ratio: float = 0.01
    # compute dtype of the HIP engine: fp32 = the reference's training precision (worker.py:333-348;
    # exact-f32 MFMA), bf16 = the fast path (bf16 operands, fp32 accumulation and master weights)
    dtype: str = "fp32"
    momentum: float = 0.0          # server optimizer (0 = reference plain SGD, server.py:133)
    weight_decay: float = 0.0
    sync_semantics: str = "barrier"  # barrier (wait-for-N) | reference (count-triggered)
    # The reference server never updates BN running statistics and every fetch overwrites the
    # workers' copies (server.py:96,131-133 + worker.py:252), so evaluation runs on near-initial
    # statistics. bn_sync=True makes workers push their running stats with each gradient push;
    # the server averages them (sync) or blends them 1/W (async). Default off = reference parity.
    bn_sync: bool = False
    deterministic: bool | None = None  # exact fixed-point BN reductions, bit-reproducible steps; None:
    # PSX_DETERMINISTIC (default 1 = on; engine)
    # fetch payload: "bf16conv" = conv weights as bf16 (exactly the bits the bf16 engine consumes)
    # + fp32 for everything else (half the bytes); "fp32" = the reference's full fp32 state;
    # "auto" = fp32 for --dtype fp32, bf16conv for --dtype bf16.
    fetch_codec: str = "auto"
    # sync rounds stream gradient buckets during the backward pass (parallel/overlap.py). None =
    # auto: on with >= 2 ranks (the gather / apply / broadcast of the first buckets hides under
    # the rest of the backward), off at N=1, where there is no transfer to hide and the
    # per-bucket graphs cost ~0.2 ms/step (profiles/README.md). resolve_overlap() decides.
    overlap: object = None
    bucket_mb: float = 4.0         # bucket target size in MiB of fp16 wire gradient
    synthetic: bool = True
    synthetic_kind: str = "proto"  # proto: prototype + noise (learnable); hard: low contrast + 20% label noise
    data_dir: str = ""
    train_samples: int = 50000
    test_samples: int = 10000
    eval_every: int = 1            # epochs between evaluations (0 = never)
    eval_workers: str = "all"      # all: every worker evaluates (reference worker.py:393-394); first: worker 0 only
    max_steps: int = 0             # stop after this many local steps (0 = full epochs)
    ckpt_every: int = 0
    ckpt_dir: str = "checkpoints"
    resume: str = ""
    seed: int = 0
    heartbeat_timeout: float = 60.0
    log_dir: str = ""
    use_graph: bool = True
    # "kill_worker:2@5" (worker 2 raises at its step 5) | "hang_worker:2@5[:secs]" (stalls, forever or secs)
    # | "crash_in_push:2@5" (async: worker 2's process dies inside its step-5 push, after the PUSH request)
    fault_inject: str = ""
    transfer_timeout: float = 300.0  # async native loop: drop a worker whose transfer is in flight longer (0: off)
    stall_timeout: float = 0.0       # async native loop: drop a worker silent (no request) that long (0: off)
    round_timeout: float = 300.0   # sync liveness guard: abort + exit 3 when no round completes (0: off)
    # sync, dedicated topology: what a lost worker does to the job. shrink: the survivors rebuild
    # the communicator in-process and go on (parallel/elastic.py); restart: abort, exit 3, the
    # launcher restarts the group from the last checkpoint
    on_worker_loss: str = "shrink"
    recovery_grace: float = 0.0    # s the server waits for survivors to check in (0: --round-timeout)
    verbose: int = 1
    extra: dict = field(default_factory=dict)

    def validate(self):
        if self.mode not in ("sync", "async"):
            raise ValueError(f"--mode must be sync or async, got {self.mode!r}")
        if not (1 <= self.workers <= 32):  # reference server.py:424-426
            raise ValueError("Number of workers must be between 1 and 32")
        if self.eval_workers not in ("all", "first"):
            raise ValueError("--eval-workers must be all or first")
        if self.codec not in ("none", "fp16", "topk"):
            raise ValueError(f"--codec must be none, fp16 or topk, got {self.codec!r}")
        if self.topology not in ("colocated", "dedicated", "sharded"):
            raise ValueError(f"--topology must be colocated, dedicated or sharded, got {self.topology!r}")
        if self.topology == "sharded":  # parallel/sharded.py scope
            if self.mode != "sync" or self.codec not in ("fp16", "none") or self.bn_sync or self.ckpt_every \
                    or self.resume or max(1, self.sync_steps) != 1 or self.overlap is True:
                raise ValueError("--topology sharded: sync mode, dense fp16/fp32 gradients, one push per batch, "
                                 "no --bn-sync / --overlap / checkpoints")
        if self.sync_semantics not in ("barrier", "reference"):
            raise ValueError("--sync-semantics must be barrier or reference")
        if self.staleness_bound < 0:
            raise ValueError("--staleness-bound must be >= 0")
        if self.on_worker_loss not in ("shrink", "restart"):
            raise ValueError("--on-worker-loss must be shrink or restart")
        if self.transfer_timeout < 0 or self.stall_timeout < 0:
            raise ValueError("--transfer-timeout / --stall-timeout must be >= 0")
        if self.dtype not in ("fp32", "bf16"):
            raise ValueError(f"--dtype must be fp32 or bf16, got {self.dtype!r}")
        if self.fetch_codec == "auto":
            self.fetch_codec = "fp32" if self.dtype == "fp32" else "bf16conv"
        if self.fetch_codec not in ("bf16conv", "fp32"):
            raise ValueError("--fetch-codec must be bf16conv or fp32")
        if self.dtype == "fp32" and self.fetch_codec != "fp32":
            raise ValueError("--fetch-codec bf16conv ships bf16 conv weights, which only the bf16 engine consumes: "
                             "add --dtype bf16 (the default since round 2 is --dtype fp32, the reference's "
                             "precision, whose fetch payload is the fp32 state)")
        if self.bucket_mb <= 0:
            raise ValueError("--bucket-mb must be > 0")
        if self.synthetic_kind not in ("proto", "hard"):
            raise ValueError("--synthetic-kind must be proto or hard")
        if not (0.0 < self.topk_ratio <= 1.0):
            raise ValueError("--topk-ratio must be in (0, 1]")
        if self.fault_inject.startswith("crash_in_push") and self.mode != "async":
            # only the async native channel can die between its PUSH request and the transfer
            raise ValueError("--fault-inject crash_in_push applies to --mode async (native event loop) only")
        return self

    def resolve_overlap(self, world: int) -> bool:
        """--overlap / --no-overlap, or auto: bucketed rounds when there are peers to exchange
        with and the round qualifies (sync, one push per batch, dense wire, rank-0 server)."""
        if self.overlap is None:
            self.overlap = (world > 1 and self.mode == "sync" and max(1, self.sync_steps) == 1
                            and self.codec != "topk" and self.topology != "sharded")
        return bool(self.overlap)

    def to_json(self) -> str:
        return json.dumps(dataclasses.asdict(self), sort_keys=True)


def add_arguments(ap: argparse.ArgumentParser) -> argparse.ArgumentParser:
    d = PSConfig()
    A = ap.add_argument
    A("--config", default="", help="JSON file with PSConfig fields")
    A("--mode", choices=["sync", "async"], default=None, help="Training mode (env SERVER_MODE)")
    A("--workers", type=int, default=None, help="Expected number of workers, 1-32 (env TOTAL_WORKERS_EXPECTED)")
    A("--lr", type=float, default=None, help="Learning rate (server SGD)")
    A("--port", type=int, default=None, help="Rendezvous port (env SERVER_PORT)")
    A("--staleness-bound", type=int, default=None, help="Maximum staleness accepted in async mode")
    A("--server", default=None, help="Server address host:port (env PARAMETER_SERVER_ADDRESS)")
    A("--worker-name", default=None, help="Worker name for identification")
    A("--epochs", type=int, default=None)
    A("--batch-size", type=int, default=None)
    A("--sync-steps", type=int, default=None, help="Local steps between push/fetch (reference semantics)")
    A("--accumulate", action="store_true", default=None,
      help="with --sync-steps K: push the mean gradient of all K batches of a window (reference: the first only)")
    A("--model", choices=["resnet18", "resnet50", "resnet_tiny"], default=None)
    A("--num-classes", type=int, default=None)
    A("--gpus", "--nproc", dest="gpus", type=int, default=None)
    A("--topology", choices=["colocated", "dedicated", "sharded"], default=None)
    A("--codec", choices=["none", "fp16", "topk"], default=None)
    A("--topk-ratio", type=float, default=None)
    A("--dtype", choices=["fp32", "bf16"], default=None,
      help="worker compute precision: fp32 (reference, default) or bf16 (fast path)")
    A("--momentum", type=float, default=None)
    A("--weight-decay", type=float, default=None)
    A("--sync-semantics", choices=["barrier", "reference"], default=None)
    A("--bn-sync", action="store_true", default=None, help="workers push BN running stats; server averages")
    A("--deterministic", dest="deterministic", action="store_true", default=None,
      help="exact fixed-point BN statistic reductions: bit-reproducible training steps (the default; "
           "+0-2%% step time, profiles/r5_deterministic_ab.jsonl)")
    A("--no-deterministic", dest="deterministic", action="store_false", default=None,
      help="float-atomic BN statistic reductions (order-dependent rounding)")
    A("--fetch-codec", choices=["auto", "bf16conv", "fp32"], default=None)
    A("--overlap", dest="overlap", action="store_true", default=None,
      help="sync mode: stream gradient buckets (reduce/apply/broadcast) during the backward pass")
    A("--no-overlap", dest="overlap", action="store_false", default=None)
    A("--bucket-mb", type=float, default=None, help="overlapped sync: gradient bucket size (MiB of fp16)")
    A("--synthetic", action="store_true", default=None)
    A("--synthetic-kind", choices=["proto", "hard"], default=None,
      help="synthetic data: proto (class prototype + noise) or hard (low contrast, 20%% label noise)")
    A("--data-dir", default=None, help="directory with cifar-100-binary/{train,test}.bin")
    A("--train-samples", type=int, default=None)
    A("--test-samples", type=int, default=None)
    A("--eval-every", type=int, default=None)
    A("--eval-workers", choices=["all", "first"], default=None,
      help="all: every worker evaluates the test set each epoch (reference); first: worker 0 only")
    A("--max-steps", type=int, default=None)
    A("--ckpt-every", type=int, default=None)
    A("--ckpt-dir", default=None)
    A("--resume", default=None)
    A("--seed", type=int, default=None)
    A("--heartbeat-timeout", type=float, default=None)
    A("--log-dir", default=None)
    A("--no-graph", dest="use_graph", action="store_false", default=None)
    A("--fault-inject", default=None,
      help="kill_worker:K@S, hang_worker:K@S[:secs] or crash_in_push:K@S (first attempt only)")
    A("--transfer-timeout", type=float, default=None,
      help="async server: seconds a gradient receive / snapshot send may stay in flight before the worker is "
           "dropped (its pair communicator aborted); 0 disables")
    A("--stall-timeout", type=float, default=None,
      help="async server: seconds a worker may send no request before it is dropped (catches a hung training "
           "loop whose heartbeat thread still runs); 0 disables")
    A("--round-timeout", type=float, default=None,
      help="sync rounds: seconds without a completed round before the communicator is aborted and the rank "
           "exits (status 3) for a launcher restart from the last checkpoint; 0 disables")
    A("--on-worker-loss", choices=["shrink", "restart"], default=None,
      help="sync, dedicated topology: shrink (default) = the surviving ranks rebuild the communicator and "
           "continue without the lost worker; restart = exit 3 for a launcher restart from the last checkpoint")
    A("--recovery-grace", type=float, default=None,
      help="shrink: seconds the server waits for the surviving ranks to check in (default: --round-timeout)")
    A("--verbose", type=int, default=None)
    return ap


def from_args(ns: argparse.Namespace) -> PSConfig:
    cfg = PSConfig()
    # environment defaults (reference env vars)
    cfg.mode = _env("SERVER_MODE", cfg.mode)
    cfg.workers = _env("TOTAL_WORKERS_EXPECTED", cfg.workers, int)
    cfg.port = _env("SERVER_PORT", cfg.port, int)
    cfg.server = _env("PARAMETER_SERVER_ADDRESS", cfg.server)
    # JSON config file
    if getattr(ns, "config", ""):
        with open(ns.config) as f:
            data = json.load(f)
        for k, v in data.items():
            if not hasattr(cfg, k):
                raise ValueError(f"unknown config key {k!r} in {ns.config}")
            setattr(cfg, k, v)
    # explicit CLI flags
    for f in dataclasses.fields(PSConfig):
        v = getattr(ns, f.name, None)
        if v is not None:
            setattr(cfg, f.name, v)
    return cfg.validate()


def parse(argv=None, description="psx parameter server") -> PSConfig:
    ap = add_arguments(argparse.ArgumentParser(description=description))
    return from_args(ap.parse_args(argv))
