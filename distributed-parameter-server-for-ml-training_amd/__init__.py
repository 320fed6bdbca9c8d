"""psx — an MI355X-native parameter-server training framework.

Capabilities of the reference (Jjjing2023/Distributed-Parameter-Server-for-ML-Training):
register / push gradients / fetch parameters / job-finished API, synchronous (wait-for-N)
and asynchronous (bounded staleness, staleness-weighted) server updates, fp16 gradient codec,
per-worker data sharding, METRICS_JSON observability, CLI/env configuration, and a
state_dict-keyed checkpoint layout — re-designed for AMD MI355X:

* transport: RCCL (torch.distributed backend "nccl") over xGMI inside one node; rank 0 holds
  the parameter server (fp32 master arena in HBM), every rank runs a data-parallel worker;
* compute: hand-written CDNA4 HIP kernels (MFMA implicit-GEMM convolution, fused BatchNorm /
  ReLU / residual, fused SGD + codec, top-k gradient compression) captured into HIP graphs;
* runtime: native C++ server core (barrier / staleness state machine), shared-memory control
  plane mailbox, CIFAR binary reader.

Sub-packages: ``models`` (reference torch models, parameter layout, HIP training engine),
``ops`` (ctypes bindings of the native libraries), ``parallel`` (transports, server, worker,
launcher), ``utils`` (config, metrics, checkpoint, data).
"""

__version__ = "0.1.0"

import os as _os

# HIP-graph replay on exactly two hardware queues (the engine's compute stream and its
# weight-gradient side stream; the HIP runtime reads this when it initialises, i.e. at the
# first device call, which comes after this import). The default spreads a captured step's
# nodes over the process's four queues, so independent nodes queue behind each other and
# every cross-queue edge costs a signal wait: same box, bf16 ResNet-18 step 1.85-1.87 -> 1.80
# ms, ResNet-50 fp32 unchanged (profiles/r4_numbers.jsonl, r4_call20/21). PSX_GRAPH_QUEUES=0
# keeps the runtime's default; any other value is used as the queue count.
_gq = _os.environ.get("PSX_GRAPH_QUEUES", "2")
if _gq != "0":
    _os.environ.setdefault("DEBUG_HIP_FORCE_GRAPH_QUEUES", _gq)

PACKAGE_DIR = _os.path.dirname(_os.path.abspath(__file__))
NATIVE_DIR = _os.path.join(PACKAGE_DIR, "_native")
