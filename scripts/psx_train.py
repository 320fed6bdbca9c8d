#!/usr/bin/env python3
"""psx training entry point (one process per GPU; also the loopback single-process runner).

  # 1 GPU, server + 1 worker co-located (loopback)
  python scripts/psx_train.py --mode sync --workers 1
  # 8 GPUs on one node, RCCL over xGMI; rank 0 = parameter server (+ worker 0)
  torchrun --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 scripts/psx_train.py --mode async
  # the reference's split (rank 0 = server only, ranks 1..7 = workers)
  torchrun ... scripts/psx_train.py --mode sync --topology dedicated

Flags and environment variables of the reference server/worker CLIs are accepted
(see utils/config.py). ``--cpu`` hides all GPUs (gloo + torch CPU compute; used by the tests).
"""
import os
import sys

if "--cpu" in sys.argv:
    sys.argv.remove("--cpu")
    os.environ["CUDA_VISIBLE_DEVICES"] = ""
    os.environ["HIP_VISIBLE_DEVICES"] = ""

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import psx  # noqa: E402,F401
from psx.parallel.runner import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main())
