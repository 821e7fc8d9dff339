"""MI355X-native map-reduce transcript summarizer."""

import os as _os
import sys as _sys

# Cross-process device memory (RCCL, the custom all-reduce's IPC buffers, the TP KV hand-off) goes
# through dmabuf IPC, the only mode the host driver supports.  HSA reads this when HIP initialises
# (lazily, at the first GPU call): the entry points (cli.py, bench.py) set it before importing torch;
# here it is only a default for embedding programs, and IPC_MODE_TOO_LATE records when it arrives
# after HIP was already initialised with another mode (parallel/custom_ar.py then names the cause
# instead of failing with an opaque hipIpcGetMemHandle error).
IPC_MODE_TOO_LATE = False
if _os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY") != "0":
    _torch = _sys.modules.get("torch")
    if _torch is not None and getattr(_torch, "cuda", None) is not None and _torch.cuda.is_initialized():
        IPC_MODE_TOO_LATE = True
    _os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
