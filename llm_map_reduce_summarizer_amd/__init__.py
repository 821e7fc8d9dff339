"""MI355X-native map-reduce transcript summarizer."""

import os as _os

# Cross-process device memory (RCCL, the custom all-reduce's IPC buffers, the TP KV hand-off) goes
# through dmabuf IPC, the only mode the host driver supports.  HSA reads this when HIP initialises,
# which happens lazily at the first GPU call, so setting it at package import is early enough.
_os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
