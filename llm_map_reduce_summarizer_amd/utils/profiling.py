"""Optional torch.profiler capture around a pipeline run.

The reference only logs wall-clock deltas (main.py:110,239; llm_executor.py:129,150;
result_aggregator.py:72,102).  Per-phase timers live in the report; this adds a kernel-level
trace: ``--profile DIR`` writes one Chrome trace per rank (``DIR/trace_rank{r}.json``, open in
Perfetto) with CPU ops and HIP kernels (ROCm activity = the ``CUDA`` activity in torch), plus a
``DIR/kernels_rank{r}.txt`` table of the top device kernels.  Graph-replayed decode steps appear
as one graph launch each; use ``--no-graphs`` or rocprofv3 for per-kernel decode timings.
"""

from __future__ import annotations

import contextlib
import os
from typing import Iterator, Optional


@contextlib.contextmanager
def maybe_profile(out_dir: Optional[str], rank: int = 0, top: int = 40) -> Iterator[None]:
    if not out_dir:
        yield
        return
    import torch
    from torch.profiler import ProfilerActivity, profile

    acts = [ProfilerActivity.CPU]
    if torch.cuda.is_available():
        acts.append(ProfilerActivity.CUDA)
    os.makedirs(out_dir, exist_ok=True)
    with profile(activities=acts, record_shapes=False) as prof:
        yield
    prof.export_chrome_trace(os.path.join(out_dir, "trace_rank%d.json" % rank))
    key = "self_cuda_time_total" if torch.cuda.is_available() else "self_cpu_time_total"
    with open(os.path.join(out_dir, "kernels_rank%d.txt" % rank), "w") as f:
        f.write(prof.key_averages().table(sort_by=key, row_limit=top))
