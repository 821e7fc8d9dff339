"""Tensor-parallel paths against the textbook fp32 forward on ONE GPU: 2 and 4 ranks share the device
(gloo + the custom all-reduce's IPC buffers), so the sequence-parallel prefill, the TP-push decode, the
vocab-parallel sampler and the context-parallel prefill + KV hand-off run their real kernels and
collectives; rank 0 checks the gathered logits with the TP=1 parity bounds (tests/_tp_parity_worker.py).
VERDICT r3 item 6."""
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.gpu
@pytest.mark.timeout(900)
@pytest.mark.parametrize("world,model,wdtype", [(2, "llama3-8b", "bf16"), (4, "llama3-8b", "bf16"),
                                                (8, "llama3-8b", "bf16"), (8, "llama3-70b", "fp8")])
def test_tp_paths_match_fp32(world, model, wdtype):
    """TP = 2 / 4 / 8 with bf16 weights (Llama-3-8B dims, 2 layers) and TP = 8 with fp8 weights at the 70B
    aggregator's geometry (hidden 8192, 64 / 8 heads, ffn 28672: shard K 1024 / 3584, 2 layers) -- config 5's
    shard shapes -- each against the textbook fp32 forward with the TP=1 bounds (bf16 0.07; fp8 0.15, top-1
    0.9).  8 ranks share the GPU (VERDICT r4 next #1c)."""
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="2" if world > 4 else "4",
               MODEL=model, WDTYPE=wdtype)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", str(world), "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "tests", "_tp_parity_worker.py")]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=850)
    fails = [ln for ln in r.stdout.splitlines() if ln.startswith("RANKFAIL")]
    assert r.returncode == 0, "\n".join(fails)[:6000] + r.stdout[-2000:] + r.stderr[-2000:]
    assert r.stdout.count("tp parity ok") == world, r.stdout[-2000:]
    print([ln for ln in r.stdout.splitlines() if "parity:" in ln])
