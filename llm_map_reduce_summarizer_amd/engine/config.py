"""Model presets for the on-node engine.

The reference never runs a model locally (its map/reduce calls go to hosted
APIs: ``llm_executor.py:250-409``); BASELINE.json names Llama-3-8B for the
map stage and Llama-3-70B (fp8, TP=8) for the aggregator.  Shapes are the
public Llama-3 configs; weights are random-init (seeded)
because no checkpoints are available offline.  ``tiny*`` presets keep the
real vocabulary and head_dim=128 (what the HIP attention kernels are built
for) so CPU tests and GPU smoke runs exercise the same code paths.
"""

from __future__ import annotations

from dataclasses import dataclass, replace
from typing import Optional, Tuple

# The engine's default chunked-prefill slice length (tokens; engine/engine.py LLMEngine ``prefill_chunk``).
# Defined here, next to the model presets, so the planner (parallel/plan.py) prices the slice length the
# engine actually runs without importing the engine; tests/test_plan.py fails if the two drift.
PREFILL_CHUNK = 8192


@dataclass(frozen=True)
class ModelConfig:
    name: str
    vocab_size: int = 128256
    hidden: int = 4096
    n_layers: int = 32
    n_heads: int = 32
    n_kv_heads: int = 8
    head_dim: int = 128
    ffn: int = 14336
    rope_theta: float = 500000.0
    rms_eps: float = 1e-5
    max_position: int = 40960
    init_std: float = 0.02
    # Llama-3.1 "llama3" RoPE frequency scaling: (factor, low_freq_factor, high_freq_factor,
    # original_max_position_embeddings); None = plain RoPE
    rope_scaling: Optional[Tuple[float, float, float, int]] = None

    @property
    def qkv_dim(self) -> int:
        return (self.n_heads + 2 * self.n_kv_heads) * self.head_dim

    def n_params(self) -> int:
        per_layer = (self.hidden * self.qkv_dim + self.n_heads * self.head_dim * self.hidden
                     + 3 * self.hidden * self.ffn + 2 * self.hidden)
        return self.n_layers * per_layer + 2 * self.vocab_size * self.hidden + self.hidden

    def kv_bytes_per_token(self, dtype_bytes: int = 2) -> int:
        return 2 * self.n_layers * self.n_kv_heads * self.head_dim * dtype_bytes


PRESETS = {
    "llama3-8b": ModelConfig("llama3-8b"),
    "llama3-70b": ModelConfig("llama3-70b", hidden=8192, n_layers=80, n_heads=64, n_kv_heads=8, ffn=28672),
    # Llama-3.1: same shapes, 128k positions with the "llama3" RoPE scaling -- the model for a single-pass
    # reduce over a whole day of summaries (--no-hierarchical on 24 h: ~100k-token prompt)
    "llama3.1-8b": ModelConfig("llama3.1-8b", max_position=131072, rope_scaling=(8.0, 1.0, 4.0, 8192)),
    "llama3.1-70b": ModelConfig("llama3.1-70b", hidden=8192, n_layers=80, n_heads=64, n_kv_heads=8, ffn=28672,
                                max_position=131072, rope_scaling=(8.0, 1.0, 4.0, 8192)),
    # test / smoke configs (real vocab, head_dim 128)
    "tiny": ModelConfig("tiny", hidden=256, n_layers=2, n_heads=2, n_kv_heads=1, ffn=512, max_position=8192),
    "tiny-gqa4": ModelConfig("tiny-gqa4", hidden=512, n_layers=2, n_heads=8, n_kv_heads=2, ffn=1024,
                             max_position=8192),
    # GQA 3:1 (Llama-3.2-3B's ratio, 24 / 8): the attention kernels' per-query-head fallback
    "tiny-gqa3": ModelConfig("tiny-gqa3", hidden=768, n_layers=2, n_heads=6, n_kv_heads=2, ffn=1024,
                             max_position=8192),
    # 8 KV heads (GQA 2:1) with heads / ffn / vocab divisible by 8: the TP=4 / TP=8 sharding paths of an
    # 8-GPU node (one or two KV heads per rank, 16032-row vocab shards, 8-way KV hand-off) on CPU ranks
    "tiny-kv8": ModelConfig("tiny-kv8", hidden=512, n_layers=2, n_heads=16, n_kv_heads=8, ffn=1024,
                            max_position=8192),
}


def get_model_config(name: str, **overrides) -> ModelConfig:
    key = name.lower()
    if key not in PRESETS:
        raise ValueError("unknown model %r (known: %s)" % (name, ", ".join(sorted(PRESETS))))
    cfg = PRESETS[key]
    return replace(cfg, **overrides) if overrides else cfg
