"""Host-side work lists and launch plans of the HIP ops (no GPU needed): the prefill-attention item list
covers every query row of every sequence exactly once at each GQA ratio, heaviest blocks first, and the
decode-attention split plan keeps its measured choices (ops/hip.py)."""
import pytest

from llm_map_reduce_summarizer_amd.ops import hip


@pytest.mark.parametrize("group", [1, 2, 4, 8, 3, 5, 16])
def test_prefill_items_cover_every_row_once(group):
    seqlens = [1, 63, 64, 65, 300, 4096]
    bm = hip.prefill_block_m(group)
    # packed GQA ratios: 256 / G positions per workgroup; others: per-query-head fallback, 256 positions
    assert bm == (256 // group if group in (1, 2, 4, 8) else 256)
    items = hip.prefill_items(seqlens, group).tolist()
    assert len(items) == sum(-(-n // bm) for n in seqlens)
    seen = {s: [0] * n for s, n in enumerate(seqlens)}
    for s, qb in items:
        assert qb % bm == 0 and 0 <= qb < seqlens[s]
        for r in range(qb, min(qb + bm, seqlens[s])):
            seen[s][r] += 1
    assert all(c == 1 for rows in seen.values() for c in rows)
    starts = [qb for _, qb in items]
    assert starts == sorted(starts, reverse=True)  # heaviest (latest) blocks first


def test_prefill_block_m_rejects_bad_ratios():
    for g in (0, 65):
        with pytest.raises(ValueError):
            hip.prefill_block_m(g)


def test_decode_groups():
    assert hip.decode_groups(32, 8) == 8 and hip.decode_groups(64, 8) == 8 and hip.decode_groups(16, 1) == 1
    assert hip.decode_groups(24, 8) == 24  # ratio 3: one group per query head
    with pytest.raises(ValueError):
        hip.decode_groups(24, 7)


def test_decode_attn_plan_measured_choices():
    # a TP shard's single kv head at B=20, 4k context: 12 fused splits (profiles/r3_plans_insitu_tp8_b39_b20.jsonl)
    assert hip.decode_attn_plan(20, 1, 4096) == (12, True)
    # the same batch over 8 kv heads (TP=1) keeps at most 8 fused splits
    s, fused = hip.decode_attn_plan(20, 8, 4096)
    assert fused is False or s <= 8
    # B=1 at TP=8 (one kv head, 4k): one workgroup per page, separate merge
    s, fused = hip.decode_attn_plan(1, 1, 4096)
    assert not fused and s == 64


def test_decode_attn_plan_class1_six_fused_splits():
    # the <= 12k context class (level-1 reduce at ~6k), per graph bucket: 6 fused splits, in situ
    # (profiles/r4_attn_plans_insitu_class1.jsonl): batch 5 (bucket 8) and batch 10 (bucket 16) faster than 4
    assert hip.decode_attn_plan(8, 8, 12288) == (6, True)
    assert hip.decode_attn_plan(16, 8, 12288) == (6, True)
    # the final reduce (B=1, ~13k, <= 32k class) keeps 32 separate splits (best of 16-64 / fused in situ)
    assert hip.decode_attn_plan(1, 8, 32768) == (32, False)
    # a TP shard's single kv head beyond 6k (config 5's 32k at TP=8): one workgroup per 2 pages, up to 128
    # splits (70B fp8 shard step at 32k: 128 splits 4.80 ms vs 64 5.07, 250 5.10, 32 5.66; r5_attn_plans*.jsonl)
    assert hip.decode_attn_plan(1, 1, 32768) == (128, False)
    assert hip.decode_attn_plan(1, 1, 12288) == (96, False)
    assert hip.decode_attn_plan(16, 1, 32768) == (48, False)
    assert all(hip.decode_attn_plan(b, h, c)[0] <= hip.MAX_SPLITS for b in (1, 2, 16, 64) for h in (1, 2, 8)
               for c in (4096, 12288, 32768, 131072))
    # TP shards keep their measured cap of 4 in the longer classes
    assert hip.decode_attn_plan(20, 1, 12288)[0] <= 4


def test_skinny_waves_rule():
    # 8-wave workgroups where the grid is about one workgroup per CU or less (TP-shard N / 16 tiles)
    assert hip.skinny_waves(3584, 1, 1) == 8      # 8B TP=8 gate_up: 224 workgroups
    assert hip.skinny_waves(4096, 1, 1) == 8      # o / down producers: 256
    assert hip.skinny_waves(7168, 1, 1) == 8      # 70B TP=8 gate_up: 448
    assert hip.skinny_waves(57344, 1, 1) == 4     # 70B TP=1 gate_up: 3584
    assert hip.skinny_waves(4096, 1, 4) == 4      # split-K slabs: 1024
    assert hip.skinny_waves(4096, 1, 1, M=10) == 4  # more than one row: 4 waves (measured 0.3-1 % faster)


def test_fp8_tp_push_producer_rule(monkeypatch):
    # 70B fp8 TP=8 shard: o (K 1024) on the fp8 register-streaming producer at every decode row count up to
    # 16, down (K 3584) only at one row (in situ, profiles/r5_fp8_skinny_push_ab.jsonl); TP=1 keeps the stream
    # producer
    import torch
    from llm_map_reduce_summarizer_amd import ops
    from llm_map_reduce_summarizer_amd.ops.reference import Fp8Weight
    monkeypatch.setattr(hip, "skinny_fp8_resid_capacity", lambda: 1024)

    def w(N, K):
        return Fp8Weight(torch.empty(N, K, dtype=torch.float8_e4m3fn, device="meta"),
                         torch.empty(N, dtype=torch.float32, device="meta"))

    def a(M, K):
        return torch.empty(M, K, dtype=torch.bfloat16, device="meta")

    assert ops._resid_plan(hip, a(1, 1024), w(8192, 1024), "o", tp=True) == ("skinny",)
    assert ops._resid_plan(hip, a(10, 1024), w(8192, 1024), "o", tp=True) == ("skinny",)
    assert ops._resid_plan(hip, a(1, 3584), w(8192, 3584), "down", tp=True) == ("skinny",)
    assert ops._resid_plan(hip, a(10, 3584), w(8192, 3584), "down", tp=True)[0] == "stream"
    assert ops._resid_plan(hip, a(1, 8192), w(8192, 8192), "o", tp=False)[0] == "stream"
    assert ops._resid_plan(hip, a(1, 1024), w(8192, 1024), "o", tp=True, force="stream")[0] == "stream"


def test_narrow_gate_up_split_rules():
    # fp8: a gate_up too narrow for one stream tile per CU takes the split-K SwiGLU (70B TP=8 shard, every decode
    # row count: profiles/r6_fp8_swiglu_split_insitu.jsonl); TP=1 / TP=4 at <= 8 rows stay on the register-
    # streaming kernel (N x K >= 64 M), and wider gate_ups keep one tile per column
    assert hip.stream_config_fp8(7168, 8192, swiglu=True, M=1) == (7, 4)
    assert hip.stream_config_fp8(7168, 8192, swiglu=True, M=39) == (7, 4)
    assert hip.stream_config_fp8(14336, 8192, swiglu=True, M=1) is None
    assert hip.stream_config_fp8(57344, 8192, swiglu=True, M=1) is None
    assert hip.stream_config_fp8(57344, 8192, swiglu=True, M=16) == (7, 1)
    # bf16: the TP=4 shard's 7168-row gate_up splits at one row too (one-round grid), the TP=8 shard's 3584 rows
    # stay on the register-streaming kernel up to 16 rows, the TP=2 shard's 14336 rows on one tile per column
    # (profiles/r6_bf16_swiglu_split_insitu.jsonl)
    assert hip.plan("gate_up", 1, 7168, 4096) == ("stream_split", 7, 4)
    assert hip.plan("gate_up", 10, 7168, 4096) == ("stream_split", 7, 4)
    assert hip.plan("gate_up", 1, 3584, 4096)[0] == "skinny"
    assert hip.plan("gate_up", 1, 14336, 4096) == ("stream", 4, 1)
