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
    # a TP shard's single kv head beyond 6k (config 5's 32k at TP=8): one workgroup per 2 pages, up to the
    # merge's 256 splits (64 splits measured 5.11 vs 5.66 ms per 70B fp8 shard step at 32, r5_attn_plans.jsonl)
    assert hip.decode_attn_plan(1, 1, 32768) == (256, False)
    assert hip.decode_attn_plan(16, 1, 32768) == (48, False)
    assert all(hip.decode_attn_plan(b, h, c)[0] <= hip.MAX_SPLITS for b in (1, 2, 16, 64) for h in (1, 2, 8)
               for c in (4096, 12288, 32768, 131072))
    # TP shards keep their measured cap of 4 in the longer classes
    assert hip.decode_attn_plan(20, 1, 12288)[0] <= 4


def test_consumer_merge_only_for_one_row_of_a_tp_shard():
    # the o projection merges the attention splits for one decode row of a TP shard when the partials every
    # o workgroup re-reads stay small (8B TP=8 at 4k: 4 heads x 63 splits = 126 KiB)
    assert hip.consumer_merge_ok(1, 4, 63, False)
    assert not hip.consumer_merge_ok(1, 4, 63, True)     # the fused (in-launch) merge has no partials left
    assert not hip.consumer_merge_ok(2, 4, 63, False)    # two rows
    assert not hip.consumer_merge_ok(1, 32, 32, False)   # TP=1: 512 KiB per workgroup
    assert not hip.consumer_merge_ok(1, 8, 256, False)   # 70B TP=8 at 32k: 1 MiB
    assert not hip.consumer_merge_ok(1, 32, 2, False)    # more heads than the kernel's LDS row holds
    old = hip.CONSUMER_MERGE_MAX_BYTES
    try:
        hip.CONSUMER_MERGE_MAX_BYTES = 0  # off (tools/exp_plans_insitu.py "cmerge:0")
        assert not hip.consumer_merge_ok(1, 4, 63, False)
    finally:
        hip.CONSUMER_MERGE_MAX_BYTES = old


def test_skinny_waves_rule():
    # 8-wave workgroups where the grid is about one workgroup per CU or less (TP-shard N / 16 tiles)
    assert hip.skinny_waves(3584, 1, 1) == 8      # 8B TP=8 gate_up: 224 workgroups
    assert hip.skinny_waves(4096, 1, 1) == 8      # o / down producers: 256
    assert hip.skinny_waves(7168, 1, 1) == 8      # 70B TP=8 gate_up: 448
    assert hip.skinny_waves(57344, 1, 1) == 4     # 70B TP=1 gate_up: 3584
    assert hip.skinny_waves(4096, 1, 4) == 4      # split-K slabs: 1024
